# span-kernel cost breakdown: the diagnostic variants side by side (config 3)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 tools/kvariants.py run --names base,span_noprio --rounds 10 --workloads csr:1048576:64:1400
