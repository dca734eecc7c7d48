# span kernel anatomy after the in-kernel setup / heads: timeline, follow-up grid sizes
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/span_timeline.py span_timeline > gpurun_out/r03f_timeline.txt 2>&1 || exit 1
cat gpurun_out/r03f_timeline.txt
timeout -k 10 300 python -u tools/kvariants.py run --names base,fix64,fix8,fix1,span_noev --rounds 10 --workloads csr:1048576:64:1400 --out gpurun_out/r03f_kv.json > gpurun_out/r03f_kv.log 2>&1 || exit 1
cat gpurun_out/r03f_kv.log
