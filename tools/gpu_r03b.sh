# span kernel anatomy: per-wave timeline + diagnostic variants + csr/append bench with the host legs
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/span_timeline.py span_timeline > gpurun_out/r03b_timeline.txt 2>&1 || exit 1
cat gpurun_out/r03b_timeline.txt
timeout -k 10 300 python -u tools/kvariants.py run --names base,span_noev,span_noflush --rounds 10 --workloads csr:1048576:64:1400 --out gpurun_out/r03b_kv.json > gpurun_out/r03b_kv.log 2>&1 || exit 1
cat gpurun_out/r03b_kv.log
timeout -k 10 300 python -u bench.py --workload append --no-cpu-baseline > gpurun_out/r03b_append.json 2> gpurun_out/r03b_append.err || exit 1
cat gpurun_out/r03b_append.json
