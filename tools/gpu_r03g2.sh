set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03g2}
timeout -k 10 120 python -u tools/span_timeline.py span_timeline > gpurun_out/${TAG}_timeline.txt 2>&1 || { cat gpurun_out/${TAG}_timeline.txt; exit 1; }
cat gpurun_out/${TAG}_timeline.txt
timeout -k 10 300 python -u tools/kvariants.py run --names base,span_noev,span_noflush,span_nofold,fix1,span_noprio --rounds 10 --workloads csr:1048576:64:1400 --out gpurun_out/${TAG}_kv.json > gpurun_out/${TAG}_kv.log 2>&1 || { tail -20 gpurun_out/${TAG}_kv.log; exit 1; }
cat gpurun_out/${TAG}_kv.log
