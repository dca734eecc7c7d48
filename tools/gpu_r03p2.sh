set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03p2}
timeout -k 10 400 python -u tools/kvariants.py run --names base,span_noprio,walk_norow,walk_none --rounds 8 --workloads fd:1048576,filter:1048576:1297:1297 --out gpurun_out/${TAG}_kv.json > gpurun_out/${TAG}_kv.log 2>&1 || { tail -20 gpurun_out/${TAG}_kv.log; exit 1; }
cat gpurun_out/${TAG}_kv.log
timeout -k 10 300 python -u tools/kvariants.py run --names base,app_nohead,app_nochunk,app_nostore --rounds 8 --workloads append:1048576:64:1400 --out gpurun_out/${TAG}_kva.json > gpurun_out/${TAG}_kva.log 2>&1 || { tail -20 gpurun_out/${TAG}_kva.log; exit 1; }
cat gpurun_out/${TAG}_kva.log
