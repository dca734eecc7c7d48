# append kernel geometry re-swept with the asm chunk stores (workgroups per CU, team size, unroll, blocked runs)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03s4}
timeout -k 10 400 python -u tools/kvariants.py run --names base,app_blk,app_w32 --rounds 8 --workloads append:1048576:64:1400 --out gpurun_out/${TAG}_kv.json > gpurun_out/${TAG}_kv.log 2>&1 || { tail -20 gpurun_out/${TAG}_kv.log; exit 1; }
cat gpurun_out/${TAG}_kv.log
