set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/kvariants.py run --names base,xgrid_w8 --rounds 10 --workloads xor:1048576:732,xor:1048576:1400,xorcsr:1048576,xorcsr:2097152 --out gpurun_out/r03k_kv.json > gpurun_out/r03k_kv.log 2>&1 || exit 1
cat gpurun_out/r03k_kv.log
