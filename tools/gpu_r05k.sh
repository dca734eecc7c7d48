set -o pipefail
timeout -k 10 200 python tools/kvariants.py run --names base,xg16,xg64,xg192 --rounds 12 --workloads xorcsr:1048576 --out gpurun_out/r05k_xor_grid.json > gpurun_out/r05k_xor_grid.log 2>&1 &&
LNL_XOR_FLAT_WG=8 timeout -k 10 100 python tools/kvariants.py run --names base --rounds 12 --workloads xor:1048576:1400 --out gpurun_out/r05k_xorflat8.json >> gpurun_out/r05k_xor_grid.log 2>&1 &&
LNL_XOR_FLAT_WG=32 timeout -k 10 100 python tools/kvariants.py run --names base --rounds 12 --workloads xor:1048576:1400 --out gpurun_out/r05k_xorflat32.json >> gpurun_out/r05k_xor_grid.log 2>&1 &&
LNL_XOR_FLAT_WG=1000000 timeout -k 10 100 python tools/kvariants.py run --names base --rounds 12 --workloads xor:1048576:1400 --out gpurun_out/r05k_xorflatnp.json >> gpurun_out/r05k_xor_grid.log 2>&1
rc=$?; cat gpurun_out/r05k_xor_grid.log; exit $rc
