set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "xor" --timeout 120 --timeout-method thread > gpurun_out/r03l_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r03l_pytest.log; exit 1; }
tail -1 gpurun_out/r03l_pytest.log
timeout -k 10 300 python -u tools/kvariants.py run --names base,xgrid_w8,xgrid_w6,xgrid_dflt --rounds 10 --workloads xorcsr:1048576,xor:1048576:732 --out gpurun_out/r03l_kv.json > gpurun_out/r03l_kv.log 2>&1 || exit 1
cat gpurun_out/r03l_kv.log
