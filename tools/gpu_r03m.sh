set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "xor" --timeout 120 --timeout-method thread > gpurun_out/r03m_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r03m_pytest.log; exit 1; }
tail -1 gpurun_out/r03m_pytest.log
timeout -k 10 300 python -u tools/kvariants.py run --names base,xgrid_w5,xgrid_w7,xgrid_u4w3,xgrid_u4w4,xgrid_u4w5,xgrid_u1w8,xgrid_u1w10 --rounds 10 --workloads xorcsr:1048576 --out gpurun_out/r03m_kv.json > gpurun_out/r03m_kv.log 2>&1 || exit 1
cat gpurun_out/r03m_kv.log
