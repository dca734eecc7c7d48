set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "xor" --timeout 120 --timeout-method thread > gpurun_out/r03i_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r03i_pytest.log; exit 1; }
tail -1 gpurun_out/r03i_pytest.log
timeout -k 10 300 python -u tools/kvariants.py run --names base,xcsr_flat,xstr_u4a1,xstr_u2a1,xstr_u2a2w8,xstr_u4a2 --rounds 10 --workloads xorcsr:1048576 --out gpurun_out/r03i_kv.json > gpurun_out/r03i_kv.log 2>&1 || exit 1
cat gpurun_out/r03i_kv.log
timeout -k 10 120 python -u tools/probe_forms.py > gpurun_out/r03i_probe.txt 2>&1 || exit 1
cat gpurun_out/r03i_probe.txt
