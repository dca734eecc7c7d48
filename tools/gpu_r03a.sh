# Round-3 first pass: the GPU suite (config-4 test included) and the default bench line.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03a_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r03a_pytest.log; exit 1; }
tail -3 gpurun_out/r03a_pytest.log
timeout -k 10 300 python -u bench.py > gpurun_out/r03a_fixed.json 2> gpurun_out/r03a_fixed.err || exit 1
cat gpurun_out/r03a_fixed.json
timeout -k 10 300 python -u bench.py --workload csr --no-cpu-baseline --no-host-path > gpurun_out/r03a_csr.json 2> gpurun_out/r03a_csr.err || exit 1
cat gpurun_out/r03a_csr.json
