set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02a_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/r02a_pytest.log; exit 1; }
tail -1 gpurun_out/r02a_pytest.log
timeout -k 10 300 python -u bench.py > gpurun_out/r02a_fixed.json 2> gpurun_out/r02a_fixed.err || exit 1
cat gpurun_out/r02a_fixed.json
timeout -k 10 300 python -u bench.py --workload csr > gpurun_out/r02a_csr.json 2> gpurun_out/r02a_csr.err || exit 1
cat gpurun_out/r02a_csr.json
timeout -k 10 300 env LNL_BENCH_BACKEND=gloo LNL_BENCH_ONE_GPU=1 python -u bench.py --gpus 2 --no-cpu-baseline > gpurun_out/r02a_2ranks.json 2> gpurun_out/r02a_2ranks.err || exit 1
cat gpurun_out/r02a_2ranks.json
