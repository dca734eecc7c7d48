set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --host-path > gpurun_out/bench_fixed_host.json 2> gpurun_out/bench_fixed_host.err && cat gpurun_out/bench_fixed_host.json || exit 1
timeout -k 10 300 python -u bench.py --workload csr --host-path --no-cpu-baseline > gpurun_out/bench_csr_host.json 2> gpurun_out/bench_csr_host.err && cat gpurun_out/bench_csr_host.json || exit 1
