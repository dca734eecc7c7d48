# GPU tests + the socket-path example (run via gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 120 ./examples/socket_path --count 400000 --burst 1024 > gpurun_out/socket_path.json 2> gpurun_out/socket_path.err; echo rc=$?; cat gpurun_out/socket_path.json gpurun_out/socket_path.err
timeout -k 10 120 ./examples/socket_path --count 400000 --burst 4096 > gpurun_out/socket_path4k.json 2>> gpurun_out/socket_path.err; cat gpurun_out/socket_path4k.json
