# outbound layer on the GPU box: append parity tests, the append bench workload
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "append" > gpurun_out/append_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/append_pytest.log; exit 1; }
tail -1 gpurun_out/append_pytest.log
timeout -k 10 300 python -u bench.py --workload append --no-cpu-baseline --no-host-path > gpurun_out/append_bench.json 2> gpurun_out/append_bench.err || { tail -20 gpurun_out/append_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/append_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['parity_on_sample'])"
