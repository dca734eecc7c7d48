# inbound filter / verify on the GPU box: parity tests, filter and csr bench lines
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "verify or filter or dispatch or socket" > gpurun_out/filter_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/filter_pytest.log; exit 1; }
tail -1 gpurun_out/filter_pytest.log
for wl in filter csr filter csr; do
timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --no-host-path > gpurun_out/b_$wl.json 2> gpurun_out/b_$wl.err || { tail -20 gpurun_out/b_$wl.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_$wl.json')); print('$wl', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
