# full GPU parity suite + filter / csr bench lines
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/full_pytest.log; exit 1; }
tail -1 gpurun_out/full_pytest.log
for wl in filter csr; do
timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --no-host-path > gpurun_out/b_$wl.json 2> gpurun_out/b_$wl.err || { tail -20 gpurun_out/b_$wl.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_$wl.json')); print('$wl', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
