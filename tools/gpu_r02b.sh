# Round-2 fused filter + dispatch: its parity tests, then the bench workloads
# around it (run via gpurun from the repo root).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "dispatch or inbound_filter or csr or verify or config3" > gpurun_out/r02b_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r02b_pytest.log; exit 1; }
tail -3 gpurun_out/r02b_pytest.log
for w in filter_dispatch filter_then_dispatch csr filter; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-host-path > gpurun_out/r02b_$w.json 2> gpurun_out/r02b_$w.err || { tail -20 gpurun_out/r02b_$w.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r02b_$w.json')); print('$w', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d.get('parity_whole_batch', d.get('parity_on_sample')))"
done
