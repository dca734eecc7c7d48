set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03h}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
for w in fixed csr filter filter_dispatch; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-host-path > gpurun_out/${TAG}_$w.json 2> gpurun_out/${TAG}_$w.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$w.json'));print('$w', d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['settle_steps'])"
done
timeout -k 10 120 python -u tools/span_timeline.py span_timeline > gpurun_out/${TAG}_timeline.txt 2>&1 || exit 1
cat gpurun_out/${TAG}_timeline.txt
timeout -k 10 300 python -u bench.py --workload xor_csr --no-cpu-baseline --no-host-path > gpurun_out/${TAG}_xor_csr.json 2> gpurun_out/${TAG}_xor_csr.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_xor_csr.json'));print('xor_csr', d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'])"
timeout -k 10 120 python -u tools/probe_forms.py > gpurun_out/${TAG}_probe.txt 2>&1 || exit 1
cat gpurun_out/${TAG}_probe.txt
