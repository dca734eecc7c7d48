# span kernel without the pre-pass: GPU suite, csr / filter / filter_dispatch / append benches
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03c_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r03c_pytest.log; exit 1; }
tail -2 gpurun_out/r03c_pytest.log
for w in csr filter filter_dispatch; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-host-path > gpurun_out/r03c_$w.json 2> gpurun_out/r03c_$w.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r03c_$w.json'));print('$w', d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'])"
done
timeout -k 10 300 python -u bench.py --workload append --no-cpu-baseline > gpurun_out/r03c_append.json 2> gpurun_out/r03c_append.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r03c_append.json'));print('append', d['ms_per_step'], d['roofline']['frac'], d['host_append'])"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r03c_prof -o t -- python3 bench.py --workload csr --steps 20 --warmup 5 --no-cpu-baseline --no-host-path > gpurun_out/r03c_prof.log 2>&1 || exit 1
find gpurun_out/r03c_prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
