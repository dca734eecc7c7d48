# span kernel: in-kernel wave-batch boundary heads; GPU suite, csr / filter bench, kernel trace
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03d}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
for w in csr filter filter_dispatch; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-host-path > gpurun_out/${TAG}_$w.json 2> gpurun_out/${TAG}_$w.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$w.json'));print('$w', d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'])"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o t -- python3 bench.py --workload csr --steps 20 --warmup 5 --no-cpu-baseline --no-host-path > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -8
