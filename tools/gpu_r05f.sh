set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r05f_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r05f_pytest.log; exit 1; }
tail -1 gpurun_out/r05f_pytest.log
for w in csr filter_dispatch xor_csr append; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-host-path > gpurun_out/r05f_$w.json 2> gpurun_out/r05f_$w.err || { echo BENCH_FAILED $w; tail gpurun_out/r05f_$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05f_$w.json'));print('$w', d['ms_per_step'], d['roofline']['frac'])"
done
