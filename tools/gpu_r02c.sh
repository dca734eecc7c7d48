# Dispatch record layout check: parity subset, the dispatch benches, and the
# fused call's write traffic (one WRITE_SIZE pass).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "dispatch or inbound_filter" > gpurun_out/r02c_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r02c_pytest.log; exit 1; }
tail -1 gpurun_out/r02c_pytest.log
for w in filter_dispatch filter_then_dispatch dispatch; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-host-path > gpurun_out/r02c_$w.json 2> gpurun_out/r02c_$w.err || { tail -20 gpurun_out/r02c_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r02c_$w.json')); print('$w', d['ms_per_step'], d['roofline']['kernel_ms'], d.get('parity_whole_batch'))"
done
timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/r02c_w -o w --output-format csv -- python3 bench.py --workload filter_dispatch --steps 5 --warmup 2 --no-cpu-baseline --no-host-path > gpurun_out/r02c_w.log 2>&1 || { tail -5 gpurun_out/r02c_w.log; exit 1; }
f=$(find gpurun_out/r02c_w -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
tot = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if 'span_kernel' in r['Kernel_Name'] or 'dispatch_' in r['Kernel_Name']:
        tot[r['Kernel_Name'][:60]].append(float(r['Counter_Value']))
for k, v in tot.items():
    print('WRITE_SIZE KiB', k, sum(v) / len(v), len(v))
PY
find gpurun_out/r02c_w -name '*.csv' -size +1M -delete
