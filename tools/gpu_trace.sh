# Kernel-trace stats of bench workloads (run via gpurun from the repo root):
#   tools/gpu_trace.sh <tag> <workload>...
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
for w in "$@"; do
  OUT=gpurun_out/tr_${TAG}_$w
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o t -- python3 bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-host-path > $OUT/log 2>&1 || { tail -20 $OUT/log; exit 1; }
  f=$(find $OUT -name '*kernel_stats.csv' | head -1)
  cp "$f" gpurun_out/tr_${TAG}_${w}_stats.csv
  echo "== $w"; python3 -c "
import csv,sys
for r in list(csv.DictReader(open('$f')))[:12]:
    print('%-70s %6s %10.2f' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3))"
  find $OUT -name '*.csv' ! -name '*stats*' -delete
done
