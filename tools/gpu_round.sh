# GPU passes on the MI355X box (each mode fits one gpurun call, <= 1200 s):
#   bash tools/gpu_round.sh <tag> tests                 parity suite, smoke, every bench workload
#   bash tools/gpu_round.sh <tag> pytest [pytest args]  the parity suite (or a selection: -k expr, files)
#   bash tools/gpu_round.sh <tag> bench [workloads]     bench.py lines (default: every workload)
#   bash tools/gpu_round.sh <tag> variants <names> <workloads> [rounds]
#                                                       tools/kvariants.py run (variants built here first:
#                                                       python tools/kvariants.py build --names ...)
#   bash tools/gpu_round.sh <tag> profiles [workloads]  rocprofv3 summaries (tools/profile_round.sh)
#   bash tools/gpu_round.sh <tag> timeline [variant]    the span kernel's per-wave timeline
#                                                       (variant span_timeline; tools/span_timeline.py)
# Every GPU step runs under its own time limit and the steps stop at the first
# failure.  Outputs go to gpurun_out/<tag>_*.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:?tag}
MODE=${2:-tests}
shift 2 2>/dev/null || shift $#
ALL_WL="fixed csr filter xor xor_csr dispatch append filter_dispatch filter_then_dispatch"

bench_lines() {  # workloads...
  for w in "$@"; do
    case $w in
      fixed) extra="" ;;                       # the headline line: CPU baseline + config 5 (2 and 4 streams)
      append) extra="--no-cpu-baseline" ;;     # host_append: the send side from pinned memory
      *) extra="--no-cpu-baseline --no-host-path" ;;
    esac
    timeout -k 10 300 python -u bench.py --workload $w $extra > gpurun_out/${TAG}_$w.json 2> gpurun_out/${TAG}_$w.err || { echo "BENCH_FAILED $w"; tail -20 gpurun_out/${TAG}_$w.err; return 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$w.json'));r=d['roofline'];print('$w', d['ms_per_step'], r['frac'], r['kernel_ms'], 'host', d.get('host_path', d.get('host_append', {})).get('value'), d.get('host_path', d.get('host_append', {})).get('value_4_streams'))" || return 1
  done
}

case $MODE in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
    tail -1 gpurun_out/${TAG}_pytest.log
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && tail -1 gpurun_out/${TAG}_smoke.log || exit 1
    bench_lines $ALL_WL || exit 1
    echo tests-done ;;
  pytest)
    timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "${@:-tests}" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
    tail -3 gpurun_out/${TAG}_pytest.log ;;
  bench)
    bench_lines ${*:-$ALL_WL} || exit 1
    echo bench-done ;;
  variants)
    NAMES=${1:?names}; WLS=${2:?workloads}; ROUNDS=${3:-10}
    timeout -k 10 900 python -u tools/kvariants.py run --names $NAMES --workloads $WLS --rounds $ROUNDS --out gpurun_out/${TAG}_kvariants.json > gpurun_out/${TAG}_kvariants.log 2>&1 || { echo VARIANTS_FAILED; tail -30 gpurun_out/${TAG}_kvariants.log; exit 1; }
    cat gpurun_out/${TAG}_kvariants.log ;;
  profiles)
    for w in ${*:-fixed csr xor_csr append filter_dispatch}; do
      timeout -k 10 400 bash tools/profile_round.sh $TAG $w || exit 1
      PROFILES_DIR=gpurun_out/profiles_$TAG python3 tools/write_profiles.py $TAG $w > /dev/null || exit 1
      rm -rf gpurun_out/prof_${TAG}_$w
    done
    echo profiles-done ;;
  timeline)
    timeout -k 10 300 python -u tools/span_timeline.py ${1:-span_timeline} > gpurun_out/${TAG}_timeline.log 2>&1 || { echo TIMELINE_FAILED; tail -30 gpurun_out/${TAG}_timeline.log; exit 1; }
    tail -40 gpurun_out/${TAG}_timeline.log ;;
  *) echo "unknown mode $MODE"; exit 2 ;;
esac
