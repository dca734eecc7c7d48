# Round GPU pass in two gpurun calls (each fits the 1200 s call limit):
#   bash tools/gpu_round.sh <tag> tests      parity suite, smoke, every bench workload
#   bash tools/gpu_round.sh <tag> profiles [workloads...]   rocprofv3 summaries
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:?tag}
MODE=${2:-tests}
if [ "$MODE" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -1 gpurun_out/${TAG}_pytest.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && tail -1 gpurun_out/${TAG}_smoke.log || exit 1
  timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_fixed.json 2> gpurun_out/${TAG}_fixed.err || exit 1
  for w in csr filter xor xor_csr dispatch filter_dispatch filter_then_dispatch; do
    timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-host-path > gpurun_out/${TAG}_$w.json 2> gpurun_out/${TAG}_$w.err || exit 1
  done
  # the send side from pinned host memory too (host_append)
  timeout -k 10 300 python -u bench.py --workload append --no-cpu-baseline > gpurun_out/${TAG}_append.json 2> gpurun_out/${TAG}_append.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_append.json'));print('host_append', d.get('host_append', {}).get('value'), 'GB/s')" || exit 1
  for w in fixed csr filter xor xor_csr dispatch append filter_dispatch filter_then_dispatch; do
    python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$w.json'));r=d['roofline'];print('$w', d['ms_per_step'], r['frac'], r['kernel_ms'])" || exit 1
  done
  echo tests-done
else
  shift 2
  WLS=${*:-fixed csr xor_csr append filter_dispatch}
  for w in $WLS; do
    timeout -k 10 400 bash tools/profile_round.sh $TAG $w || exit 1
    PROFILES_DIR=gpurun_out/profiles_$TAG python3 tools/write_profiles.py $TAG $w > /dev/null || exit 1
    rm -rf gpurun_out/prof_${TAG}_$w
  done
  echo profiles-done
fi
