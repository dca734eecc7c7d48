# End-of-round GPU pass (run via gpurun from the repo root): parity tests,
# every bench workload, smoke, and the round's profiles.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r01d}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/final_fixed.json 2> gpurun_out/final_fixed.err || exit 1
for w in csr filter xor xor_csr dispatch append filter_dispatch filter_then_dispatch; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-host-path > gpurun_out/final_$w.json 2> gpurun_out/final_$w.err || exit 1
done
timeout -k 10 300 python -u bench.py --workload csr > gpurun_out/final_csr_host.json 2> gpurun_out/final_csr_host.err || exit 1
timeout -k 10 300 env LNL_BENCH_BACKEND=gloo LNL_BENCH_ONE_GPU=1 python -u bench.py --gpus 2 --no-cpu-baseline > gpurun_out/final_fixed_2ranks.json 2> gpurun_out/final_fixed_2ranks.err || exit 1
# summaries on the box (the rocprof databases are too big to copy back)
for w in fixed csr filter dispatch xor xor_csr append filter_dispatch; do
  timeout -k 10 900 bash tools/profile_round.sh $TAG $w || exit 1
  PROFILES_DIR=gpurun_out/profiles_$TAG python3 tools/write_profiles.py $TAG $w > /dev/null || exit 1
  rm -rf gpurun_out/prof_${TAG}_$w
done
echo final-done
