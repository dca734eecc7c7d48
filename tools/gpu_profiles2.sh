# profiles + benches of the extra workloads (run via gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r01c}
timeout -k 10 200 python -u bench.py --workload filter > gpurun_out/bench_filter.json 2>gpurun_out/bench_filter.err && cat gpurun_out/bench_filter.json || exit 1
timeout -k 10 900 bash tools/profile_round.sh $TAG xor || exit 1
timeout -k 10 900 bash tools/profile_round.sh $TAG filter || exit 1
echo profiles-done
