# One GPU call (run via gpurun from the repo root): gpu tests, both benches,
# CSR profile, kernel-variant timings.  Every step has its own time limit and
# the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01b}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_fixed.json 2> gpurun_out/bench_fixed.err && cat gpurun_out/bench_fixed.json || exit 1
timeout -k 10 300 python -u bench.py --workload csr > gpurun_out/bench_csr.json 2> gpurun_out/bench_csr.err && cat gpurun_out/bench_csr.json || exit 1
timeout -k 10 900 bash tools/profile_round.sh $TAG csr || exit 1
timeout -k 10 300 python -u tools/kvariants.py run --names base,seg,seg_nofold,nocomp,nobucket --rounds 8 --workloads csr:1048576:64:1400 > gpurun_out/kv.log 2>&1 && cat gpurun_out/kv.log
