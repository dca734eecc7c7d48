# quick GPU check (run via gpurun from the repo root): gpu tests, CSR bench, kernel trace, variants
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --workload csr --no-cpu-baseline > gpurun_out/bench_csr.json 2> gpurun_out/bench_csr.err && cat gpurun_out/bench_csr.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pq -o t -- python3 bench.py --workload csr --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/pq.log 2>&1 || exit 1
python3 litenetlibpp_amd/tools/prof_summary.py gpurun_out/pq/t_results.db > gpurun_out/pq.md && sed -n 1,14p gpurun_out/pq.md
if [ -n "$KV" ]; then timeout -k 10 300 python -u tools/kvariants.py run --names $KV --rounds 6 --workloads ${KVW:-csr:1048576:64:1400} > gpurun_out/kv.log 2>&1 && cat gpurun_out/kv.log; fi
