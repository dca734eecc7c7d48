# CSR kernel study (run via gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/kvariants.py run --names base,bucketed,csr_edge_nt,csr_dflt,nocomp --rounds 8 --workloads csr:1048576:64:1400 > gpurun_out/kv.log 2>&1 && cat gpurun_out/kv.log || exit 1
B="python3 bench.py --workload csr --steps 10 --warmup 2 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pf -o f -- $B > gpurun_out/pf.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_BUSY_CYCLES -d gpurun_out/ps -o s -- $B > gpurun_out/ps.log 2>&1 || exit 1
python3 litenetlibpp_amd/tools/prof_summary.py gpurun_out/pf/f_results.db > gpurun_out/pf.md
python3 litenetlibpp_amd/tools/prof_summary.py gpurun_out/ps/s_results.db > gpurun_out/ps.md
grep -h "csr\|crc32c\|plan" gpurun_out/pf.md gpurun_out/ps.md | grep "FETCH\|INSTS\|WAVES\|BUSY"
