# SQ counters of the bucketed and uniform CSR paths (run via gpurun)
set -o pipefail
mkdir -p gpurun_out/pmc2; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc2/avail.txt 2>&1 || true
grep -o "SQ_[A-Z_]*" gpurun_out/pmc2/avail.txt | sort -u > gpurun_out/pmc2/sq_names.txt || true
wc -l gpurun_out/pmc2/sq_names.txt
for path in bucketed uniform; do
  LNL_CSR_PATH=$path timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM -d gpurun_out/pmc2/$path -o p -- python3 bench.py --workload csr --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/pmc2/$path.log 2>&1 || { echo FAIL $path; tail -5 gpurun_out/pmc2/$path.log; exit 1; }
  python3 litenetlibpp_amd/tools/prof_summary.py gpurun_out/pmc2/$path/p_results.db > gpurun_out/pmc2/$path.md
  grep -E "crc32c_batch|crc32c_csr" gpurun_out/pmc2/$path.md | grep SQ_
done
