#!/bin/bash
# Round profiles (run on the GPU box from the repo root):
#   tools/profile_round.sh <tag> [workload]
# 1. rocprofv3 --kernel-trace --stats of the bench command (CSV + db)
# 2. PMC passes, one counter group per pass (FETCH_SIZE and WRITE_SIZE cannot
#    share a pass; never combined with sys/runtime traces)
# Output under gpurun_out/prof_<tag>_<workload>/ ; summarised locally into profiles/.
set -e
TAG=${1:-r01}
WL=${2:-fixed}
OUT=gpurun_out/prof_${TAG}_${WL}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --workload $WL --steps 20 --warmup 5 --no-cpu-baseline --no-host-path"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d "$OUT/trace" -o t -- $B > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o f -- $B > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" -o w -- $B > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES -d "$OUT/clk" -o c -- $B > "$OUT/clk.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM -d "$OUT/sq" -o s -- $B > "$OUT/sq.log" 2>&1
echo done
