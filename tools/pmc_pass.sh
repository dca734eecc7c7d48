#!/bin/bash
# PMC passes for the bench kernel (run on the GPU box from the repo root).
# Counters go in separate passes (TCC FETCH_SIZE and WRITE_SIZE cannot share
# one); only --kernel-trace/--stats beside --pmc (never sys/runtime traces).
set -e
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc FETCH_SIZE -d "$OUT/fetch" -o f -- $B > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc WRITE_SIZE -d "$OUT/write" -o w -- $B > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES -d "$OUT/clk" -o c -- $B > "$OUT/clk.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d "$OUT/sq" -o s -- $B > "$OUT/sq.log" 2>&1
