# PMC passes for the CSR workload's kernels (run on the GPU box from the repo
# root); one counter group per rocprofv3 run, CSV output, summarised by
# tools/pmc_summary.py.
set -o pipefail
OUT=${1:-gpurun_out/pmc_csr}
WL=${2:-csr}
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --workload $WL --steps 5 --warmup 1 --no-cpu-baseline --no-host-path"
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM" \
           "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_ANY" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$i" -o p -- $B > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT"
