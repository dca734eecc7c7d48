set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/fixed_as_csr.py 12 20 > gpurun_out/r05b_fixed_as_csr.log 2>&1 || { echo FAIL1; tail gpurun_out/r05b_fixed_as_csr.log; exit 1; }
cat gpurun_out/r05b_fixed_as_csr.log
for m in "whole 8" "sliced 8" "sliced 4" "sliced 16"; do
  set -- $m
  d=gpurun_out/r05b_mall_$1_$2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o t -- python3 tools/mall_probe.py $1 $2 6 > $d.log 2>&1 || { echo FAIL $m; tail $d.log; exit 1; }
  grep -h "per burst\|sliced ==" $d.log
  find $d -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c "cut -d, -f1-4 {} | head -8"
done
echo done
