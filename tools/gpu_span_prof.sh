# span-kernel profile on the GPU box: kernel trace of the config-3 bench
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT=gpurun_out/span_prof
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o t -- python3 bench.py --workload csr --steps 20 --warmup 5 --no-cpu-baseline --no-host-path > $OUT/log 2>&1 || { tail -20 $OUT/log; exit 1; }
f=$(find $OUT -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -20
