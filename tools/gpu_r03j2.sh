set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03j2}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o t -- python3 bench.py --workload append --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > gpurun_out/${TAG}_prof.log 2>&1 || { tail -5 gpurun_out/${TAG}_prof.log; exit 1; }
echo prof-done
