set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/span_timeline.py span_timeline > gpurun_out/r03g_timeline.txt 2>&1 || exit 1
cat gpurun_out/r03g_timeline.txt
timeout -k 10 120 python -u tools/timing_probe.py csr > gpurun_out/r03g_timing_csr.json 2>&1 || exit 1
cat gpurun_out/r03g_timing_csr.json
timeout -k 10 120 python -u tools/timing_probe.py > gpurun_out/r03g_timing_fixed.json 2>&1 || exit 1
cat gpurun_out/r03g_timing_fixed.json
