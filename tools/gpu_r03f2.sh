set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03f2}
timeout -k 10 120 python -u tools/probe_forms.py > gpurun_out/${TAG}_probe.txt 2>&1 || { cat gpurun_out/${TAG}_probe.txt; exit 1; }
cat gpurun_out/${TAG}_probe.txt
