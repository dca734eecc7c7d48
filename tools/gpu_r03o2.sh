set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03o2}
timeout -k 10 120 python -u tools/pcie_probe.py > gpurun_out/${TAG}_pcie.txt 2>&1 || { cat gpurun_out/${TAG}_pcie.txt; exit 1; }
cat gpurun_out/${TAG}_pcie.txt
