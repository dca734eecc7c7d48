# span-kernel bring-up on the GPU box: CSR parity tests, the config-3 bench, PMC
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "csr or config3 or golden or host_streaming or host_multi" > gpurun_out/span_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/span_pytest.log; exit 1; }
tail -1 gpurun_out/span_pytest.log
timeout -k 10 300 python -u bench.py --workload csr --no-cpu-baseline --no-host-path > gpurun_out/span_csr.json 2> gpurun_out/span_csr.err || { tail -20 gpurun_out/span_csr.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/span_csr.json')); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
if [ "$1" = "pmc" ]; then bash tools/pmc_csr.sh gpurun_out/pmc_span csr | grep -E "span_kernel|span_prep|batch_kernel" | grep -E "INSTS|GRBM|FETCH|WRITE|LDS_BANK"; fi
