# Flat CSR XOR kernel: the XOR parity tests and the two XOR bench workloads.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_xor_layer.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "xor" > gpurun_out/r02d_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r02d_pytest.log; exit 1; }
tail -1 gpurun_out/r02d_pytest.log
for w in xor_csr xor; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-host-path > gpurun_out/r02d_$w.json 2> gpurun_out/r02d_$w.err || { tail -20 gpurun_out/r02d_$w.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r02d_$w.json').read().strip().splitlines()[-1]); print('$w', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
