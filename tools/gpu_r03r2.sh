set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03r2}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config4.py -m gpu -x -q -k "fixed or config2 or config4 or smoke or run" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -u tools/kvariants.py run --names base,run_late --rounds 12 --workloads 1048576:1400:1400:0 --out gpurun_out/${TAG}_kv.json > gpurun_out/${TAG}_kv.log 2>&1 || { tail -20 gpurun_out/${TAG}_kv.log; exit 1; }
cat gpurun_out/${TAG}_kv.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-path > gpurun_out/${TAG}_fixed.json 2> gpurun_out/${TAG}_fixed.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_fixed.json'));r=d['roofline'];print('fixed', d['ms_per_step'], d['value'], r['frac'], r['kernel_ms'])"
