# append chunk-store cache policy: the product (sc0) against the default policy, then the append parity tests + bench
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03s3}
timeout -k 10 300 python -u tools/kvariants.py run --names base,app_scdf --rounds 8 --workloads append:1048576:64:1400 --out gpurun_out/${TAG}_kv.json > gpurun_out/${TAG}_kv.log 2>&1 || { tail -20 gpurun_out/${TAG}_kv.log; exit 1; }
cat gpurun_out/${TAG}_kv.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -u bench.py --workload append --no-cpu-baseline > gpurun_out/${TAG}_append.json 2> gpurun_out/${TAG}_append.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_append.json'));r=d['roofline'];print('append', d['ms_per_step'], r['frac'], r['kernel_ms'], d.get('host_append', {}).get('value'))"
