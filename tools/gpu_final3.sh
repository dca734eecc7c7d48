# final-tree check: the GPU parity suite and smoke, as the round-end driver runs them
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03c}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && tail -1 gpurun_out/${TAG}_smoke.log || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_fixed.json 2> gpurun_out/${TAG}_fixed.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_fixed.json'));r=d['roofline'];print('fixed', d['ms_per_step'], d['value'], r['frac'], r['kernel_ms'])"
