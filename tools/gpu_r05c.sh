set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_append.py tests/test_gpu_parity.py -k "append" > gpurun_out/r05c_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r05c_pytest.log; exit 1; }
tail -2 gpurun_out/r05c_pytest.log
timeout -k 10 600 python -u tools/kvariants.py run --names base,app_team,app_fu2,app_fu4,app_fb4,app_fb16,app_fw4,app_fw16 --workloads append:1048576:64:1400 --rounds 10 --out gpurun_out/r05c_kvariants.json > gpurun_out/r05c_kvariants.log 2>&1 || { echo KV_FAILED; tail -30 gpurun_out/r05c_kvariants.log; exit 1; }
cat gpurun_out/r05c_kvariants.log | grep -v amdgpu.ids
timeout -k 10 300 python -u bench.py --workload append --no-cpu-baseline > gpurun_out/r05c_append.json 2> gpurun_out/r05c_append.err || { echo BENCH_FAILED; tail gpurun_out/r05c_append.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r05c_append.json'));print(d['ms_per_step'], d['roofline']['frac'], d.get('host_append'))"
