set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
d=gpurun_out/r05e_fetchcal
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $d -o f -- python3 tools/fetch_calibration.py > $d.log 2>&1 || { echo CAL_FAILED; tail $d.log; exit 1; }
python3 tools/fetch_calibration.py summarize $d/f_counter_collection.csv gpurun_out/r05e_fetch_calibration.json || exit 1
cp gpurun_out/r05e_fetch_calibration.json profiles/fetch_calibration.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05e_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r05e_pytest.log; exit 1; }
tail -1 gpurun_out/r05e_pytest.log
for w in dispatch filter_dispatch; do
  timeout -k 10 400 bash tools/profile_round.sh r05e $w > gpurun_out/r05e_prof_$w.log 2>&1 || { echo PROF_FAILED $w; tail gpurun_out/r05e_prof_$w.log; exit 1; }
  PROFILES_DIR=gpurun_out/profiles_r05e python3 tools/write_profiles.py r05e $w | tail -1 | cut -c1-600
  rm -rf gpurun_out/prof_r05e_$w
done
echo done
