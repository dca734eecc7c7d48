set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
d=gpurun_out/r05d_fetchcal
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $d -o f -- python3 tools/fetch_calibration.py > $d.log 2>&1 || { echo CAL_FAILED; tail $d.log; exit 1; }
grep -h "sectors\|stream" $d.log | tail -3
f=$(find $d -name "*counter_collection.csv" | head -1); head -1 $f; grep -h "sector_read\|stream_read" $f | cut -c1-300 | head -20
timeout -k 10 400 bash tools/profile_round.sh r05d dispatch > gpurun_out/r05d_prof.log 2>&1 || { echo PROF_FAILED; tail gpurun_out/r05d_prof.log; exit 1; }
PROFILES_DIR=gpurun_out/profiles_r05d python3 tools/write_profiles.py r05d dispatch | tail -2
rm -rf gpurun_out/prof_r05d_dispatch/trace/*.db
echo done
