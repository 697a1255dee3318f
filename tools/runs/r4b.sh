# round 4: FETCH/WRITE calibration incl. K2's and K4's access shapes, SQ counters
# of the shipped 3 x 24 bench build, kernel trace + traffic of the bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
C=$R/gpurun_out/calib_r4b
mkdir -p $C
timeout -k 10 60 $R/tools/ubench/calib > $C/calib.json || exit 1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $C/fetch -o run --output-format csv -- $R/tools/ubench/calib > $C/fetch.txt 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $C/write -o run --output-format csv -- $R/tools/ubench/calib > $C/write.txt 2>&1 || exit 1
echo calib done
SQ_BENCH=1 bash $R/tools/sq_counters.sh r4b || { echo SQ_FAILED; exit 1; }
echo sq done
bash $R/tools/profile.sh r4b 20 && echo PROFILE_OK
