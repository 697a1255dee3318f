# round 3: the profile passes again, bench workload only (--no-side)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -rf gpurun_out/prof_r3x
bash tools/profile.sh r3x 20 && echo PROFILE_OK
python3 -c "import json; d=json.load(open('gpurun_out/prof_r3x/bench_trace.json')); print('bench under trace', d['value'], d['roofline']['avg_launch_us'])"
