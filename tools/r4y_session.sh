set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4y; mkdir -p $O
PYTEST_FILES="tests/test_replay.py tests/test_golden.py" PYTEST_TIMEOUT=600 PYTEST_FILES="tests/test_replay.py tests/test_golden.py" bash tools/gpu_session.sh r4y tests || exit 1
cd $R && AB=PZ_VOTE_GROUPS AB_VALUES=0,1 REPS=3 timeout -k 10 300 python3 tools/replay_profile.py 65536 10000 > $O/replay_ab.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay_ab.txt; exit 4; }
grep -E "^median" $O/replay_ab.txt; grep phases $O/replay_ab.txt | tail -1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tl -o run --output-format csv -- python3 $R/tools/replay_timeline.py $O/timeline.json > $O/tl.log 2>&1 || { echo TL_FAIL; tail -5 $O/tl.log; exit 5; }
echo DONE
