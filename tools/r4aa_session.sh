set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4aa; mkdir -p $O
PYTEST_FILES="tests/test_replay.py tests/test_golden.py" PYTEST_TIMEOUT=600 bash tools/gpu_session.sh r4aa tests || exit 1
for G in 1 0; do
  echo "== PZ_VOTE_GROUPS=$G" >> $O/trace.txt
  PZ_VOTE_GROUPS=$G timeout -k 10 200 python3 tools/vote_trace.py >> $O/trace.txt 2>&1 || { echo TRACE_FAIL; tail -5 $O/trace.txt; exit 3; }
done
grep -v amdgpu.ids $O/trace.txt
cd $R && AB=PZ_VOTE_GROUPS AB_VALUES=0,1 REPS=3 timeout -k 10 300 python3 tools/replay_profile.py 65536 10000 > $O/replay_ab.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay_ab.txt; exit 4; }
grep -E "^median" $O/replay_ab.txt; grep phases $O/replay_ab.txt | tail -2
echo DONE
