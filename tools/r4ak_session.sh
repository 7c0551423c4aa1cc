set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4ak; mkdir -p $O
PZ_VOTE_GTHREADS=512 PYTEST_FILES="tests/test_replay.py" PYTEST_K="wide_committees or vote_queue or configs4" PYTEST_TIMEOUT=600 bash tools/gpu_session.sh r4ak tests || exit 1
for G in 512 256; do
  echo "== PZ_VOTE_GTHREADS=$G" >> $O/trace.txt
  PZ_VOTE_GTHREADS=$G timeout -k 10 200 python3 tools/vote_trace.py >> $O/trace.txt 2>&1 || { echo TRACE_FAIL; tail -5 $O/trace.txt; exit 3; }
done
grep -v amdgpu.ids $O/trace.txt
cd $R && AB=PZ_VOTE_GTHREADS AB_VALUES=256,512 REPS=5 timeout -k 10 300 python3 tools/replay_profile.py 65536 10000 > $O/replay_ab.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay_ab.txt; exit 4; }
grep -E "^median" $O/replay_ab.txt
echo DONE
