set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4ai; mkdir -p $O
PYTEST_FILES="tests/test_replay.py" PYTEST_K="wide_committees or vote_queue" PYTEST_TIMEOUT=600 bash tools/gpu_session.sh r4ai tests || exit 1
grep -E "PASSED|FAILED" $O/pytest_gpu.txt | head -20
echo DONE
cd $R && REPS=5 timeout -k 10 300 python3 tools/replay_profile.py 65536 10000 > $O/replay.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay.txt; exit 4; }
PZ_PROBE_LIB=build/old/libprysm_hip.so REPS=5 timeout -k 10 300 python3 tools/replay_profile.py 65536 10000 > $O/replay_old.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay_old.txt; exit 4; }
echo "new: $(grep -E '^median' $O/replay.txt)"; echo "old: $(grep -E '^median' $O/replay_old.txt)"
PZ_VOTE_TRACE=1 timeout -k 10 200 python3 tools/vote_trace.py 524288 390 > $O/trace_33.txt 2>&1 || { echo TRACE_FAIL; tail -3 $O/trace_33.txt; exit 5; }
grep -v amdgpu $O/trace_33.txt
echo DONE2
