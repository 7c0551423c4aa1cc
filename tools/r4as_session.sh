# A/B: the grouped tally's member and balance loads hoisted before the record loop, and the loop
# over the group's id words only
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4as; mkdir -p $O
PYTEST_FILES="tests/test_replay.py tests/test_golden.py" PYTEST_TIMEOUT=600 bash tools/gpu_session.sh r4as tests || exit 1
timeout -k 10 200 python3 tools/vote_trace.py > $O/trace.txt 2>&1 || { echo TRACE_FAIL; tail -5 $O/trace.txt; exit 3; }
grep -v amdgpu.ids $O/trace.txt
for i in 1 2; do
  REPS=5 timeout -k 10 300 python3 tools/replay_profile.py 65536 10000 > $O/replay_new_$i.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay_new_$i.txt; exit 4; }
  PZ_PROBE_LIB=build/old/libprysm_hip.so REPS=5 timeout -k 10 300 python3 tools/replay_profile.py 65536 10000 > $O/replay_old_$i.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay_old_$i.txt; exit 4; }
  echo "new $i: $(grep -E '^median' $O/replay_new_$i.txt)"; echo "old $i: $(grep -E '^median' $O/replay_old_$i.txt)"
done
echo DONE
