set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4ag; mkdir -p $O
PYTEST_FILES="tests/test_replay.py tests/test_golden.py" PYTEST_TIMEOUT=600 bash tools/gpu_session.sh r4ag tests || exit 1
cd $R && REPS=5 timeout -k 10 300 python3 tools/replay_profile.py 65536 10000 > $O/replay.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay.txt; exit 4; }
grep -E "^median" $O/replay.txt; grep phases $O/replay.txt | tail -1
PZ_PROBE_LIB=build/old/libprysm_hip.so REPS=5 timeout -k 10 300 python3 tools/replay_profile.py 65536 10000 > $O/replay_old.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay_old.txt; exit 4; }
echo "old: $(grep -E '^median' $O/replay_old.txt)"
echo DONE
