set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4l; mkdir -p $O
PYTEST_FILES="tests/test_native_gpu.py tests/test_replay.py tests/test_golden.py" PYTEST_TIMEOUT=900 bash tools/gpu_session.sh r4l tests || exit 1
cd $R && VARIANTS=0,131072,0,131072 timeout -k 10 300 python3 tools/epoch_cold_ab.py > $O/cold_ab.txt 2>&1 || { echo COLD_FAIL; tail -5 $O/cold_ab.txt; exit 3; }
sed 's/  frac(layout).*//' $O/cold_ab.txt
AB=PZ_VOTE_PATH AB_VALUES=direct,segments REPS=4 timeout -k 10 200 python3 tools/replay_profile.py 65536 10000 > $O/replay.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay.txt; exit 4; }
grep median $O/replay.txt; grep phases $O/replay.txt | tail -1
echo DONE
