# A/B: the epoch's count and reward passes in one grid (PZ_EPOCH_FOLD=1), tests first
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4at; mkdir -p $O
PZ_EPOCH_FOLD=1 timeout -k 10 400 python -u -m pytest tests/test_replay.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_fold.txt 2>&1 || { echo FOLD_TESTS_FAIL; tail -30 $O/pytest_fold.txt; exit 1; }
tail -1 $O/pytest_fold.txt
cd $R && AB=PZ_EPOCH_FOLD AB_VALUES=0,1 REPS=5 timeout -k 10 300 python3 tools/replay_profile.py 65536 10000 > $O/replay_ab.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay_ab.txt; exit 4; }
grep -E "^median" $O/replay_ab.txt; grep phases $O/replay_ab.txt | tail -2
cd $R && AB=PZ_EPOCH_FOLD AB_VALUES=0,1 REPS=5 timeout -k 10 300 python3 tools/replay_profile.py 65536 10000 > $O/replay_ab2.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay_ab2.txt; exit 4; }
grep -E "^median" $O/replay_ab2.txt
echo DONE
