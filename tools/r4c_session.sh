set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4c; mkdir -p $O
PYTEST_FILES="tests/test_replay.py" PYTEST_K="vote_queue or configs4 or golden or panic" PYTEST_TIMEOUT=600 bash tools/gpu_session.sh r4c tests || exit 1
cd $R && AB=PZ_VOTE_PATH AB_VALUES=segments,packed,direct REPS=3 timeout -k 10 200 python3 tools/replay_profile.py 65536 10000 > $O/replay_ab_path.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay_ab_path.txt; exit 4; }
grep median $O/replay_ab_path.txt
AB=PZ_VOTE_UNION AB_VALUES=item,att REPS=3 timeout -k 10 200 python3 tools/replay_profile.py 65536 10000 > $O/replay_ab_union.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay_ab_union.txt; exit 5; }
grep median $O/replay_ab_union.txt
AB=PZ_EPOCH_PACK AB_VALUES=copy,direct REPS=3 timeout -k 10 200 python3 tools/replay_profile.py 65536 10000 > $O/replay_ab_epack.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay_ab_epack.txt; exit 6; }
grep median $O/replay_ab_epack.txt
echo DONE
