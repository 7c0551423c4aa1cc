set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4i; mkdir -p $O
PYTEST_FILES="tests/test_replay.py tests/test_golden.py tests/test_native_gpu.py tests/test_shm_multiprocess_gpu.py tests/test_votes_gpu.py" PYTEST_TIMEOUT=900 bash tools/gpu_session.sh r4i tests || exit 1
cd $R && VARIANTS=0,0/nl,0,0/nl timeout -k 10 300 python3 tools/epoch_cold_ab.py > $O/cold_ab.txt 2>&1 || { echo COLD_FAIL; tail -5 $O/cold_ab.txt; exit 3; }
sed 's/  frac(layout).*//' $O/cold_ab.txt
AB=PZ_VOTE_PATH AB_VALUES=segments,packed,direct REPS=3 timeout -k 10 200 python3 tools/replay_profile.py 65536 10000 > $O/replay.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay.txt; exit 4; }
grep median $O/replay.txt; grep phases $O/replay.txt | tail -3
cd /tmp && export TMPDIR=/tmp
AB=PZ_VOTE_PATH AB_VALUES=segments REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_replay -o run --output-format csv -- python3 $R/tools/replay_profile.py 65536 10000 > $O/prof_replay.log 2>&1 || { echo PROF_REPLAY_FAIL; tail -5 $O/prof_replay.log; exit 5; }
echo DONE
