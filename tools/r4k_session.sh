set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4k; mkdir -p $O
PYTEST_FILES="tests/test_replay.py tests/test_shm_multiprocess_gpu.py tests/test_native_gpu.py" PYTEST_TIMEOUT=900 bash tools/gpu_session.sh r4k tests || exit 1
for i in 1 2; do
  AB=PZ_VOTE_PATH AB_VALUES=segments,direct,packed REPS=3 timeout -k 10 200 python3 tools/replay_profile.py 65536 10000 > $O/replay_new_$i.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay_new_$i.txt; exit 4; }
  grep median $O/replay_new_$i.txt; grep phases $O/replay_new_$i.txt | tail -1
  PZ_PROBE_LIB=build/old/libprysm_hip.so AB=PZ_VOTE_PATH AB_VALUES=packed REPS=3 timeout -k 10 200 python3 tools/replay_profile.py 65536 10000 > $O/replay_old_$i.txt 2>&1 || { echo REPLAY_OLD_FAIL; tail -5 $O/replay_old_$i.txt; exit 5; }
  grep median $O/replay_old_$i.txt | sed 's/^/old /'; grep phases $O/replay_old_$i.txt | tail -1
done
PZ_PROBE_LIB=build/prof/libprysm_hip.so timeout -k 10 200 python3 tools/walk_sampler.py 10000 6 50 > $O/walk_sampler.txt 2>&1 || { echo SAMPLER_FAIL; tail -5 $O/walk_sampler.txt; }
echo DONE
