set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4f; mkdir -p $O
PYTEST_FILES="tests/test_replay.py tests/test_shm_multiprocess_gpu.py tests/test_golden.py tests/test_votes_gpu.py tests/test_native_gpu.py" PYTEST_TIMEOUT=1000 bash tools/gpu_session.sh r4f tests || exit 1
cd $R && VARIANTS=0,131072,65536,262144,0,131072,65536,262144 timeout -k 10 300 python3 tools/epoch_cold_ab.py > $O/cold_ab.txt 2>&1 || { echo COLD_FAIL; tail -5 $O/cold_ab.txt; exit 3; }
cat $O/cold_ab.txt
AB=PZ_VOTE_PATH AB_VALUES=segments,packed REPS=4 timeout -k 10 200 python3 tools/replay_profile.py 65536 10000 > $O/replay.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay.txt; exit 4; }
grep median $O/replay.txt; grep phases $O/replay.txt | tail -2
PZ_PROBE_LIB=build/prof/libprysm_hip.so timeout -k 10 200 python3 tools/walk_sampler.py 10000 6 50 > $O/walk_sampler.txt 2>&1 || { echo SAMPLER_FAIL; tail -5 $O/walk_sampler.txt; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $O/list_avail.txt 2>&1 || echo LIST_FAIL
echo DONE
