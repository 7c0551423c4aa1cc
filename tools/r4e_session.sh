set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4e; mkdir -p $O
PYTEST_FILES="tests/test_native_gpu.py tests/test_epoch_gpu.py tests/test_shm_multiprocess_gpu.py tests/test_replay.py" PYTEST_TIMEOUT=900 bash tools/gpu_session.sh r4e tests || exit 1
cd $R && VARIANTS=0,65536,32768,0,65536,32768 timeout -k 10 300 python3 tools/epoch_cold_ab.py > $O/cold_ab.txt 2>&1 || { echo COLD_FAIL; tail -5 $O/cold_ab.txt; exit 3; }
cat $O/cold_ab.txt
AB=PZ_VOTE_PATH AB_VALUES=segments REPS=5 timeout -k 10 200 python3 tools/replay_profile.py 65536 10000 > $O/replay.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay.txt; exit 4; }
grep median $O/replay.txt; grep phases $O/replay.txt | tail -1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $R/tools/pmc_workload.py epoch1m_cold > $O/kt.log 2>&1 || { echo KT_FAIL; tail -5 $O/kt.log; exit 2; }
head -6 $O/kt/kt_kernel_stats.csv | cut -c1-150
echo DONE
