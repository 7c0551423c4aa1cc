set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4b; mkdir -p $O
PYTEST_FILES="tests/test_shm_multiprocess_gpu.py tests/test_replay.py tests/test_native_gpu.py" PYTEST_TIMEOUT=900 bash tools/gpu_session.sh r4b tests || exit 1
cd $R && AB=PZ_VOTE_STAGED REPS=3 timeout -k 10 200 python3 tools/replay_profile.py 65536 10000 > $O/replay_ab.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay_ab.txt; exit 4; }
grep median $O/replay_ab.txt
cd /tmp && export TMPDIR=/tmp
for v in 0 4096; do
  FUSED_VARIANT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o kt -- python3 $R/tools/pmc_workload.py epoch1m_cold > $O/kt_$v.log 2>&1 || { echo KT_FAIL $v; tail -5 $O/kt_$v.log; exit 2; }
done
cd $R && VARIANTS=0,4096,0,4096 timeout -k 10 300 python3 tools/epoch_cold_ab.py > $O/cold_ab.txt 2>&1 || { echo COLD_FAIL; tail -5 $O/cold_ab.txt; exit 3; }
cat $O/cold_ab.txt
PZ_EPOCH_SE32=1 VARIANTS=0,4096 timeout -k 10 300 python3 tools/epoch_cold_ab.py > $O/cold_ab_se32.txt 2>&1 || { echo COLD32_FAIL; tail -5 $O/cold_ab_se32.txt; exit 5; }
cat $O/cold_ab_se32.txt
echo DONE
