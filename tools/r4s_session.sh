set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4s; mkdir -p $O
PYTEST_FILES="tests/test_replay.py tests/test_native_gpu.py tests/test_shm_multiprocess_gpu.py tests/test_golden.py" PYTEST_K="not 2097152" PYTEST_TIMEOUT=900 bash tools/gpu_session.sh r4s tests || exit 1
cd $R && REPS=4 timeout -k 10 200 python3 tools/replay_profile.py 65536 10000 > $O/replay.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay.txt; exit 4; }
grep -E "median|blocks/s" $O/replay.txt | tail -5; grep phases $O/replay.txt | tail -1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tl -o run --output-format csv -- python3 $R/tools/replay_timeline.py $O/timeline.json > $O/tl.log 2>&1 || { echo TL_FAIL; tail -5 $O/tl.log; exit 5; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_single -o run --output-format csv -- python3 $R/tools/pmc_workload.py epoch_single > $O/prof_single.log 2>&1 || { echo PROF_SINGLE_FAIL; tail -5 $O/prof_single.log; exit 6; }
grep -i "one" $O/prof_single/run_kernel_stats.csv | head -3
echo DONE
