set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4n; mkdir -p $O
PYTEST_FILES="tests/test_native_gpu.py" PYTEST_TIMEOUT=600 bash tools/gpu_session.sh r4n tests || exit 1
cd $R && VARIANTS=0,4096,0,4096 timeout -k 10 300 python3 tools/epoch_cold_ab.py > $O/cold_ab.txt 2>&1 || { echo COLD_FAIL; tail -5 $O/cold_ab.txt; exit 3; }
sed 's/  frac(layout).*//' $O/cold_ab.txt
AB=PZ_EPOCH_PREP AB_VALUES=merged,after REPS=4 timeout -k 10 200 python3 tools/replay_profile.py 65536 10000 > $O/replay_prep.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay_prep.txt; exit 5; }
grep median $O/replay_prep.txt; grep phases $O/replay_prep.txt | tail -2
cd /tmp && export TMPDIR=/tmp
FUSED_VARIANT=4096 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_xcd1m/fetch -o fetch -- python3 $R/tools/pmc_workload.py epoch1m > $O/pmc_xcd.log 2>&1 || { echo PMC_FAIL; tail -5 $O/pmc_xcd.log; exit 4; }
FUSED_VARIANT=4096 timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_xcd1m/write -o write -- python3 $R/tools/pmc_workload.py epoch1m >> $O/pmc_xcd.log 2>&1 || { echo PMC_FAIL; tail -5 $O/pmc_xcd.log; exit 4; }
python3 $R/tools/pmc_summary.py $O/pmc_xcd1m > $O/pmc_xcd1m/summary.json && echo pmc ok
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_single -o run --output-format csv -- python3 $R/tools/pmc_workload.py epoch_single > $O/prof_single.log 2>&1 || { echo PROF_SINGLE_FAIL; tail -5 $O/prof_single.log; exit 6; }
grep -i "one" $O/prof_single/run_kernel_stats.csv | head -3
echo DONE
