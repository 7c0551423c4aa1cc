set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4d; mkdir -p $O
PYTEST_FILES="tests/test_native_gpu.py tests/test_epoch_gpu.py tests/test_shm_multiprocess_gpu.py" PYTEST_K="not replay and not chain" PYTEST_TIMEOUT=900 bash tools/gpu_session.sh r4d tests || exit 1
cd $R && VARIANTS=0,32768,0,32768 timeout -k 10 300 python3 tools/epoch_cold_ab.py > $O/cold_ab.txt 2>&1 || { echo COLD_FAIL; tail -5 $O/cold_ab.txt; exit 3; }
cat $O/cold_ab.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $R/tools/pmc_workload.py epoch1m_cold > $O/kt.log 2>&1 || { echo KT_FAIL; tail -5 $O/kt.log; exit 2; }
head -6 $O/kt/kt_kernel_stats.csv | cut -c1-150
echo DONE
