set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4ae; mkdir -p $O
PYTEST_FILES="tests/test_native_gpu.py tests/test_golden.py" PYTEST_K="single or one or golden" PYTEST_TIMEOUT=600 bash tools/gpu_session.sh r4ae tests || exit 1
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
  for L in new old; do
    LIB=$R/prysm_amd/libprysm_hip.so; [ $L = old ] && LIB=$R/build/old/libprysm_hip.so
    PZ_PROBE_LIB=$LIB timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_${L}_$i -o run --output-format csv -- python3 $R/tools/pmc_workload.py epoch_single > $O/prof_${L}_$i.log 2>&1 || { echo PROF_FAIL; tail -5 $O/prof_${L}_$i.log; exit 6; }
    echo "$L $i: $(grep -i one_se16 $O/prof_${L}_$i/run_kernel_stats.csv | cut -d, -f1-8)"
  done
done
echo DONE
