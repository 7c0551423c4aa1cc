set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r3d; mkdir -p $O
PYTEST_FILES="tests/test_native_gpu.py tests/test_replay.py tests/test_canonical_gpu.py tests/test_state_mirror_gpu.py tests/test_golden.py" bash tools/gpu_session.sh r3d tests || exit $?
for i in 1 2 3; do
  timeout -k 10 150 python -u tools/replay_profile.py 65536 10000 > $O/replay_$i.txt 2>&1 || { echo REPLAY_FAIL; tail $O/replay_$i.txt; exit 11; }
  grep -E "process_serialized|phases" $O/replay_$i.txt
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/tools/pmc_workload.py epoch_single > $O/kt.log 2>&1) || { echo KT_FAIL; tail $O/kt.log; exit 12; }
find $O/kt -name "*kernel_stats.csv" | head -1 | xargs cat
BENCH_ARGS="--no-replay --no-wire --no-attcheck --no-cpu-baseline" bash tools/gpu_session.sh r3d bench
