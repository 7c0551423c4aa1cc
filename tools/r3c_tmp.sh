set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r3e; mkdir -p $O
PYTEST_FILES="tests/test_bench_launch.py tests/test_replay.py tests/test_canonical_gpu.py tests/test_state_mirror_gpu.py tests/test_golden.py tests/test_votes_gpu.py" bash tools/gpu_session.sh r3e tests || exit $?
for i in 1 2; do
  timeout -k 10 150 python -u tools/replay_profile.py 65536 10000 > $O/replay_$i.txt 2>&1 || { echo REPLAY_FAIL; tail $O/replay_$i.txt; exit 11; }
  grep -E "process_serialized|phases" $O/replay_$i.txt
done
