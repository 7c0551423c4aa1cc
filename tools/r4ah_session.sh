set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4ah; mkdir -p $O
PYTEST_FILES="tests/test_replay.py" PYTEST_K="wide_committees or vote_queue" PYTEST_TIMEOUT=600 bash tools/gpu_session.sh r4ah tests || exit 1
grep -E "PASSED|FAILED" $O/pytest_gpu.txt | head -20
echo DONE
