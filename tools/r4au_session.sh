# Final-tree sanity after the last rebuild: smoke and the golden + replay suites
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4au; mkdir -p $O
PYTEST_FILES="tests/test_golden.py tests/test_replay.py" PYTEST_TIMEOUT=600 bash tools/gpu_session.sh r4au tests,smoke || exit 1
echo DONE
