set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
PYTEST_FILES="tests/test_wire_att_gpu.py" TOOL_ARGS="50" bash tools/gpu_session.sh r3g tests,tool:wire_att_probe
