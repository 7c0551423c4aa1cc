#!/bin/bash
# r2s: wire encoder tests incl. the multi-window look-back variants.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r2s; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_wire_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_wire.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_wire.txt; exit 12; }
tail -4 $O/pytest_wire.txt
