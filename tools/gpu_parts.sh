#!/bin/bash
# Epoch per-part timing + epoch parity tests (quick iteration on the epoch kernels).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/${1:-parts}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_epoch_gpu.py tests/test_multirank.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.txt; exit 12; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 200 python -u tools/epoch_parts.py > $O/epoch_parts.txt 2>&1 || { echo EP_FAIL; tail -20 $O/epoch_parts.txt; exit 14; }
tail -1 $O/epoch_parts.txt
