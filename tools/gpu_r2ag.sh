#!/bin/bash
# r2ag: epoch pre kernel with batched popcount loads: epoch GPU tests, step ablation.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r2ag; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_epoch_gpu.py tests/test_native_gpu.py tests/test_onepass_multirank.py tests/test_state_mirror_gpu.py tests/test_multirank.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_epoch.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_epoch.txt; exit 12; }
tail -2 $O/pytest_epoch.txt
timeout -k 10 300 python -u tools/fused_parts.py > $O/fused_parts.json 2>&1 || { echo PARTS_FAIL; tail -20 $O/fused_parts.json; exit 13; }
cat $O/fused_parts.json
