#!/bin/bash
# r2z: epoch pre kernel with batched popcount loads: epoch GPU tests, step ablation.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r2z; mkdir -p $O
true
tail -2 $O/pytest_epoch.txt
timeout -k 10 300 python -u tools/fused_parts.py > $O/fused_parts.json 2>&1 || { echo PARTS_FAIL; tail -20 $O/fused_parts.json; exit 13; }
cat $O/fused_parts.json
