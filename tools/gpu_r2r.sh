#!/bin/bash
# r2r: the one-pass epoch step's ablation incl. nontemporal balance loads (variant 64).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r2r; mkdir -p $O
timeout -k 10 300 python -u tools/fused_parts.py > $O/fused_parts.json 2>&1 || { echo PARTS_FAIL; tail -20 $O/fused_parts.json; exit 13; }
cat $O/fused_parts.json
