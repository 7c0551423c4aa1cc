#!/bin/bash
# Quick GPU iteration: GPU tests + in-process kernel timing tools.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/${1:-quick}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.txt; exit 12; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 200 python -u tools/hash_ab.py > $O/hash_ab.txt 2>&1 || { echo AB_FAIL; tail -20 $O/hash_ab.txt; exit 13; }
cat $O/hash_ab.txt
timeout -k 10 200 python -u tools/epoch_parts.py > $O/epoch_parts.txt 2>&1 || { echo EP_FAIL; tail -20 $O/epoch_parts.txt; exit 14; }
cat $O/epoch_parts.txt
