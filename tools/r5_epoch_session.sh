#!/bin/bash
# Round 5 epoch session: the epoch GPU suite, the product's cold step, the window-pass ablations
# (the A/B library: tools/epoch_cold.py ABL=...).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd "$R" || exit 2
O=$R/gpurun_out/${1:-r5a}; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_native_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$O/pytest_epoch.txt" 2>&1 || { echo TESTS_FAIL; tail -40 "$O/pytest_epoch.txt"; exit 12; }
tail -3 "$O/pytest_epoch.txt"
timeout -k 10 300 python -u tools/epoch_cold.py > "$O/epoch_cold.txt" 2>&1 || { echo COLD_FAIL; tail -20 "$O/epoch_cold.txt"; exit 13; }
cat "$O/epoch_cold.txt"
PZ_LIB=build/ab/libprysm_hip.so ABL=${ABL:-0x200,0x300,0x400,1,2,4,8,15} REPS=1 timeout -k 10 400 python -u tools/epoch_cold.py \
  > "$O/epoch_abl.txt" 2>&1 || { echo ABL_FAIL; tail -20 "$O/epoch_abl.txt"; exit 14; }
cat "$O/epoch_abl.txt"
