#!/bin/bash
# Round 5 epoch session: the window-pass lab, the epoch GPU suite, the product's cold step.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd "$R" || exit 2
O=$R/gpurun_out/${1:-r5a}; mkdir -p "$O"
timeout -k 10 150 build/epoch_lab 1048576 16 16 > "$O/lab_1m.txt" 2>&1 || { echo LAB1_FAIL; tail -20 "$O/lab_1m.txt"; exit 11; }
tail -14 "$O/lab_1m.txt"
timeout -k 10 150 build/epoch_lab 65536 256 1 > "$O/lab_65k.txt" 2>&1 || { echo LAB2_FAIL; tail -20 "$O/lab_65k.txt"; exit 11; }
tail -14 "$O/lab_65k.txt"
timeout -k 10 900 python -u -m pytest tests/test_native_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$O/pytest_epoch.txt" 2>&1 || { echo TESTS_FAIL; tail -40 "$O/pytest_epoch.txt"; exit 12; }
tail -3 "$O/pytest_epoch.txt"
timeout -k 10 300 python -u tools/epoch_cold.py > "$O/epoch_cold.txt" 2>&1 || { echo COLD_FAIL; tail -20 "$O/epoch_cold.txt"; exit 13; }
cat "$O/epoch_cold.txt"
