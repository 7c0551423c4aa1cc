#!/bin/bash
# Round 5 epoch session: the epoch GPU suite (and its A/B tests against the A/B library), the
# product's cold step, the window-pass ablations (tools/epoch_cold.py ABL=...), phase stamps
# (tools/epoch_trace.py), then the attestation encoder's tests and probe.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd "$R" || exit 2
O=$R/gpurun_out/${1:-r5a}; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_native_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$O/pytest_epoch.txt" 2>&1 || { echo TESTS_FAIL; tail -40 "$O/pytest_epoch.txt"; exit 12; }
tail -3 "$O/pytest_epoch.txt"
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py -m ab -x -v --timeout 120 --timeout-method thread \
  > "$O/pytest_epoch_ab.txt" 2>&1 || { echo AB_TESTS_FAIL; tail -40 "$O/pytest_epoch_ab.txt"; exit 18; }
tail -3 "$O/pytest_epoch_ab.txt"
ABL= timeout -k 10 300 python -u tools/epoch_cold.py > "$O/epoch_cold.txt" 2>&1 || { echo COLD_FAIL; tail -20 "$O/epoch_cold.txt"; exit 13; }
cat "$O/epoch_cold.txt"
PZ_PROBE_LIB=build/ab/libprysm_hip.so ABL=${EABL:-4096,1,2,4,7} REPS=1 timeout -k 10 400 python -u tools/epoch_cold.py \
  > "$O/epoch_abl.txt" 2>&1 || { echo ABL_FAIL; tail -20 "$O/epoch_abl.txt"; exit 14; }
cat "$O/epoch_abl.txt"
timeout -k 10 300 python -u tools/epoch_trace.py > "$O/epoch_trace.txt" 2>&1 || { echo TRACE_FAIL; tail -20 "$O/epoch_trace.txt"; exit 15; }
cat "$O/epoch_trace.txt"
timeout -k 10 300 python -u -m pytest tests/test_wire_att_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$O/pytest_wire_att.txt" 2>&1 || { echo WATT_TESTS_FAIL; tail -40 "$O/pytest_wire_att.txt"; exit 16; }
tail -3 "$O/pytest_wire_att.txt"
PZ_PROBE_LIB=$R/build/ab/libprysm_hip.so timeout -k 10 300 python -u tools/wire_att_probe.py 50 > "$O/wire_att_probe.txt" 2>&1 \
  || { echo WATT_PROBE_FAIL; tail -20 "$O/wire_att_probe.txt"; exit 17; }
cat "$O/wire_att_probe.txt"
