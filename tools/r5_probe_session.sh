#!/bin/bash
# Round 5 probe session: the attestation encoder (GPU tests, same-process A/B of the one-pass
# kernel against round 4's three launches) and the window pass's phase stamps.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd "$R" || exit 2
O=$R/gpurun_out/${1:-r5d}; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_wire_att_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$O/pytest_wire_att.txt" 2>&1 || { echo WATT_TESTS_FAIL; tail -40 "$O/pytest_wire_att.txt"; exit 12; }
tail -3 "$O/pytest_wire_att.txt"
PZ_PROBE_LIB=$R/build/ab/libprysm_hip.so timeout -k 10 300 python -u tools/wire_att_probe.py 50 > "$O/wire_att_probe.txt" 2>&1 \
  || { echo WATT_PROBE_FAIL; tail -20 "$O/wire_att_probe.txt"; exit 13; }
cat "$O/wire_att_probe.txt"
timeout -k 10 300 python -u tools/epoch_trace.py > "$O/epoch_trace.txt" 2>&1 || { echo TRACE_FAIL; tail -20 "$O/epoch_trace.txt"; exit 14; }
ABL=0xf timeout -k 10 300 python -u tools/epoch_trace.py >> "$O/epoch_trace.txt" 2>&1 || { echo TRACE_FAIL; tail -20 "$O/epoch_trace.txt"; exit 14; }
cat "$O/epoch_trace.txt"
