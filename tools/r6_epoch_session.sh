#!/bin/bash
# Round 6 epoch session: the epoch GPU suite (+ its A/B tests), then same-process cold steps of
# the window-pass forms (tools/epoch_cold.py, ABL=$EABL against the A/B library: 0 the product,
# 0x40000 round 5's prologue) and phase stamps of the product and of $TABL.
#   tools/r6_epoch_session.sh TAG [skip-tests]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd "$R" || exit 2
O=$R/gpurun_out/${1:-r6e}; mkdir -p "$O"
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_native_gpu.py ${EXTRA_TESTS} -m gpu -x -v --timeout 120 \
    --timeout-method thread > "$O/pytest_epoch.txt" 2>&1 || { echo TESTS_FAIL; tail -40 "$O/pytest_epoch.txt"; exit 12; }
  tail -3 "$O/pytest_epoch.txt"
  timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py -m ab -x -v --timeout 120 --timeout-method thread \
    > "$O/pytest_epoch_ab.txt" 2>&1 || { echo AB_TESTS_FAIL; tail -40 "$O/pytest_epoch_ab.txt"; exit 18; }
  tail -3 "$O/pytest_epoch_ab.txt"
fi
PZ_PROBE_LIB=build/ab/libprysm_hip.so ABL=${EABL:-0,0x40000} REPS=${REPS:-2} timeout -k 10 500 python -u tools/epoch_cold.py \
  > "$O/epoch_cold_ab.txt" 2>&1 || { echo COLD_FAIL; tail -20 "$O/epoch_cold_ab.txt"; exit 13; }
cat "$O/epoch_cold_ab.txt"
timeout -k 10 300 python -u tools/epoch_trace.py > "$O/epoch_trace.txt" 2>&1 || { echo TRACE_FAIL; tail -20 "$O/epoch_trace.txt"; exit 15; }
cat "$O/epoch_trace.txt"
if [ -n "$TABL" ]; then
  ABL=$TABL timeout -k 10 300 python -u tools/epoch_trace.py > "$O/epoch_trace_abl.txt" 2>&1 \
    || { echo TRACE2_FAIL; tail -20 "$O/epoch_trace_abl.txt"; exit 16; }
  cat "$O/epoch_trace_abl.txt"
fi

if [ -n "$WABL" ]; then
  PZ_PROBE_LIB=build/ab/libprysm_hip.so ABL=$WABL timeout -k 10 300 python -u tools/epoch_warm.py > "$O/epoch_warm_ab.txt" 2>&1 \
    || { echo WARM_FAIL; tail -20 "$O/epoch_warm_ab.txt"; exit 17; }
  cat "$O/epoch_warm_ab.txt"
fi
echo "SESSION_DONE"
