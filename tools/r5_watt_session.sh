#!/bin/bash
# Round 5 attestation-encoder session: GPU tests, then the same-process A/B probe (product,
# round 4's three launches, the byte-wise stage, the other sizing tiles) and a kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd "$R" || exit 2
O=$R/gpurun_out/${1:-r5w}; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_wire_att_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$O/pytest_wire_att.txt" 2>&1 || { echo WATT_TESTS_FAIL; tail -40 "$O/pytest_wire_att.txt"; exit 16; }
tail -2 "$O/pytest_wire_att.txt"
PZ_PROBE_LIB=$R/build/ab/libprysm_hip.so timeout -k 10 300 python -u tools/wire_att_probe.py 50 > "$O/wire_att_probe.txt" 2>&1 \
  || { echo WATT_PROBE_FAIL; tail -20 "$O/wire_att_probe.txt"; exit 17; }
cat "$O/wire_att_probe.txt"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o watt --output-format csv \
  -- python3 "$R/tools/wire_att_probe.py" 20 > "$O/prof.log" 2>&1) || { echo PROF_FAIL; tail -20 "$O/prof.log"; exit 18; }
grep -h "wire_att" "$O"/prof/*kernel_stats.csv | cut -c1-120
echo SESSION_DONE
