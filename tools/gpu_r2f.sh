#!/bin/bash
# r2f: GPU tests, bench, rocprof kernel stats, then the wire encoder's probe and phase trace.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r2f; mkdir -p $O
bash tools/gpu_session.sh r2f || exit $?
cd $R
timeout -k 10 120 python -u tools/wire_probe.py 30 > $O/wire_probe.txt 2>&1 || { echo PROBE_FAIL; tail -20 $O/wire_probe.txt; exit 11; }
cat $O/wire_probe.txt
timeout -k 10 120 python -u tools/wire_trace.py 32 > $O/wire_trace32.json 2>&1 || { echo TRACE_FAIL; tail -20 $O/wire_trace32.json; exit 15; }
echo TRACE_OK
