#!/bin/bash
# r2h: wire encoder A/B (mid-build re-read of the look-back window), its tests, phase trace.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r2m; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_wire_gpu.py tests/test_replay.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_wire.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_wire.txt; exit 12; }
tail -2 $O/pytest_wire.txt
timeout -k 10 200 python -u tools/wire_probe.py 30 ab > $O/wire_probe.txt 2>&1 || { echo PROBE_FAIL; tail -20 $O/wire_probe.txt; exit 11; }
cat $O/wire_probe.txt
timeout -k 10 120 python -u tools/wire_trace.py 32 > $O/wire_trace32.json 2>&1 || { echo TRACE_FAIL; tail -20 $O/wire_trace32.json; exit 15; }
echo TRACE_OK
