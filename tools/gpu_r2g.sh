#!/bin/bash
# r2g: wire encoder A/B (32-bit stage build vs loop form), its tests, phase traces, then the PMC passes.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r2g; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_wire_gpu.py tests/test_replay.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_wire.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_wire.txt; exit 12; }
tail -2 $O/pytest_wire.txt
timeout -k 10 200 python -u tools/wire_probe.py 30 ab > $O/wire_probe.txt 2>&1 || { echo PROBE_FAIL; tail -20 $O/wire_probe.txt; exit 11; }
cat $O/wire_probe.txt
timeout -k 10 120 python -u tools/wire_trace.py 32 > $O/wire_trace32.json 2>&1 || { echo TRACE_FAIL; tail -20 $O/wire_trace32.json; exit 15; }
timeout -k 10 120 python -u tools/wire_trace.py 544 > $O/wire_trace544.json 2>&1 || { echo TRACE_FAIL; tail -20 $O/wire_trace544.json; exit 16; }
timeout -k 10 120 python -u tools/wire_trace.py 288 > $O/wire_trace288.json 2>&1 || { echo TRACE_FAIL; tail -20 $O/wire_trace288.json; exit 17; }
echo TRACE_OK
bash tools/gpu_pmc.sh r2g_pmc || exit $?
cd $R && python3 tools/pmc_summary.py gpurun_out/r2g_pmc > gpurun_out/r2g/pmc_summary.json && python3 tools/pmc_summary.py gpurun_out/r2g_pmc_epoch1m > gpurun_out/r2g/pmc_summary_epoch1m.json && echo PMC_SUMMARY_OK
