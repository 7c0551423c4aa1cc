#!/bin/bash
# r2u: attestation encoder write kernel with nontemporal loads: tests and same-process A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r2u; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_wire_att_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_watt.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_watt.txt; exit 12; }
tail -2 $O/pytest_watt.txt
timeout -k 10 200 python -u tools/wire_att_probe.py > $O/wire_att_probe.txt 2>&1 || { echo PROBE_FAIL; tail -20 $O/wire_att_probe.txt; exit 11; }
cat $O/wire_att_probe.txt
