#!/bin/bash
# r2o: attestation checks with nontemporal column loads: tests and same-process A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r2o; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_attcheck_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_attcheck.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_attcheck.txt; exit 12; }
tail -2 $O/pytest_attcheck.txt
timeout -k 10 200 python -u tools/attcheck_probe.py > $O/attcheck_probe.txt 2>&1 || { echo PROBE_FAIL; tail -20 $O/attcheck_probe.txt; exit 11; }
cat $O/attcheck_probe.txt
