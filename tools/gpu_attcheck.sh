#!/bin/bash
# processAttestation checks: GPU tests, then the bench's attcheck leg on this build and (if
# present) build/ab/libprysm_hip_old.so, via tools/attcheck_probe.py.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/${1:-attc}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_attcheck_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.txt; exit 12; }
tail -2 $O/pytest.txt
timeout -k 10 200 python -u tools/attcheck_probe.py > $O/probe_new.txt 2>&1 || { echo PROBE_FAIL; tail -20 $O/probe_new.txt; exit 13; }
cat $O/probe_new.txt
if [ -f build/ab/libprysm_hip_old.so ]; then
  PZ_PROBE_LIB=$R/build/ab/libprysm_hip_old.so timeout -k 10 200 python -u tools/attcheck_probe.py > $O/probe_old.txt 2>&1 || { echo OLD_FAIL; tail -20 $O/probe_old.txt; exit 14; }
  cat $O/probe_old.txt
fi
echo ALLDONE
