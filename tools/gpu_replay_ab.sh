#!/bin/bash
# Block pipeline: replay + vote GPU tests, then tools/replay_profile.py on this build and (if
# present) on build/ab/libprysm_hip_old.so for a same-box A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/${1:-rpab}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_replay.py tests/test_votes_gpu.py tests/test_canonical_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.txt; exit 12; }
tail -2 $O/pytest.txt
timeout -k 10 200 python -u tools/replay_profile.py 65536 10000 > $O/new.txt 2>&1 || { echo NEW_FAIL; tail -20 $O/new.txt; exit 13; }
grep -E "process_serialized|phases" $O/new.txt
if [ -f build/ab/libprysm_hip_old.so ]; then
  PZ_PROBE_LIB=$R/build/ab/libprysm_hip_old.so timeout -k 10 200 python -u tools/replay_profile.py 65536 10000 > $O/old.txt 2>&1 || { echo OLD_FAIL; tail -20 $O/old.txt; exit 14; }
  grep -E "process_serialized|phases" $O/old.txt
fi
echo ALLDONE
