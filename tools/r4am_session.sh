# Robustness: the chain suites with the per-attestation tally forced (PZ_VOTE_GROUPS=0) and with
# round 3's packed queue path (PZ_VOTE_PATH=packed), on the final tree.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4am; mkdir -p $O
F="tests/test_replay.py tests/test_golden.py tests/test_shm_multiprocess_gpu.py"
PZ_VOTE_GROUPS=0 timeout -k 10 600 python -u -m pytest $F -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_groups0.txt 2>&1 || { echo FAIL_G0; tail -30 $O/pytest_groups0.txt; exit 1; }
tail -1 $O/pytest_groups0.txt
PZ_VOTE_PATH=packed timeout -k 10 600 python -u -m pytest $F -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_packed.txt 2>&1 || { echo FAIL_PACKED; tail -30 $O/pytest_packed.txt; exit 2; }
tail -1 $O/pytest_packed.txt
echo DONE
