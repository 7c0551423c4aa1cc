set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r3o; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_replay.py tests/test_votes_gpu.py tests/test_canonical_gpu.py -m gpu > $O/tests.txt 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.txt; exit 12; }
tail -2 $O/tests.txt
for k in 1 2 3; do
  timeout -k 10 150 python -u tools/replay_profile.py 65536 10000 > $O/replay_$k.txt 2>&1 || { echo REPLAY_FAIL; tail $O/replay_$k.txt; exit 11; }
  grep -E "process_serialized|phases" $O/replay_$k.txt
done
timeout -k 10 300 python -u tools/epoch_cold_ab.py > $O/cold_ab.txt 2>&1 || { echo AB_FAIL; tail -20 $O/cold_ab.txt; exit 14; }
grep variant $O/cold_ab.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o replay -- python3 -u $R/tools/replay_profile.py 65536 2000 > $O/trace.txt 2>&1 || { echo TRACE_FAIL; tail -20 $O/trace.txt; exit 13; }
