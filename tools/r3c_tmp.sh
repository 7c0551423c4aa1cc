set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r3k; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_replay.py tests/test_canonical_gpu.py -m gpu > $O/tests.txt 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.txt; exit 12; }
tail -2 $O/tests.txt
for mode in pipe nopipe pipe nopipe; do
  if [ $mode = pipe ]; then export PZ_CHAIN_PIPELINE=1; else unset PZ_CHAIN_PIPELINE; fi
  PZ_CHAIN_PROFILE=1 timeout -k 10 150 python -u tools/replay_profile.py 65536 10000 > $O/replay_$mode.txt 2>&1 || { echo REPLAY_FAIL; tail $O/replay_$mode.txt; exit 11; }
  echo $mode; grep -E "process_serialized|phases" $O/replay_$mode.txt
done
