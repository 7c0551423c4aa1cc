set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r3n; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_replay.py tests/test_votes_gpu.py tests/test_native_gpu.py tests/test_epoch_gpu.py -m gpu > $O/tests.txt 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.txt; exit 12; }
tail -2 $O/tests.txt
for k in 1 2 3; do
  timeout -k 10 150 python -u tools/replay_profile.py 65536 10000 > $O/replay_$k.txt 2>&1 || { echo REPLAY_FAIL; tail $O/replay_$k.txt; exit 11; }
  grep -E "process_serialized|phases" $O/replay_$k.txt
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-replay --no-wire --no-attcheck --no-single-process-leg > $O/bench_epoch.txt 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench_epoch.txt; exit 14; }
python3 tools/show_epoch.py $O/bench_epoch.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o replay -- python3 -u $R/tools/replay_profile.py 65536 2000 > $O/trace.txt 2>&1 || { echo TRACE_FAIL; tail -20 $O/trace.txt; exit 13; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/single -o single -- python3 -u $R/tools/pmc_workload.py epoch_single > $O/single.txt 2>&1 || { echo SINGLE_FAIL; tail -20 $O/single.txt; exit 15; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cold -o cold -- python3 -u $R/tools/pmc_workload.py epoch65k_cold > $O/cold.txt 2>&1 || { echo COLD_FAIL; tail -20 $O/cold.txt; exit 16; }
