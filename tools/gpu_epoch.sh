#!/bin/bash
# Epoch-path GPU iteration: epoch/multirank/replay parity tests, then the bench (epoch leg).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/${1:-epoch}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_epoch_gpu.py tests/test_multirank.py tests/test_replay.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.txt; exit 12; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python -u bench.py --no-replay --no-cpu-baseline > $O/bench.txt 2>&1 || { echo BENCH_FAIL; tail -30 $O/bench.txt; exit 13; }
tail -1 $O/bench.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-replay > $R/$O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $R/$O/prof.log; exit 14; }
grep -E "epoch|Name" $R/$O/prof/run_kernel_stats.csv | cut -c1-150
