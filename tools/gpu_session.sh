#!/bin/bash
# One GPU session: parity tests, bench, rocprof kernel stats.  Usage: tools/gpu_session.sh TAG [bench args]
set -o pipefail
TAG=${1:-run}; shift
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.txt; exit 12; }
tail -3 $O/pytest_gpu.txt
timeout -k 10 400 python -u bench.py "$@" > $O/bench.txt 2>&1 || { echo BENCH_FAIL; tail -30 $O/bench.txt; exit 13; }
tail -1 $O/bench.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/$O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $R/$O/prof.log; exit 14; }
echo ALLDONE
