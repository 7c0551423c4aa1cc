#!/bin/bash
# Device proto3 encoder: its GPU tests, the replay tests (state roots now use it), the bench's
# wire leg alone, and a rocprofv3 kernel-stats pass of the same command.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/${1:-wire}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_wire_gpu.py tests/test_replay.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_wire.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_wire.txt; exit 12; }
tail -3 $O/pytest_wire.txt
timeout -k 10 200 python -u bench.py --no-epoch --no-replay --steps 20 --warmup 3 --records 65536 --no-cpu-baseline > $O/bench_wire.json 2> $O/bench_wire.err || { echo BENCH_FAIL; tail -20 $O/bench_wire.err; exit 13; }
python -c "import json;d=json.loads(open('$O/bench_wire.json').read().strip().splitlines()[-1]);print(json.dumps(d['wire'],indent=1))"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o wire --output-format csv -- python3 bench.py --no-epoch --no-replay --steps 20 --warmup 3 --records 65536 --no-cpu-baseline > $O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof.log; exit 14; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'grep -E "Name|wire" {}'
