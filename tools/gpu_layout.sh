#!/bin/bash
# Committee-order vs index-order epoch layout: native epoch parity tests, then the epoch legs
# of the bench in both layouts (same box).  Usage: tools/gpu_layout.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/${1:-layout}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_native_gpu.py tests/test_epoch_gpu.py tests/test_multirank.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.txt; exit 12; }
tail -1 $O/pytest_gpu.txt
for L in auto twopass index auto; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-replay --no-wire --no-attcheck --epoch-layout $L > $O/bench_$L.txt 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench_$L.txt; exit 13; }
  tail -1 $O/bench_$L.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); [print('$L', k, d[k]['value'], d[k]['ms_per_step'], d[k]['roofline']['frac'], d[k]['config'].get('layout'), d[k]['parity']) for k in ('epoch', 'epoch_1m_single_gpu') if k in d]"
done
