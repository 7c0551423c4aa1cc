#!/bin/bash
# GPU session: microbench VALU rates, GPU parity tests, bench, rocprof kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
rocminfo | grep -m3 -E 'gfx|Marketing' > gpurun_out/device.txt 2>&1
nproc >> gpurun_out/device.txt; lscpu | grep 'Model name' >> gpurun_out/device.txt
timeout -k 10 120 ./build/valu_rates > gpurun_out/valu_rates.txt 2>&1 || exit 11
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || exit 12
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench.txt 2>&1 || exit 13
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_hash -o hash --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_hash.log 2>&1 || exit 14
echo ALLDONE
