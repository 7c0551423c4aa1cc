#!/bin/bash
# Per-kernel device time of the epoch legs in each layout (rocprofv3 kernel trace + stats).
# Usage: tools/gpu_layout_prof.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-lprof}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for L in auto twopass index; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$L -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-replay --no-wire --no-attcheck --epoch-layout $L > $O/$L.log 2>&1 || { echo PROF_FAIL $L; tail -20 $O/$L.log; exit 14; }
  S=$(find $O/$L -name 'run_kernel_stats.csv' | head -1)
  echo "== $L"; python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$S')))
for r in rows:
    if 'epoch' in r['Name']: print('%-40s calls %6s avg_us %9.2f' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3))
"
done
