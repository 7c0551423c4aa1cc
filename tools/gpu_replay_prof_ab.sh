#!/bin/bash
# Kernel stats of tools/replay_profile.py for this build and build/ab/libprysm_hip_old.so.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-rpprof}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/new -o run --output-format csv -- python3 $R/tools/replay_profile.py 65536 10000 > $O/new.txt 2>&1 || { echo NEW_FAIL; tail -20 $O/new.txt; exit 13; }
PZ_PROBE_LIB=$R/build/ab/libprysm_hip_old.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/old -o run --output-format csv -- python3 $R/tools/replay_profile.py 65536 10000 > $O/old.txt 2>&1 || { echo OLD_FAIL; tail -20 $O/old.txt; exit 14; }
for v in new old; do
  echo "== $v"; grep process_serialized $O/$v.txt
  S=$(find $O/$v -name 'run_kernel_stats.csv' | head -1)
  python3 -c "
import csv
for r in list(csv.DictReader(open('$S')))[:12]: print('%-34s calls %7s total_ms %8.2f avg_us %8.2f' % (r['Name'][:34], r['Calls'], float(r['TotalDurationNs'])/1e6, float(r['AverageNs'])/1e3))
"
done
