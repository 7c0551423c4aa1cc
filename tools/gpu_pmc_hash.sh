#!/bin/bash
# SQ stall counters for the hash kernel vs the register-only compression microbenchmark.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-pmch}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $C GRBM_GUI_ACTIVE --output-format csv -d $O/k -o k -- python3 $R/tools/pmc_workload.py > $O/k.log 2>&1 || { echo K FAILED; tail -5 $O/k.log; exit 20; }
timeout -s KILL 120 rocprofv3 --pmc $C GRBM_GUI_ACTIVE --output-format csv -d $O/m -o m -- $R/build/compress_rate > $O/m.log 2>&1 || { echo M FAILED; tail -5 $O/m.log; exit 21; }
echo ALLDONE
