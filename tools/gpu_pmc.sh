#!/bin/bash
# rocprofv3 counter passes (one counter group per run, each under its own kill timeout).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-pmc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # name, counters...  (PMC_ARGS: workload mode, e.g. epoch_1m; PMC_DIR: output dir)
  local name=$1; shift
  local d=${PMC_DIR:-$O}; mkdir -p $d
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $d/$name -o $name -- python3 $R/tools/pmc_workload.py $PMC_ARGS > $d/$name.log 2>&1 || { echo "PASS $name FAILED"; tail -5 $d/$name.log; exit 20; }
  echo "pass $name ok"
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT
run grbm GRBM_GUI_ACTIVE GRBM_COUNT
# the configs[3]-sized epoch (1M validators x 16 instances) in its own workload and summary
PMC_ARGS=epoch_1m PMC_DIR=${O}_epoch1m run fetch FETCH_SIZE
PMC_ARGS=epoch_1m PMC_DIR=${O}_epoch1m run write WRITE_SIZE
echo ALLDONE
