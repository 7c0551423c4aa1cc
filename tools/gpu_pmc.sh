#!/bin/bash
# rocprofv3 counter passes over ONE workload of tools/pmc_workload.py (one counter group per
# run, each under its own kill timeout), written to gpurun_out/OUT/<pass>/.
#   tools/gpu_pmc.sh OUT WORKLOAD [bytes|full]
# bytes: FETCH_SIZE and WRITE_SIZE passes (HBM traffic); full: also SQ and GRBM passes.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:?out}; W=${2:-main}; MODE=${3:-bytes}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o $name -- python3 $R/tools/pmc_workload.py $W > $O/$name.log 2>&1 || { echo "PASS $W/$name FAILED"; tail -5 $O/$name.log; exit 20; }
  echo "pass $W/$name ok"
}
run fetch FETCH_SIZE
run write WRITE_SIZE
if [ "$MODE" = full ]; then
  run sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT
  run grbm GRBM_GUI_ACTIVE GRBM_COUNT
fi
python3 $R/tools/pmc_summary.py $O > $O/summary.json && echo "summary $O/summary.json"
