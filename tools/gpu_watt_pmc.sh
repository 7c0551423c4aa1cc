#!/bin/bash
# Counter passes over the attestation encoder probe (tools/wire_att_probe.py, 10 launches).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-watt_pmc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o $name -- python3 $R/tools/wire_att_probe.py 10 > $O/$name.log 2>&1 || { echo "PASS $name FAILED"; tail -5 $O/$name.log; exit 20; }
  echo "pass $name ok"
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run sq2 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR
run fetch FETCH_SIZE
run write WRITE_SIZE
echo ALLDONE
