#!/bin/bash
# Wire encoder: timing + PMC passes (one counter group per run; no trace options with --pmc).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/${1:-wirepmc}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/wire_probe.py 50 > $O/probe.txt 2>&1 || { echo PROBE_FAIL; tail -20 $O/probe.txt; exit 12; }
cat $O/probe.txt
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $O/pmc$i -o p --output-format csv -- python3 tools/wire_probe.py 5 > $O/pmc$i.log 2>&1 || { echo PMC_FAIL $i; tail -5 $O/pmc$i.log; exit 13; }
done
echo done
