#!/bin/bash
# r2af: round evidence at the current build: GPU tests, smoke, bench, rocprof kernel stats, PMC passes.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_session.sh r2af || exit $?
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/r2af/smoke.txt 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/r2af/smoke.txt; exit 18; }
tail -1 gpurun_out/r2af/smoke.txt
bash tools/gpu_pmc.sh r2af_pmc || exit $?
cd $R && python3 tools/pmc_summary.py gpurun_out/r2af_pmc > gpurun_out/r2af/pmc_summary.json && python3 tools/pmc_summary.py gpurun_out/r2af_pmc_epoch1m > gpurun_out/r2af/pmc_summary_epoch1m.json && echo PMC_SUMMARY_OK
