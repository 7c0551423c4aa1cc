#!/bin/bash
# r2ah: round evidence at the current build: GPU tests, smoke, bench, rocprof kernel stats, PMC passes.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_session.sh r2ah || exit $?
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/r2ah/smoke.txt 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/r2ah/smoke.txt; exit 18; }
tail -1 gpurun_out/r2ah/smoke.txt
bash tools/gpu_pmc.sh r2ah_pmc || exit $?
cd $R && python3 tools/pmc_summary.py gpurun_out/r2ah_pmc > gpurun_out/r2ah/pmc_summary.json && python3 tools/pmc_summary.py gpurun_out/r2ah_pmc_epoch1m > gpurun_out/r2ah/pmc_summary_epoch1m.json && echo PMC_SUMMARY_OK
