#!/bin/bash
# Round-end style evidence in one call: GPU tests, bench, rocprof kernel stats, PMC passes.
set -o pipefail
TAG=${1:-full}
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_session.sh $TAG || exit $?
bash tools/gpu_pmc.sh ${TAG}_pmc || exit $?
cd $R && python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc > gpurun_out/${TAG}_pmc_summary.json && python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc_epoch1m > gpurun_out/${TAG}_pmc_summary_epoch1m.json && echo PMC_SUMMARY_OK
