#!/bin/bash
# Round 5 counter session: tools/gpu_pmc.sh over the main workload (bytes + SQ/GRBM passes:
# VALU-busy fractions and clocks), the warm and cold epoch workloads (bytes), then the N = 2
# rehearsal (two ranks sharing the GPU over the shared-memory communicator).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd "$R" || exit 2
T=${1:-r5p}; O=$R/gpurun_out/$T; mkdir -p "$O"
bash tools/gpu_pmc.sh ${T}/pmc_main main full || exit 21
for w in epoch65k epoch1m epoch65k_cold epoch1m_cold; do
  bash tools/gpu_pmc.sh ${T}/pmc_$w $w bytes || exit 22
done
timeout -k 10 700 python -u bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 > "$O/n2.out" 2> "$O/n2.err" \
  || { echo N2_FAIL; tail -30 "$O/n2.err"; exit 24; }
grep '^{' "$O/n2.out" | tail -1 > "$O/bench_n2.json"; python3 tools/bench_summary.py "$O/bench_n2.json"
echo SESSION_DONE
