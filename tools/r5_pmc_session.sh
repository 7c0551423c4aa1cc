#!/bin/bash
# Round 5 counter session: tools/gpu_pmc.sh over the main workload (bytes + SQ/GRBM passes:
# the hash kernel's VALU-busy fraction and clock) and the two cold epoch workloads (bytes);
# the N = 2 rehearsal (two ranks sharing the GPU over the shared-memory communicator); the
# XCD-grouped window pass (A/B).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd "$R" || exit 2
T=${1:-r5p}; O=$R/gpurun_out/$T; mkdir -p "$O"
bash tools/gpu_pmc.sh ${T}/pmc_main main full || exit 21
bash tools/gpu_pmc.sh ${T}/pmc_epoch1m_cold epoch1m_cold bytes || exit 22
bash tools/gpu_pmc.sh ${T}/pmc_epoch65k_cold epoch65k_cold bytes || exit 23
timeout -k 10 700 python -u bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 > "$O/n2.out" 2> "$O/n2.err" \
  || { echo N2_FAIL; tail -30 "$O/n2.err"; exit 24; }
grep '^{' "$O/n2.out" | tail -1 > "$O/bench_n2.json"; python3 tools/bench_summary.py "$O/bench_n2.json"
PZ_LIB=build/ab/libprysm_hip.so ABL=128,144 REPS=1 timeout -k 10 300 python -u tools/epoch_cold.py > "$O/epoch_abl_xcd.txt" 2>&1 \
  || { echo ABL_FAIL; tail -20 "$O/epoch_abl_xcd.txt"; exit 25; }
cut -c1-100 "$O/epoch_abl_xcd.txt"
echo SESSION_DONE
