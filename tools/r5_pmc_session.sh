#!/bin/bash
# Round 5 counter session: tools/gpu_pmc.sh over the main workload (bytes + SQ/GRBM passes:
# the hash kernel's VALU-busy fraction and clock) and the two cold epoch workloads (bytes).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd "$R" || exit 2
T=${1:-r5p}
bash tools/gpu_pmc.sh ${T}_main main full || exit 21
bash tools/gpu_pmc.sh ${T}_epoch1m_cold epoch1m_cold bytes || exit 22
bash tools/gpu_pmc.sh ${T}_epoch65k_cold epoch65k_cold bytes || exit 23
