#!/bin/bash
# Round 6 end-of-round evidence on the final tree, in two calls:
#   tools/r6_final_session.sh TAG a   GPU suite, A/B suite, smoke, bench line, rocprof kernel stats
#   tools/r6_final_session.sh TAG b   counter passes (main: bytes + SQ/GRBM; the four epoch
#                                     workloads: bytes), then the N = 2 gloo rehearsal
# Output under gpurun_out/TAG/; copy what is judged into profiles/r06/.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd "$R" || exit 2
T=${1:?tag}; PART=${2:-a}; O=$R/gpurun_out/$T; mkdir -p "$O"
if [ "$PART" = a ]; then
  BENCH_ARGS="${BENCH_ARGS:---steps 20 --warmup 5}" bash tools/gpu_session.sh "$T" tests,abtests,smoke,bench,prof || exit $?
else
  bash tools/gpu_pmc.sh ${T}/pmc_main main full || exit 21
  for w in epoch65k_cold epoch1m_cold epoch65k epoch1m; do
    bash tools/gpu_pmc.sh ${T}/pmc_$w $w bytes || exit 22
  done
  timeout -k 10 700 python -u bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 > "$O/n2.out" 2> "$O/n2.err" \
    || { echo N2_FAIL; tail -30 "$O/n2.err"; exit 24; }
  grep '^{' "$O/n2.out" | tail -1 > "$O/bench_n2.json"; python3 tools/bench_summary.py "$O/bench_n2.json"
fi
echo SESSION_DONE
