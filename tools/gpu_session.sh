#!/bin/bash
# One parameterised GPU session on the gpurun box (replaces the per-run scripts of rounds 1-2).
#
#   tools/gpu_session.sh TAG STEPS
#
# STEPS is a comma-separated list, run in order; the first failing step ends the session:
#   tests      pytest -m gpu (PYTEST_K: a -k expression; PYTEST_FILES: test paths)
#   abtests    pytest -m ab (the A/B library's forms)
#   smoke      __graft_entry__.smoke()
#   bench      python bench.py $BENCH_ARGS               -> $O/bench.json (the JSON line)
#   prof       rocprofv3 --kernel-trace --stats of a short bench run -> $O/prof/
#   pmc:W      counter passes (bytes) over tools/pmc_workload.py's workload W -> $O/pmc_W/summary.json
#   pmcfull:W  the same plus the SQ and GRBM passes
#   tool:X     python tools/X.py $TOOL_ARGS              -> $O/X.txt
# Output goes to gpurun_out/TAG/; copy what is to be judged into profiles/rNN/.
set -o pipefail
TAG=${1:?tag}; STEPS=${2:-tests,bench}
R=$GRAFT_REPO_ROOT; cd "$R" || exit 2
O=$R/gpurun_out/$TAG
mkdir -p "$O"
run_tests() {
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -v --timeout 120 \
    --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$O/pytest_gpu.txt" 2>&1 \
    || { echo "TESTS_FAIL"; tail -40 "$O/pytest_gpu.txt"; exit 12; }
  tail -2 "$O/pytest_gpu.txt"
}
run_abtests() {  # the A/B forms against build/ab/libprysm_hip.so (tests/conftest.py: -m ab)
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m ab -x -v --timeout 120 --timeout-method thread \
    > "$O/pytest_ab.txt" 2>&1 || { echo "AB_TESTS_FAIL"; tail -40 "$O/pytest_ab.txt"; exit 18; }
  tail -2 "$O/pytest_ab.txt"
}
run_smoke() {
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > "$O/smoke.txt" 2>&1 \
    || { echo "SMOKE_FAIL"; tail -20 "$O/smoke.txt"; exit 13; }
  tail -1 "$O/smoke.txt"
}
run_bench() {
  timeout -k 10 ${BENCH_TIMEOUT:-500} python -u bench.py $BENCH_ARGS > "$O/bench.out" 2> "$O/bench.err" \
    || { echo "BENCH_FAIL"; tail -30 "$O/bench.err"; exit 14; }
  grep '^{' "$O/bench.out" | tail -1 > "$O/bench.json"
  python3 tools/bench_summary.py "$O/bench.json"
}
run_prof() {
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run \
    --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline ${PROF_ARGS} \
    > "$O/prof.log" 2>&1) || { echo "PROF_FAIL"; tail -20 "$O/prof.log"; exit 15; }
  echo "prof ok"
}
run_pmc() {  # workload, mode
  bash tools/gpu_pmc.sh "$TAG/pmc_$1" "$1" "$2" || exit 16
}
run_tool() {
  timeout -k 10 ${TOOL_TIMEOUT:-300} python -u "tools/$1.py" $TOOL_ARGS > "$O/$1.txt" 2>&1 \
    || { echo "TOOL_FAIL $1"; tail -30 "$O/$1.txt"; exit 17; }
  tail -${TOOL_TAIL:-30} "$O/$1.txt"
}
IFS=, read -ra LIST <<< "$STEPS"
for s in "${LIST[@]}"; do
  case $s in
    tests) run_tests ;;
    abtests) run_abtests ;;
    smoke) run_smoke ;;
    bench) run_bench ;;
    prof) run_prof ;;
    pmc:*) run_pmc "${s#pmc:}" bytes ;;
    pmcfull:*) run_pmc "${s#pmcfull:}" full ;;
    tool:*) run_tool "${s#tool:}" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "SESSION_DONE $TAG"
