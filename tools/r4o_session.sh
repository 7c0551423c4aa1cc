# End-of-round evidence: the full GPU suite, smoke, the default bench line, a rocprofv3 kernel
# profile of a short bench run, and the N = 2 gloo rehearsal (two ranks sharing the GPU over the
# SHM communicator).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4o; mkdir -p $O
PYTEST_TIMEOUT=1000 bash tools/gpu_session.sh r4o tests,smoke,bench,prof || exit 1
cd $R && timeout -k 10 600 python3 bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --no-cpu-baseline > $O/gloo2.out 2> $O/gloo2.err || { echo GLOO_FAIL; tail -20 $O/gloo2.err; exit 2; }
grep '^{' $O/gloo2.out | tail -1 > $O/gloo2.json && python3 tools/bench_summary.py $O/gloo2.json
echo DONE
