# End-of-round evidence (final tree) (full GPU suite, smoke, the default bench line,
# a rocprofv3 kernel profile of a short bench run, the N = 2 gloo rehearsal), then the replay's
# transition timeline and the in-kernel tally trace.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4ap; mkdir -p $O
PYTEST_TIMEOUT=900 bash tools/gpu_session.sh r4ap tests,smoke,bench,prof || exit 1
cd $R && timeout -k 10 420 python3 bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --no-cpu-baseline > $O/gloo2.out 2> $O/gloo2.err || { echo GLOO_FAIL; tail -20 $O/gloo2.err; exit 2; }
grep '^{' $O/gloo2.out | tail -1 > $O/gloo2.json && python3 tools/bench_summary.py $O/gloo2.json
echo EVIDENCE_DONE
timeout -k 10 200 python3 tools/vote_trace.py > $O/vote_trace.txt 2>&1 || { echo TRACE_FAIL; tail -5 $O/vote_trace.txt; exit 3; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tl -o run --output-format csv -- python3 $R/tools/replay_timeline.py $O/timeline.json > $O/tl.log 2>&1 || { echo TL_FAIL; tail -5 $O/tl.log; exit 4; }
tail -2 $O/tl.log
echo DONE
