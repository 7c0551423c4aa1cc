# End-of-round evidence (full GPU suite, smoke, the default bench line, a rocprofv3 kernel
# profile of a short bench run, the N = 2 gloo rehearsal), then two experiments: the two-piece
# epoch A/B and the replay's transition timeline.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4q; mkdir -p $O
PYTEST_K="not 2097152" PYTEST_TIMEOUT=900 bash tools/gpu_session.sh r4q tests,smoke,bench,prof || exit 1
cd $R && timeout -k 10 420 python3 bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --no-cpu-baseline > $O/gloo2.out 2> $O/gloo2.err || { echo GLOO_FAIL; tail -20 $O/gloo2.err; exit 2; }
grep '^{' $O/gloo2.out | tail -1 > $O/gloo2.json && python3 tools/bench_summary.py $O/gloo2.json
echo EVIDENCE_DONE
timeout -k 10 200 python -u -m pytest tests/test_native_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "2097152" > $O/pytest_q2.txt 2>&1 || { echo Q2_TEST_FAIL; tail -20 $O/pytest_q2.txt; exit 5; }
tail -1 $O/pytest_q2.txt
cd $R && VARIANTS=0,2097152,0,2097152 timeout -k 10 200 python3 tools/epoch_cold_ab.py > $O/cold_ab.txt 2>&1 || { echo COLD_FAIL; tail -5 $O/cold_ab.txt; exit 3; }
sed 's/  frac(layout).*//' $O/cold_ab.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tl -o run --output-format csv -- python3 $R/tools/replay_timeline.py $O/timeline.json > $O/tl.log 2>&1 || { echo TL_FAIL; tail -5 $O/tl.log; exit 4; }
tail -2 $O/tl.log
echo DONE
