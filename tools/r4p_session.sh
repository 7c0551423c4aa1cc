set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4p; mkdir -p $O
PYTEST_FILES="tests/test_native_gpu.py" PYTEST_K="bal32" PYTEST_TIMEOUT=300 bash tools/gpu_session.sh r4p tests || exit 1
cd $R && VARIANTS=0,2097152,0,2097152 timeout -k 10 300 python3 tools/epoch_cold_ab.py > $O/cold_ab.txt 2>&1 || { echo COLD_FAIL; tail -5 $O/cold_ab.txt; exit 3; }
sed 's/  frac(layout).*//' $O/cold_ab.txt
echo DONE
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/tl -o run --output-format csv -- python3 $R/tools/replay_timeline.py $O/timeline.json > $O/tl.log 2>&1 || { echo TL_FAIL; tail -5 $O/tl.log; exit 4; }
tail -2 $O/tl.log
echo DONE2
