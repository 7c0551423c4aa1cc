set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4g; mkdir -p $O
PYTEST_FILES="tests/test_native_gpu.py tests/test_wire_gpu.py tests/test_epoch_gpu.py" PYTEST_TIMEOUT=700 bash tools/gpu_session.sh r4g tests || exit 1
cd $R && VARIANTS=0,0/64,65536/64,0,0/64,65536/64 timeout -k 10 400 python3 tools/epoch_cold_ab.py > $O/cold_ab.txt 2>&1 || { echo COLD_FAIL; tail -5 $O/cold_ab.txt; exit 3; }
cat $O/cold_ab.txt
WIRE_GEOM=0,32768,65536,98304,0,32768,65536,98304 timeout -k 10 200 python3 tools/wire_probe.py 50 > $O/wire_geom.txt 2>&1 || { echo WIRE_FAIL; tail -5 $O/wire_geom.txt; exit 4; }
cat $O/wire_geom.txt
BENCH_ARGS="" BENCH_TIMEOUT=500 bash tools/gpu_session.sh r4g bench || exit 5
echo DONE
