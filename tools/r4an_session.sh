# A/B: the streaming pass with the last bitfield in LDS on the u32 offsets (variant 1 << 22)
# against the product's quad kernel (0), cold; the forms test first.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4an; mkdir -p $O
PYTEST_FILES="tests/test_native_gpu.py" PYTEST_K="bal32_forms" PYTEST_TIMEOUT=600 bash tools/gpu_session.sh r4an tests || exit 1
cd $R && VARIANTS=0,4194304,0,4194304 timeout -k 10 300 python3 tools/epoch_cold_ab.py > $O/cold_ab.txt 2>&1 || { echo COLD_FAIL; tail -5 $O/cold_ab.txt; exit 3; }
sed 's/  frac(layout).*//' $O/cold_ab.txt
echo DONE
