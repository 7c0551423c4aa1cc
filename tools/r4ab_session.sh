set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4ab; mkdir -p $O
bash tools/gpu_session.sh r4ab bench || exit 1
PZ_PROBE_LIB=build/prof/libprysm_hip.so timeout -k 10 200 python3 tools/walk_sampler.py 10000 6 50 > $O/walk_sampler.txt 2>&1 || { echo SAMPLER_FAIL; tail -5 $O/walk_sampler.txt; exit 3; }
head -60 $O/walk_sampler.txt
echo DONE
