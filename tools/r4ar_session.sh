set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4ar; mkdir -p $O
PZ_PROBE_LIB=build/prof/libprysm_hip.so timeout -k 10 200 python3 tools/walk_sampler.py 10000 6 50 > $O/walk_sampler.txt 2>&1 || { echo SAMPLER_FAIL; tail -5 $O/walk_sampler.txt; exit 3; }
sed -n '/engine line/,$p' $O/walk_sampler.txt | head -40
echo DONE
