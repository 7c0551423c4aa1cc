set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4af; mkdir -p $O
cd $R && AB=PZ_EPOCH_PACK AB_VALUES=copy,direct REPS=5 timeout -k 10 300 python3 tools/replay_profile.py 65536 10000 > $O/replay_ab.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay_ab.txt; exit 4; }
grep -E "^median" $O/replay_ab.txt; grep phases $O/replay_ab.txt | tail -2
echo DONE
