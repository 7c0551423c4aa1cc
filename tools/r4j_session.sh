set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4j; mkdir -p $O
for i in 1 2; do
  AB=PZ_VOTE_PATH AB_VALUES=segments,direct REPS=3 timeout -k 10 200 python3 tools/replay_profile.py 65536 10000 > $O/replay_new_$i.txt 2>&1 || { echo REPLAY_FAIL; tail -5 $O/replay_new_$i.txt; exit 4; }
  grep median $O/replay_new_$i.txt; grep phases $O/replay_new_$i.txt | tail -1
  PZ_PROBE_LIB=build/old/libprysm_hip.so AB=PZ_VOTE_PATH AB_VALUES=segments,packed REPS=3 timeout -k 10 200 python3 tools/replay_profile.py 65536 10000 > $O/replay_old_$i.txt 2>&1 || { echo REPLAY_OLD_FAIL; tail -5 $O/replay_old_$i.txt; exit 5; }
  grep median $O/replay_old_$i.txt | sed 's/^/old /'; grep phases $O/replay_old_$i.txt | tail -1
done
PZ_PROBE_LIB=build/prof/libprysm_hip.so timeout -k 10 200 python3 tools/walk_sampler.py 10000 6 50 > $O/walk_sampler.txt 2>&1 || { echo SAMPLER_FAIL; tail -5 $O/walk_sampler.txt; }
echo DONE
