set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4h; mkdir -p $O
B=1048576
cd $R && VARIANTS=0,$((B+1)),$((B+2)),$((B+4)),$((B+8)),$((B+3)),$((B+7)),$((B+15)),0 timeout -k 10 400 python3 tools/epoch_cold_ab.py > $O/cold_abl.txt 2>&1 || { echo COLD_FAIL; tail -5 $O/cold_abl.txt; exit 3; }
cat $O/cold_abl.txt
cd /tmp && export TMPDIR=/tmp
VARIANTS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_epoch -o run --output-format csv -- python3 $R/tools/epoch_cold_ab.py > $O/prof_epoch.log 2>&1 || { echo PROF_EPOCH_FAIL; tail -5 $O/prof_epoch.log; exit 4; }
REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_replay -o run --output-format csv -- python3 $R/tools/replay_profile.py 65536 10000 > $O/prof_replay.log 2>&1 || { echo PROF_REPLAY_FAIL; tail -5 $O/prof_replay.log; exit 5; }
echo DONE
