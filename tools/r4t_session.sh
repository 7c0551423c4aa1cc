set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4t; mkdir -p $O
timeout -k 10 60 ./build/bar_probe > $O/bar_probe.txt 2>&1; echo "bar_probe rc=$?"; cat $O/bar_probe.txt
cd /tmp && export TMPDIR=/tmp
for P in segments direct; do
  PZ_VOTE_PATH=$P timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tl_$P -o run --output-format csv -- python3 $R/tools/replay_timeline.py $O/timeline_$P.json > $O/tl_$P.log 2>&1 || { echo TL_FAIL $P; tail -5 $O/tl_$P.log; exit 5; }
  tail -1 $O/tl_$P.log
done
echo DONE
