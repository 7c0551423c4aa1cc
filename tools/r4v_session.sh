set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4v; mkdir -p $O
for cfg in "320 128 65536 4 1" "320 128 65536 16 1" "320 128 65536 4 0" "80 128 65536 4 1" "1280 128 65536 4 1" "320 128 65536 1 1"; do
  timeout -k 10 60 ./build/tally_probe $cfg >> $O/probe.txt 2>&1 || { echo PROBE_FAIL $cfg; tail -5 $O/probe.txt; exit 3; }
done
cat $O/probe.txt
echo DONE
