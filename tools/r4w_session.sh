set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4w; mkdir -p $O
run() { echo "== $*" >> $O/probe.txt; timeout -k 10 60 "$@" >> $O/probe.txt 2>&1 || { echo PROBE_FAIL "$@"; tail -5 $O/probe.txt; exit 3; }; }
run ./build/tally_probe 320 128 65536 4 1 1 0
run ./build/tally_probe 320 128 65536 4 1 1 60
run ./build/tally_probe 320 128 65536 4 1 0 60
run ./build/tally_probe 320 128 65536 4 1 0 0
run ./build/tally_probe_wt 320 128 65536 4 1 1 60
run ./build/tally_probe_wt 320 128 65536 4 1 0 60
run ./build/tally_probe 320 128 65536 8 1 1 60
cat $O/probe.txt | grep -v "^totals"
echo DONE
