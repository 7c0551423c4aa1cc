set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4r; mkdir -p $O
timeout -k 10 120 ./build/bar_probe > $O/bar_probe.txt 2>&1; echo "rc=$?" >> $O/bar_probe.txt
cat $O/bar_probe.txt
echo DONE
