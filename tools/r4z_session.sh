set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4z; mkdir -p $O
for G in 1 0; do
  echo "== PZ_VOTE_GROUPS=$G" >> $O/trace.txt
  PZ_VOTE_GROUPS=$G timeout -k 10 200 python3 tools/vote_trace.py >> $O/trace.txt 2>&1 || { echo TRACE_FAIL; tail -5 $O/trace.txt; exit 3; }
done
cat $O/trace.txt
echo DONE
