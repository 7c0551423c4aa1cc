set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4aq; mkdir -p $O
bash tools/gpu_session.sh r4aq bench || exit 1
python3 -c "import json; r=json.load(open('$O/bench.json'))['replay']; print(r['value'], r['replay_walls_ms'], r['timing'])"
echo DONE
