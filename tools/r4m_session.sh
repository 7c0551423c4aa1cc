set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4m; mkdir -p $O
for w in epoch1m epoch65k epoch1m_cold epoch65k_cold epoch_single main; do
  bash tools/gpu_pmc.sh r4m/pmc_$w $w bytes || exit 2
done
echo DONE
