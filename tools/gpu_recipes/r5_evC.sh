# Round 5 evidence C: initialisation per stage, host-synchronisation bench A/B, then the chain / GEMM + Adam counters.
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_recipes/r5_init.sh ${1:-r5init} && bash $R/tools/gpu_recipes/r5_sync.sh ${2:-r5sync} && \
  bash $R/tools/gpu_recipes/r5_pmc.sh ${3:-r5pmc}
