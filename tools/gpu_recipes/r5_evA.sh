# Round 5 evidence A: initialisation per stage (r5_init.sh) then the host-synchronisation bench A/B (r5_sync.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_recipes/r5_init.sh ${1:-r5init} && bash $R/tools/gpu_recipes/r5_sync.sh ${2:-r5sync}
