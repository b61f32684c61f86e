# Round 5 evidence E: chain prefetch step A/B (r5_chain.sh), the one-rank RCCL round (r5_sync2.sh), then 8 emulated
# clients and the wide knobs (r5_evB.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_recipes/r5_chain.sh r5chain && bash $R/tools/gpu_recipes/r5_sync2.sh r5sync2 && \
  bash $R/tools/gpu_recipes/r5_evB.sh r5kq r5widek
