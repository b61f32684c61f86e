# Round 5 evidence D: stalls after the formatter warm-up (r5_stall.sh), then init / sync / counters (r5_evC.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_recipes/r5_stall.sh r5stall && bash $R/tools/gpu_recipes/r5_evC.sh r5init r5sync r5pmc
