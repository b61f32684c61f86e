# Round 5 evidence B: 8 emulated clients (queues / batched, r5_kq.sh) then the wide-table knob A/B (r5_widek.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_recipes/r5_kq.sh ${1:-r5kq} && bash $R/tools/gpu_recipes/r5_widek.sh ${2:-r5widek}
