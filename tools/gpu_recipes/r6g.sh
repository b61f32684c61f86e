# Round 6: epoch-graph step time A/B (no profiler): multi_draw on/off x graph_unroll 8/16, alternating
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6g
mkdir -p $OUT
cd $R
for rep in 1 2; do
for cfg in "multi_draw=1 graph_unroll=8" "multi_draw=0 graph_unroll=8" "multi_draw=1 graph_unroll=16" "multi_draw=1 graph_unroll=40"; do
  set -- $cfg
  timeout -k 10 120 python3 tools/microbench.py --step-only --epochs-only --engine $1 --engine $2 2>&1 | grep "engine epoch" | sed "s/^/[$cfg] /" >> $OUT/ab.txt || exit 1
done
done
echo done
