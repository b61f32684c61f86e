# Same-box A/B: the round-2 tree (git worktree _r2tree at f0ac677, built in-tree) against HEAD -- the full
# captured step (microbench --step-only) and bench.py rounds, alternating.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3r2}
mkdir -p $O
R=$GRAFT_REPO_ROOT
for i in 1 2; do
  (cd $R/_r2tree && timeout -k 10 200 python tools/microbench.py --step-only > $O/r2_step_$i.txt 2>&1) && \
  (cd $R && timeout -k 10 200 python tools/microbench.py --step-only > $O/head_step_$i.txt 2>&1) && \
  (cd $R/_r2tree && timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/r2_bench_$i.log 2>&1) && \
  (cd $R && timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/head_bench_$i.log 2>&1) || exit 1
done
echo "exit 0"
