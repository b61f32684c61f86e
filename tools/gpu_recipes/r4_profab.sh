# Same box: kernel traces of the captured step (microbench --step-only) and of bench.py, round-3 tree vs HEAD;
# critical-path summaries computed on the box, the databases deleted.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4profab}
mkdir -p $OUT
cd /tmp
for t in base head; do
  D=$R; [ $t = base ] && D=$R/_basetree
  (cd $D && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/step_$t -o run -- python3 tools/microbench.py --step-only > $OUT/step_$t.log 2>&1) || exit 1
  python3 $R/tools/step_breakdown.py $OUT/step_$t/run_results.db > $OUT/step_breakdown_$t.txt 2>&1 || exit 1
  (cd $D && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/bench_$t -o run -- python3 bench.py --steps 10 --warmup 3 > $OUT/bench_$t.log 2>&1) || exit 1
  python3 $R/tools/prof_summary.py $OUT/bench_$t/run_results.db > $OUT/bench_kernels_$t.txt 2>&1 || exit 1
  rm -rf $OUT/step_$t $OUT/bench_$t
done
echo done
