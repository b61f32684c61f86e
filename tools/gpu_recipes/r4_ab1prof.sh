# Same box: per-kernel critical path of the one-client step, round-3 tree (_basetree) vs HEAD.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4ab1prof}
mkdir -p $OUT
for t in base head; do
  D=$R; [ $t = base ] && D=$R/_basetree
  (cd $D && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_$t -o run -- python3 tools/gpu_probe.py --backend hip --steps 40 > $OUT/prof_$t.log 2>&1) || break
  python3 $R/tools/step_breakdown.py $OUT/prof_$t/run_results.db > $OUT/step_$t.txt 2>&1
  rm -f $OUT/prof_$t/run_results.db
done
echo "exit $?"
