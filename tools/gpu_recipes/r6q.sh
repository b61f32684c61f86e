# Round 6: wide table (100k x 512) s/epoch with this build (multi-step draw on / off) + kernel trace per launch
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6q
mkdir -p $OUT
cd $R
W="python tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 3 --n-sample 10000"
for i in 1 2; do
  for v in "" "--engine multi_draw=0"; do
    timeout -k 10 200 $W $v 2>&1 | grep '"mean_sec_per_epoch_after_first"' | sed "s/^/[$v] /" >> $OUT/wide.jsonl || exit 1
  done
done
cd /tmp
(cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 2 --n-sample 10000 > $OUT/prof.log 2>&1) || exit 1
python3 $R/tools/prof_summary.py $OUT/prof/run_results.db --shape > $OUT/prof_summary.txt 2>&1 || true
python3 $R/tools/step_breakdown.py $OUT/prof/run_results.db --order > $OUT/step.txt 2>&1 || true
rm -rf $OUT/prof
echo done
