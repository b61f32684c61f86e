# Round 6: short-K weight-gradient kernel (gemm_shortk_kernel) -- numerics tests, isolated dW0 timing, wide-table
# s/epoch A/B (gemm_shortk on / off, alternating) and a kernel trace of the wide step
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6u
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gemm_shortk.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 180 python3 tools/gout_probe.py > $OUT/probe.txt 2>&1 || { cat $OUT/probe.txt; exit 1; }
grep dW0 $OUT/probe.txt
W="python tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 3 --n-sample 10000"
for i in 1 2; do
  for v in "" "--tuning gemm_shortk=0"; do
    timeout -k 10 200 $W $v 2>&1 | grep '"mean_sec_per_epoch_after_first"' | sed "s/^/[$v] /" >> $OUT/wide.jsonl || exit 1
  done
done
cut -c1-200 $OUT/wide.jsonl
cd /tmp
(cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 2 --n-sample 10000 > $OUT/prof.log 2>&1) || exit 1
python3 $R/tools/prof_summary.py $OUT/prof/run_results.db --shape > $OUT/prof_summary.txt 2>&1 || true
python3 $R/tools/step_breakdown.py $OUT/prof/run_results.db --order > $OUT/step.txt 2>&1 || true
rm -rf $OUT/prof
head -20 $OUT/step.txt
