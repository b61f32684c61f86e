# Round 6: D0 weight gradient + Adam in the short-K kernel (EngineConfig.fuse_d0_shortk) -- GPU tests, wide-table
# s/epoch A/B against the gradient-then-Adam schedule (alternating, same box), a kernel trace of each, Intrusion bench
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6x
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gemm_shortk.py tests/test_hip_engine.py tests/test_batched.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
W="python tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 4 --n-sample 10000"
for i in 1 2 3; do
  for v in "fuse_d0_shortk=1" "fuse_d0_shortk=0"; do
    timeout -k 10 200 $W --engine $v 2>&1 | grep '"mean_sec_per_epoch_after_first"' | sed "s/^/[$v] /" >> $OUT/wide.jsonl || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/wide.jsonl'):
    t, j = l.split('] ', 1); print(t + ']', json.loads(j)['mean_sec_per_epoch_after_first'])
"
cd /tmp
for v in "fuse_d0_shortk=1" "fuse_d0_shortk=0"; do
  (cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run -- python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 2 --n-sample 10000 --engine $v > $OUT/prof_$v.log 2>&1) || exit 1
  python3 $R/tools/step_breakdown.py $OUT/prof_$v/run_results.db --order > $OUT/step_$v.txt 2>&1 || true
  python3 $R/tools/prof_summary.py $OUT/prof_$v/run_results.db --shape > $OUT/prof_summary_$v.txt 2>&1 || true
  rm -rf $OUT/prof_$v
  echo "== $v"; head -14 $OUT/step_$v.txt
done
cd $R
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit 1
tail -1 $OUT/bench.log
