# Round 6: wide activation with the fused slerp's condition tail in registers (act_tail_reg) -- engine tests (wide
# layouts), wide s/epoch A/B alternating on one box, kernel trace of the default arm
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6af
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_hip_engine.py tests/test_hip_ops.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
W="python tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 4 --n-sample 10000"
for i in 1 2 3; do
  for v in "act_tail_reg=1" "act_tail_reg=0"; do
    timeout -k 10 200 $W --tuning $v 2>&1 | grep '"mean_sec_per_epoch_after_first"' | sed "s/^/[$v] /" >> $OUT/wide.jsonl || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/wide.jsonl'):
    t, j = l.split('] ', 1); print(t + ']', json.loads(j)['mean_sec_per_epoch_after_first'])
"
cd /tmp
for v in "act_tail_reg=1" "act_tail_reg=0"; do
  (cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 2 --n-sample 10000 --tuning $v > $OUT/prof.log 2>&1) || exit 1
  python3 $R/tools/step_breakdown.py $OUT/prof/run_results.db > $OUT/step_$v.txt 2>&1 || true
  rm -rf $OUT/prof
  echo "== $v"; grep "activate_rowreg" $OUT/step_$v.txt | head -2
done
