# Round 6: same-box A/B of the short-K dW0 kernel on the wide table: wall-clock (3 x alternating, 4 epochs) and a
# kernel trace of each arm (critical path per kernel)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6v
mkdir -p $OUT
cd $R
W="python tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 4 --n-sample 10000"
for i in 1 2 3; do
  for v in "--tuning gemm_shortk=1" "--tuning gemm_shortk=0"; do
    timeout -k 10 200 $W $v 2>&1 | grep '"mean_sec_per_epoch_after_first"' | sed "s/^/[$v] /" >> $OUT/wide.jsonl || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/wide.jsonl'):
    t, j = l.split('] ', 1); print(t + ']', json.loads(j)['mean_sec_per_epoch_after_first'])
"
cd /tmp
for a in 1 0; do
  (cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof$a -o run -- python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 2 --n-sample 10000 --tuning gemm_shortk=$a > $OUT/prof$a.log 2>&1) || exit 1
  python3 $R/tools/step_breakdown.py $OUT/prof$a/run_results.db > $OUT/step$a.txt 2>&1 || true
  rm -rf $OUT/prof$a
  head -12 $OUT/step$a.txt
done
