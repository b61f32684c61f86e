# Round 6: short-K dW0 output store policy (gemm_shortk_store 0 plain / 1 non-temporal / 2 write-through) vs the tile
# GEMM (gemm_shortk=0) on the wide table -- wall-clock alternating and a kernel trace per arm
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6w
mkdir -p $OUT
cd $R
W="python tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 4 --n-sample 10000"
for i in 1 2; do
  for v in "gemm_shortk_store=0" "gemm_shortk_store=1" "gemm_shortk_store=2" "gemm_shortk=0"; do
    timeout -k 10 200 $W --tuning $v 2>&1 | grep '"mean_sec_per_epoch_after_first"' | sed "s/^/[$v] /" >> $OUT/wide.jsonl || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/wide.jsonl'):
    t, j = l.split('] ', 1); print(t + ']', json.loads(j)['mean_sec_per_epoch_after_first'])
"
cd /tmp
for v in "gemm_shortk_store=1" "gemm_shortk_store=2"; do
  (cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run -- python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 2 --n-sample 10000 --tuning $v > $OUT/prof_$v.log 2>&1) || exit 1
  python3 $R/tools/step_breakdown.py $OUT/prof_$v/run_results.db > $OUT/step_$v.txt 2>&1 || true
  rm -rf $OUT/prof_$v
  echo "== $v"; head -10 $OUT/step_$v.txt
done
