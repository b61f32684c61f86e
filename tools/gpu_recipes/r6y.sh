# Round 6: fused short-K Adam with float4 operands (operand-swapped MFMA) -- tests, wide A/B, trace of the fused arm
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6y
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gemm_shortk.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
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
v="fuse_d0_shortk=1"
(cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 2 --n-sample 10000 --engine $v > $OUT/prof.log 2>&1) || exit 1
python3 $R/tools/step_breakdown.py $OUT/prof/run_results.db > $OUT/step.txt 2>&1 || true
rm -rf $OUT/prof
head -14 $OUT/step.txt
