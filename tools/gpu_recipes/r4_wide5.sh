# Sampler 16-B one-hot stores + chunk-split gradient-penalty scale: tests, wide A/B, Intrusion step.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4wide5}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_ops.py tests/test_hip_engine.py tests/test_gpu_engine.py -k "gp_scale or sample or wide or onehot or autograd or batch" > $OUT/pytest.log 2>&1 || exit 1
W="python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 2 --n-sample 10000"
for v in "--tuning gp_split=0" "" "--tuning gp_split=0" ""; do
  timeout -k 10 200 $W $v 2>&1 | grep '"mean_sec_per_epoch_after_first"' >> $OUT/wide.jsonl || exit 1
done
for i in 1 2; do
  (cd $R/_basetree && timeout -k 10 150 python tools/microbench.py --step-only >> $OUT/base_step.txt 2>&1) || exit 1
  (cd $R && timeout -k 10 150 python tools/microbench.py --step-only >> $OUT/head_step.txt 2>&1) || exit 1
done
echo done
