# One-client step knob sweep (microbench --step-only, two passes) + wide-table store knob.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4knobs1}
mkdir -p $OUT
cd $R
for pass in 1 2; do
  for v in "" "--tuning bn_cols=4" "--tuning bn_cols=16" "--tuning gemm_store_wt=1" "--tuning gemm_xcd_remap=0" "--tuning gemm_xcd_remap=2" "--tuning adam_store=0"; do
    echo "== $v" >> $OUT/step.txt
    timeout -k 10 120 python tools/microbench.py --step-only $v 2>&1 | grep "full step" >> $OUT/step.txt || exit 1
  done
done
W="python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 2 --n-sample 10000"
for v in "" "--tuning gemm_store_wt=1"; do
  timeout -k 10 200 $W $v 2>&1 | grep '"mean_sec_per_epoch_after_first"' >> $OUT/wide.jsonl || exit 1
done
echo done
