# Wide 100k x 512: GEMM ordering / pairing knobs (2 epochs each, sec/epoch of epoch 1)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4wide3}
mkdir -p $OUT
W="python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 2 --n-sample 10000"
for v in "" "--tuning gemm_xcd_remap=2" "--tuning gemm_pairs=0" "--tuning gemm_xcd_remap=2 --tuning gemm_pairs=0" "--tuning gemm_xcd_remap=0"; do
  timeout -k 10 200 $W $v 2>&1 | grep '"mean_sec_per_epoch_after_first"' >> $OUT/wide3.jsonl || break
done
echo "exit $?"
