# Round 5: wide table (100k x 512) knob A/B, 2 epochs each (mean s/epoch after the first), two passes:
# D0's weight gradient applying Adam in its own tiles (fuse_d0_adam, 64-tiles) instead of dW1 in the D Adam launch;
# 64x64 tiles for the G-out forward (WAVE_FILL_64); BatchNorm folded vs launches (default).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5widek}
mkdir -p $OUT
cd $R
W="python tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 2 --n-sample 10000"
for i in 1 2; do
  for v in "" "--engine fuse_d_adam=0 --engine fuse_d0_adam=1" "--plan WAVE_FILL_64=1"; do
    timeout -k 10 200 $W $v 2>&1 | grep '"mean_sec_per_epoch_after_first"' >> $OUT/wide.jsonl || exit 1
  done
done
echo done
