# Batched 8-client step: EngineConfig knob A/B (fusions designed for the one-client latency regime).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3o}
mkdir -p $OUT
for v in "" "--engine chain_d1=0" "--engine fuse_d_adam=0" "--engine chain_d1=0 --engine fuse_d_adam=0" "--engine fuse_g_adam=0" "--engine paired=0" "--engine onehot=0" "--engine g_wt=0"; do
  timeout -k 10 200 python tools/batched_probe.py --ks 8 --reps 4 --skip-plain $v > $OUT/tmp.log 2>&1 || exit 1
  grep '"batched"' $OUT/tmp.log >> $OUT/knobs.txt
done
echo ok
