# 8-client batched step: D0 weight-gradient tile A/B (the dW0 || R0 pair is 102 of 701 us at 8 clients).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3k}
mkdir -p $OUT
P="timeout -k 10 200 python tools/batched_probe.py --ks 8 --skip-plain --plan on --reps 4"
$P > $OUT/k8_default.log 2>&1 && \
$P --engine dw0_tile=128 > $OUT/k8_dw0_128.log 2>&1 && \
$P --engine dw0_tile=32 > $OUT/k8_dw0_32.log 2>&1
echo "exit $?"
