# Same box, 8 batched clients: defaults vs each new default turned off, and 2 stream groups x 4; two passes.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4b8ab}
mkdir -p $OUT
P="python tools/batched_probe.py --ks 8 --skip-plain --reps 4"
for pass in 1 2; do
  for v in "" "--module LONG_K_64=0" "--tuning bn_cols=8" "--tuning xcd_clients=0" "--groups 2"; do
    echo "== $v" >> $OUT/ab.log
    timeout -k 10 120 $P $v 2>&1 | grep '^{' | grep -v plain >> $OUT/ab.log || exit 1
  done
done
echo "exit $?"
