# A/B of the round's phase-timer and CSV modes on one box: plain vs --force-dist, events vs sync timers.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3f}
mkdir -p $OUT
for i in 1 2; do
for v in "" "--phase-timer sync" "--force-dist" "--force-dist --phase-timer sync" "--sync-csv"; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-eval $v > $OUT/tmp.log 2>&1 || exit 1
  echo "[$v] $(grep '^{' $OUT/tmp.log)" >> $OUT/ab.txt
done
done
echo ok
