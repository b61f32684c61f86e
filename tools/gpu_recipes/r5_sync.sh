# Round 5: host synchronisation in the round -- the train-phase wait before the aggregation (train_sync), the
# end-of-round wait (round_sync) and the per-collective event timers (phase_detail), plain and over a one-rank
# RCCL communicator (--force-dist); bench lines alternate, two passes.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5sync}
mkdir -p $OUT
cd $R
B="python bench.py --steps 20 --warmup 5"
for i in 1 2; do
  for v in "" "--fed round_sync=0" "--fed train_sync=0 --fed round_sync=0" "--force-dist" "--force-dist --fed round_sync=0" \
           "--force-dist --fed train_sync=0 --fed round_sync=0" "--force-dist --fed phase_detail=0"; do
    echo "== $v" >> $OUT/sync.txt
    timeout -k 10 150 $B $v 2>/dev/null | tail -1 >> $OUT/sync.txt || exit 1
  done
done
echo done
