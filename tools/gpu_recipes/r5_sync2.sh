# Round 5: where the one-rank RCCL round's extra ~0.3 ms goes -- plain vs --force-dist with stream-synchronised
# phase timers (host wall time per phase), with 8 CSV formatter threads, and a torch.profiler trace of one
# --force-dist round.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5sync2}
mkdir -p $OUT
cd $R
B="python bench.py --steps 20 --warmup 5"
for i in 1 2; do
  for v in "--fed phase_timer=sync" "--force-dist --fed phase_timer=sync" "--fed csv_threads=8" "--force-dist --fed csv_threads=8"; do
    echo "== $v" >> $OUT/sync2.txt
    timeout -k 10 150 $B $v 2>/dev/null | tail -1 >> $OUT/sync2.txt || exit 1
  done
done
timeout -k 10 150 $B --force-dist --fed profile_dir=$OUT/trace_dist --fed profile_epoch=12 2>/dev/null | tail -1 > $OUT/trace_dist.json.log || exit 1
timeout -k 10 150 $B --fed profile_dir=$OUT/trace_plain --fed profile_epoch=12 2>/dev/null | tail -1 > $OUT/trace_plain.json.log || exit 1
echo done
