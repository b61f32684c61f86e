# Round 5: deferred table hand-off (FedConfig.defer_handoff) A/B, plain and over a one-rank RCCL communicator,
# three passes alternating.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5defer}
mkdir -p $OUT
cd $R
B="python bench.py --steps 20 --warmup 5"
for i in 1 2 3; do
  for v in "" "--fed defer_handoff=0" "--force-dist" "--force-dist --fed defer_handoff=0"; do
    echo "== $v" >> $OUT/defer.txt
    timeout -k 10 150 $B $v 2>/dev/null | tail -1 >> $OUT/defer.txt || exit 1
  done
done
echo done
