# Round 5: the pipelined generation stream at high priority (its own hardware queue) vs normal, with and without the
# deferred hand-off, plain and over a one-rank RCCL communicator; two passes alternating.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5genprio}
mkdir -p $OUT
cd $R
B="python bench.py --steps 20 --warmup 5"
for i in 1 2; do
  for v in "" "--fed gen_stream_priority=-1" "--fed gen_stream_priority=-1 --fed defer_handoff=1" \
           "--force-dist" "--force-dist --fed gen_stream_priority=-1" "--force-dist --fed gen_stream_priority=-1 --fed defer_handoff=1"; do
    echo "== $v" >> $OUT/prio.txt
    timeout -k 10 150 $B $v 2>/dev/null | tail -1 >> $OUT/prio.txt || exit 1
  done
done
echo done
