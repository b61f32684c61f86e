# Same box: bench line round-3 tree vs HEAD (alternating), then one kernel-trace profile of each.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4benchab4}
mkdir -p $OUT
for i in 1 2 3; do
  (cd $R/_basetree && timeout -k 10 150 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 >> $OUT/base_bench.jsonl) || exit 1
  (cd $R && timeout -k 10 150 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 >> $OUT/head_bench.jsonl) || exit 1
done
echo done
