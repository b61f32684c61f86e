# Same box: bench line round-3 tree vs HEAD (alternating), then one kernel-trace profile of each.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4benchab3}
mkdir -p $OUT
for i in 1 2 3; do
  (cd $R/_basetree && timeout -k 10 150 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 >> $OUT/base_bench.jsonl) || exit 1
  (cd $R && timeout -k 10 150 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 >> $OUT/head_bench.jsonl) || exit 1
done
cd /tmp
(cd $R/_basetree && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_base -o run -- python3 bench.py --steps 10 --warmup 3 > $OUT/prof_base.log 2>&1) || exit 1
(cd $R && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_head -o run -- python3 bench.py --steps 10 --warmup 3 > $OUT/prof_head.log 2>&1) || exit 1
du -ah $OUT | sort -h | tail -12
find $OUT -name "*kernel_trace.csv" -delete
find $OUT -type f -size +4M -delete
echo done
