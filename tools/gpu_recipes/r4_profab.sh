# Same box: kernel-trace stats of the bench, round-3 tree vs HEAD (CSV summaries only).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4profab}
mkdir -p $OUT
cd /tmp
for t in base head; do
  D=$R; [ $t = base ] && D=$R/_basetree
  (cd $D && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$t -o run -- python3 bench.py --steps 10 --warmup 3 > $OUT/prof_$t.log 2>&1) || exit 1
done
find $OUT -name "*kernel_trace.csv" -delete
find $OUT -type f -size +4M -delete
du -ah $OUT | sort -h | tail -8
echo done
