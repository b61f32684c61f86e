# Same-box A/B of the one-client step: round-3 tree (_basetree) vs HEAD, alternating, plus the bench line of each.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r4ab1}
mkdir -p $OUT
R=$GRAFT_REPO_ROOT
for i in 1 2; do
  (cd $R/_basetree && timeout -k 10 150 python tools/microbench.py --step-only >> $OUT/base_step.txt 2>&1) || break
  (cd $R && timeout -k 10 150 python tools/microbench.py --step-only >> $OUT/head_step.txt 2>&1) || break
done
(cd $R/_basetree && timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $OUT/base_bench.log 2>&1) && \
(cd $R && timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $OUT/head_bench.log 2>&1)
echo "exit $?"
