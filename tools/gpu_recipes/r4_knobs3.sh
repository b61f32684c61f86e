# BN geometry combos on the final tree (microbench --step-only, two passes).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4knobs3}
mkdir -p $OUT
cd $R
for pass in 1 2; do
  for v in "" "--tuning bn_cols=4 --tuning bn_threads=1024" "--tuning bn_cols=16 --tuning bn_threads=1024" "--engine graph_unroll=80"; do
    echo "== $v" >> $OUT/step.txt
    timeout -k 10 120 python tools/microbench.py --step-only $v 2>&1 | grep "full step" >> $OUT/step.txt || exit 1
  done
done
echo done
