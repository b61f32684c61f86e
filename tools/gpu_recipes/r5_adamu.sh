# Round 5: the step's two Adam launches (D: 1.67 M, G: ~0.5 M parameters) with 4 float4 per thread in flight
# (adam_u_min=0) vs one (default below 4 M elements), three passes, alternating; plus a 2-epoch wide check.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5adamu}
mkdir -p $OUT
cd $R
for i in 1 2 3; do
  for v in "" "--tuning adam_u_min=0" "--tuning adam_u_min=0 --tuning adam_max_blocks=256"; do
    echo "== $v" >> $OUT/adamu.txt
    timeout -k 10 120 python tools/microbench.py --step-only $v 2>&1 | grep "full step" >> $OUT/adamu.txt || exit 1
  done
done
echo done
