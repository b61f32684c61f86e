# Round 5: native knob sweep on the current step (unrolled Adam): Adam store policy, activation row modes, GP
# threads, split-K reduction, store policy, BN shapes; two passes, alternating.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5knobs2}
mkdir -p $OUT
cd $R
for i in 1 2; do
  for v in "" "--tuning adam_store=2" "--tuning adam_store=16" "--tuning act_row_mode=1" "--tuning gp_threads=1024" \
           "--tuning gemm_splitk_inlaunch=0" "--tuning gemm_store_wt=1" "--tuning bn_threads=1024" "--tuning bn_cols=4"; do
    echo "== $v" >> $OUT/knobs.txt
    timeout -k 10 120 python tools/microbench.py --step-only $v 2>&1 | grep "full step" >> $OUT/knobs.txt || exit 1
  done
done
echo done
