# Round 5: one-client step knob sweep on the current tree (two passes each, alternating): D0 weight-gradient tile,
# D0 weight gradient applying Adam in its tiles, transposed one-hot gathers, forced chain prefetch.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5knobs}
mkdir -p $OUT
cd $R
for i in 1 2; do
  for v in "" "--engine dw0_tile=32" "--engine dw0_tile=64" "--engine dw0_tile=128" "--engine fuse_d_adam=0 --engine fuse_d0_adam=1" \
           "--engine onehot_trans=1" "--tuning chain_pre=2 --tuning chain_rows=1" "--tuning gemm_pair_max_wg=512"; do
    echo "== $v" >> $OUT/knobs.txt
    timeout -k 10 120 python tools/microbench.py --step-only $v 2>&1 | grep "full step" >> $OUT/knobs.txt || exit 1
  done
done
echo done
