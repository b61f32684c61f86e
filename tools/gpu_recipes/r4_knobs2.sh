# One-client step: EngineConfig / tuning knobs on top of the always-remap default (two passes).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4knobs2}
mkdir -p $OUT
cd $R
for pass in 1 2; do
  for v in "" "--engine chain_d1=0" "--engine fuse_d_adam=0" "--engine fuse_g_adam=0" "--engine fuse_d0_adam=1" "--engine onehot_trans=1" "--engine dw0_tile=64" "--engine dw0_tile=128" "--engine graph_unroll=16" "--tuning gemm_pairs=0" "--tuning adam_store=0" "--tuning gemm_splitk_inlaunch=1"; do
    echo "== $v" >> $OUT/step.txt
    timeout -k 10 120 python tools/microbench.py --step-only $v 2>&1 | grep "full step" >> $OUT/step.txt || exit 1
  done
done
echo done
