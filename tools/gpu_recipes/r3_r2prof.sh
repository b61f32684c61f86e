# Same box: the round-2 tree (_r2tree, f0ac677), HEAD, and HEAD without the batched-client GEMM prologues
# (_nbtree, -DFEDTGAN_NO_BATCH_PROLOGUE): full captured step (microbench --step-only), then kernel traces.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3r2p}
mkdir -p $O
for t in _r2tree . _nbtree; do
  n=$(basename $(cd $R/$t && pwd)); [ "$t" = "." ] && n=head
  (cd $R/$t && timeout -k 10 200 python tools/microbench.py --step-only > $O/${n}_step.txt 2>&1) || exit 1
done
cd /tmp
for t in _r2tree . _nbtree; do
  n=$(basename $(cd $R/$t && pwd)); [ "$t" = "." ] && n=head
  (cd $R/$t && timeout -k 10 300 rocprofv3 --kernel-trace -d $O/$n -o run -- python3 tools/microbench.py --step-only > $O/$n.log 2>&1) && \
  python3 $R/tools/step_breakdown.py $O/$n/run_results.db > $O/${n}_breakdown.txt 2>&1 && \
  python3 $R/tools/kernel_names.py $O/$n/run_results.db gemm > $O/${n}_names.txt && rm -rf $O/$n || exit 1
done
echo "exit 0"
