# Round 5: hardware counters of the chain kernels (chain_epilogue_kernel: D0 split-K reduce + LeakyReLU/dropout
# + the next Linear) and the fused GEMM + Adam launches (gemm_adam_kernel) of the one-client Intrusion step
# (rocprofv3 --pmc, one pass per counter group, kernels filtered by name), then per-kernel means + ratios.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5pmc}
mkdir -p $O
cd /tmp
P="python3 $R/tools/microbench.py --step-only"
K="chain_epilogue|gemm_adam"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES" \
           "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd $R && timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "$K" --output-format csv -d $O/p$i -o run -- $P > $O/p$i.log 2>&1) || exit 1
done
python3 $R/tools/pmc_summary.py $O/p1 $O/p2 $O/p3 $O/p4 --out=$O/pmc_summary.txt > $O/pmc_stdout.txt 2>&1 || exit 1
rm -rf $O/p1 $O/p2 $O/p3 $O/p4
echo done
