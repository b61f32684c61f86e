# Round 6: hardware counters of the wide table's G.out forward GEMM (128 x 128 tiles, 440 workgroups) in isolation
# (tools/gout_probe.py --only-gout, 20 launches), one counter pass per run
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6ag
mkdir -p $OUT
cd /tmp
i=0
for pmc in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
  i=$((i+1))
  (cd $R && timeout -s KILL 90 rocprofv3 --pmc $pmc -d $OUT/pmc$i -o run -- python3 tools/gout_probe.py --only-gout --reps 20 > $OUT/pmc$i.log 2>&1) || { tail -5 $OUT/pmc$i.log; exit 1; }
done
ls -R $OUT | head -30
