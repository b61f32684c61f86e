# Round 6: per-kernel instruction mix of the Intrusion step after the hardware bf16 pack (tools/gpu_probe.py --steps 5,
# one counter pass)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6ak
mkdir -p $OUT
cd /tmp
(cd $R && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VMEM SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $OUT/pmc -o run -- python3 tools/gpu_probe.py --backend hip --rows 40000 --steps 5 > $OUT/pmc.log 2>&1) || { tail -5 $OUT/pmc.log; exit 1; }
ls $OUT/pmc
