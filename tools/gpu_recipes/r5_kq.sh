# Round 5: 8 emulated Intrusion clients on one GPU -- client threads with HIP's 4 hardware queues per process
# (8 client streams share 4 in-order queues) vs 8 / 16 queues, and the batched engine; 12 epochs each, per-round
# metrics.  Then a kernel trace of the 4-queue thread run (per-queue timelines).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5kq}
mkdir -p $OUT
cd $R
RC="python tools/run_config.py --spec intrusion --clients 8 --epochs 12"
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 150 $RC --batched off --fed metrics_log=$OUT/m_q$q.jsonl > $OUT/q$q.log 2>&1 || exit 1
done
timeout -k 10 150 $RC --batched on --fed metrics_log=$OUT/m_b.jsonl > $OUT/b.log 2>&1 || exit 1
GPU_MAX_HW_QUEUES=16 timeout -k 10 150 $RC --batched on --fed metrics_log=$OUT/m_b16.jsonl > $OUT/b16.log 2>&1 || exit 1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 $R/tools/run_config.py --spec intrusion --clients 8 --epochs 6 --batched off > $OUT/kt.log 2>&1 || exit 1
echo done
