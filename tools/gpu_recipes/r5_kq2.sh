# Round 5: (first GPU process of the call) cold Intrusion initialisation; then K = 2 / 4 / 8 emulated Intrusion
# clients on one GPU, client threads (streams created back to back: even over HIP's 4 hardware queues) vs the
# batched engine, 12 epochs each with per-round metrics; then the chain-prefetch step A/B.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5kq2}
mkdir -p $OUT
cd $R
timeout -k 10 200 python tools/init_profile.py --spec intrusion --rows 40000 --json $OUT/init_cold.jsonl > $OUT/init_cold.log 2>&1 || exit 1
RC="python tools/run_config.py --spec intrusion --epochs 12"
for k in 8 4 2; do
  timeout -k 10 150 $RC --clients $k --batched off --fed metrics_log=$OUT/m_t$k.jsonl > $OUT/t$k.log 2>&1 || exit 1
  timeout -k 10 150 $RC --clients $k --batched on --fed metrics_log=$OUT/m_b$k.jsonl > $OUT/b$k.log 2>&1 || exit 1
done
timeout -k 10 150 $RC --clients 8 --batched off --fed metrics_log=$OUT/m_t8b.jsonl > $OUT/t8b.log 2>&1 || exit 1
bash $R/tools/gpu_recipes/r5_chain.sh r5chain2 || exit 1
echo done
