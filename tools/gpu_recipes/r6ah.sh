# Round 6: early host wake at the round boundary -- bench A/B of FedConfig.sync_lead_blocks (the host waits for the
# epoch up to its last N graph blocks, then queues aggregation / sampling / next round behind them) with and without
# round_sync, alternating on one box
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6ah
mkdir -p $OUT
cd $R
for i in 1 2 3; do
  for v in "train_sync=1" "round_sync=0" "sync_lead_blocks=1 --fed round_sync=0" "sync_lead_blocks=2 --fed round_sync=0"; do
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --fed $v 2>/dev/null | tail -1 | sed "s/^/[$v] /" >> $OUT/bench.jsonl || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/bench.jsonl'):
    t, j = l.split('] ', 1); d = json.loads(j); print(t + ']', d['ms_per_step'], d['phase_s'], d.get('avg_jsd'))
"
