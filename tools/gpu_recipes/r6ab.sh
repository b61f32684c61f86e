# Round 6: round-boundary host waits on the current tree -- bench A/B of FedConfig.train_sync (host wait for the
# epoch's kernels before the aggregation / sampling issue) and defer_handoff, alternating on one box
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6ab
mkdir -p $OUT
cd $R
for i in 1 2 3; do
  for v in "train_sync=1" "train_sync=0" "defer_handoff=1"; do
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --fed $v 2>/dev/null | tail -1 | sed "s/^/[$v] /" >> $OUT/bench.jsonl || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/bench.jsonl'):
    t, j = l.split('] ', 1); d = json.loads(j); print(t + ']', d['ms_per_step'], d['phase_s'])
"
