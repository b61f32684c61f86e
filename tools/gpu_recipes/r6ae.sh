# Round 6: host wake-up at the round's stream waits -- blocking synchronize vs event polling (FEDTGAN_SYNC_POLL=1),
# bench A/B, 4 alternating pairs on one box
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6ae
mkdir -p $OUT
cd $R
for i in 1 2 3 4; do
  for v in 1 0; do
    FEDTGAN_SYNC_POLL=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 | sed "s/^/[poll=$v] /" >> $OUT/bench.jsonl || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/bench.jsonl'):
    t, j = l.split('] ', 1); d = json.loads(j); print(t + ']', d['ms_per_step'], d['phase_s'])
"
