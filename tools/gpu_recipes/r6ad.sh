# Round 6: deferred hand-off A/B, 4 alternating pairs on one box (variance check of r6ab / r6ac)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6ad
mkdir -p $OUT
cd $R
for i in 1 2 3 4; do
  for v in "defer_handoff=1" "defer_handoff=0"; do
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --fed $v 2>/dev/null | tail -1 | sed "s/^/[$v] /" >> $OUT/bench.jsonl || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/bench.jsonl'):
    t, j = l.split('] ', 1); d = json.loads(j); print(t + ']', d['ms_per_step'], d['phase_s'])
"
