# Round 6 final tree: the driver's bench command three times back to back on one box (spread of the round time)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6am
mkdir -p $OUT
cd $R
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 >> $OUT/bench.jsonl || exit 1
done
python3 -c "
import json
for l in open('$OUT/bench.jsonl'):
    d = json.loads(l); print(d['ms_per_step'], d['phase_s'], d['init_s']['total'])
"
