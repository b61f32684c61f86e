# Round 6: one step graph per epoch (EngineConfig.graph_blocks = 0: the epoch's 10 blocks of 8 steps in one graph)
# vs one graph per 8-step block -- engine GPU tests, bench A/B alternating on one box
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6aa
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_hip_engine.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for i in 1 2 3; do
  for v in "graph_blocks=0" "graph_blocks=1"; do
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --engine $v 2>/dev/null | tail -1 | sed "s/^/[$v] /" >> $OUT/bench.jsonl || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/bench.jsonl'):
    t, j = l.split('] ', 1); d = json.loads(j); print(t + ']', d['ms_per_step'], d['phase_s'], d['init_s']['total'])
"
