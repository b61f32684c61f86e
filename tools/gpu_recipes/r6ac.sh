# Round 6: GPU federation tests + bench (x3) + kernel trace of the bench with the deferred hand-off default
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6ac
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_federation.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 >> $OUT/bench.jsonl || exit 1
done
python3 -c "
import json
for l in open('$OUT/bench.jsonl'):
    d = json.loads(l); print(d['ms_per_step'], d['phase_s'], d['init_s']['total'])
"
cd /tmp
(cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 5 > $OUT/prof.log 2>&1) || exit 1
python3 $R/tools/step_breakdown.py $OUT/prof/run_results.db --gaps > $OUT/step.txt 2>&1 || true
rm -rf $OUT/prof
grep -A14 "^gaps" $OUT/step.txt
