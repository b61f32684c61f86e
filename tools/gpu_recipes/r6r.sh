# Round 6: fused A-chain (EngineConfig.fuse_achain) -- engine GPU tests, epoch-graph step A/B, bench, kernel trace
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6r
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_hip_engine.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for rep in 1 2 3; do
for cfg in "fuse_achain=1" "fuse_achain=0"; do
  timeout -k 10 120 python3 tools/microbench.py --step-only --epochs-only --engine $cfg 2>&1 | grep "engine epoch" | sed "s/^/[$cfg] /" >> $OUT/ab.txt || exit 1
done
done
cat $OUT/ab.txt
timeout -k 10 120 python3 tools/gout_probe.py > $OUT/gout.txt 2>&1 || exit 1
cat $OUT/gout.txt
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit 1
tail -1 $OUT/bench.log
cd /tmp
(cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 5 --warmup 2 > $OUT/prof.log 2>&1) || exit 1
python3 $R/tools/prof_summary.py $OUT/prof/run_results.db --shape > $OUT/prof_summary.txt 2>&1 || true
python3 $R/tools/step_breakdown.py $OUT/prof/run_results.db --order --gaps > $OUT/step.txt 2>&1 || true
rm -rf $OUT/prof
echo done
