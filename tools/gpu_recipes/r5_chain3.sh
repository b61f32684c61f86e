# Round 5: (first GPU process of the call) cold Intrusion initialisation with the HIP context timed apart and a
# cProfile; the chain-tail tests; step A/B of two head rows per workgroup in the D-phase chain (chain_rows 2 vs 1);
# kernel trace of the step; two bench lines.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5chain3}
mkdir -p $OUT
cd $R
timeout -k 10 200 python tools/init_profile.py --spec intrusion --rows 40000 --cuda-first --cprofile --top 40 --json $OUT/init_cold.jsonl > $OUT/init_cold.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_engine.py > $OUT/pytest_engine.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 120 python tools/microbench.py --step-only >> $OUT/step.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/microbench.py --step-only --tuning chain_rows=1 >> $OUT/step_rows1.txt 2>&1 || exit 1
done
cd /tmp
(cd $R && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 tools/microbench.py --step-only > $OUT/prof.log 2>&1) || exit 1
python3 $R/tools/step_breakdown.py $OUT/prof/run_results.db > $OUT/step_breakdown.txt 2>&1 || exit 1
rm -rf $OUT/prof
cd $R
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 >> $OUT/bench.jsonl || exit 1
done
echo done
