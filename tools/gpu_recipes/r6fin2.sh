# Round 6 (final session): full GPU verification of the tree -- every gpu test, smoke(), the driver's bench line, and a kernel trace
# of the Intrusion step (step_breakdown_r6)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6fin2
mkdir -p $OUT
cd $R
timeout -k 10 1000 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit 1
tail -1 $OUT/bench.log
cd /tmp
(cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 5 > $OUT/prof.log 2>&1) || exit 1
python3 $R/tools/step_breakdown.py $OUT/prof/run_results.db --order --gaps > $OUT/step.txt 2>&1 || true
python3 $R/tools/prof_summary.py $OUT/prof/run_results.db > $OUT/prof_summary.txt 2>&1 || true
rm -rf $OUT/prof
head -30 $OUT/step.txt
