# Round 5: the chain kernels' tail weights requested before the slab reduction -- full-step time (three passes) and
# a kernel trace of the captured step (critical path per kernel).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5chain}
mkdir -p $OUT
cd $R
for i in 1 2 3; do
  timeout -k 10 120 python tools/microbench.py --step-only >> $OUT/step.txt 2>&1 || exit 1
done
cd /tmp
(cd $R && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 tools/microbench.py --step-only > $OUT/prof.log 2>&1) || exit 1
python3 $R/tools/step_breakdown.py $OUT/prof/run_results.db > $OUT/step_breakdown.txt 2>&1 || exit 1
rm -rf $OUT/prof
echo done
