# Round 6: idle gaps of the engine's epoch graphs (kernel trace), multi-draw on / off
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6f
mkdir -p $OUT
cd /tmp
for md in 1 0; do
(cd $R && timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/step$md -o run -- python3 tools/microbench.py --step-only --epochs-only --engine multi_draw=$md > $OUT/step$md.log 2>&1) || exit 1
python3 $R/tools/step_breakdown.py $OUT/step$md/run_results.db --gaps > $OUT/gaps$md.txt 2>&1 || exit 1
rm -rf $OUT/step$md
done
echo done
