# Round 5: kernel traces of the captured one-client step with the generator's BatchNorm folded into its GEMMs
# (bn_fold=1) and as launches (bn_fold=0): critical path per kernel (tools/step_breakdown.py).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5foldprof}
mkdir -p $OUT
cd /tmp
for f in 1 0; do
  (cd $R && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/step_$f -o run -- python3 tools/microbench.py --step-only --engine bn_fold=$f > $OUT/step_$f.log 2>&1) || exit 1
  python3 $R/tools/step_breakdown.py $OUT/step_$f/run_results.db > $OUT/step_breakdown_fold$f.txt 2>&1 || exit 1
  rm -rf $OUT/step_$f
done
(cd $R && timeout -k 10 200 python tools/microbench.py --cfg-ab bn_fold > $OUT/step_ab.txt 2>&1) || exit 1
echo done
