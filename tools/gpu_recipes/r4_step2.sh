# Step time (4 runs) + the step's kernel breakdown after a sampler change.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4step2}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_ops.py -k "sample" > $OUT/pytest.log 2>&1 || exit 1
for i in 1 2 3 4; do
  timeout -k 10 120 python tools/microbench.py --step-only 2>&1 | grep "full step" >> $OUT/step.txt || exit 1
done
cd /tmp
(cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_step -o run -- python3 tools/microbench.py --step-only > $OUT/prof_step.log 2>&1) || exit 1
python3 $R/tools/step_breakdown.py $OUT/prof_step/run_results.db > $OUT/step_breakdown.txt 2>&1 || exit 1
rm -rf $OUT/prof_step
echo done
