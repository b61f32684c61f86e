# Step A/B against the round-2 tree on one box (two runs each), GPU tests first, then the per-kernel trace.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3ta}
mkdir -p $O
(cd $R && timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 170 --timeout-method thread > $O/pytest_gpu.log 2>&1) && \
(cd $R/_r2tree && timeout -k 10 200 python tools/microbench.py --step-only > $O/r2_step.txt 2>&1) && \
(cd $R && timeout -k 10 200 python tools/microbench.py --step-only > $O/head_step.txt 2>&1) && \
(cd $R/_r2tree && timeout -k 10 200 python tools/microbench.py --step-only > $O/r2_step2.txt 2>&1) && \
(cd $R && timeout -k 10 200 python tools/microbench.py --step-only > $O/head_step2.txt 2>&1) && \
cd /tmp && (cd $R && timeout -k 10 300 rocprofv3 --kernel-trace -d $O/head -o run -- python3 tools/microbench.py --step-only > $O/head.log 2>&1) && \
python3 $R/tools/step_breakdown.py $O/head/run_results.db > $O/head_breakdown.txt 2>&1 && rm -rf $O/head
echo "exit $?"
