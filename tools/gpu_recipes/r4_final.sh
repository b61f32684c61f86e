# End-of-round-4 check: GPU tests, smoke, bench (plain and over a one-rank RCCL communicator), then kernel traces of
# the captured step and of bench.py with their summaries (databases deleted on the box).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-final_r4}
mkdir -p $O
cd $R
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 170 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 100 python -c "import __graft_entry__ as e; e.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 && \
timeout -k 10 200 python bench.py --force-dist --steps 20 --warmup 5 > $O/bench_rccl1.log 2>&1 && \
cd /tmp && \
(cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_step -o run -- python3 tools/microbench.py --step-only > $O/prof_step.log 2>&1) && \
(cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run -- python3 bench.py --steps 5 --warmup 2 > $O/prof_bench.log 2>&1) && \
python3 $R/tools/step_breakdown.py $O/prof_step/run_results.db > $O/step_breakdown.txt 2>&1 && \
python3 $R/tools/prof_summary.py $O/prof_bench/run_results.db > $O/bench_kernels.txt 2>&1 && \
rm -rf $O/prof_step $O/prof_bench
echo "exit $?"
