# End-of-round-3 check: GPU tests, smoke, RCCL self-test, bench (plain and over a one-rank RCCL communicator),
# the batched 2/4/8-client step, then kernel traces of the captured step and of bench.py with their summaries.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-final_r3}
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 170 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 100 python -c "import __graft_entry__ as e; e.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 150 python tools/rccl_selftest.py > $O/rccl.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 && \
timeout -k 10 200 python bench.py --force-dist --steps 20 --warmup 5 > $O/bench_rccl1.log 2>&1 && \
timeout -k 10 300 python tools/batched_probe.py --ks 1 2 4 8 --plan on --reps 4 > $O/batched.log 2>&1 && \
cd /tmp && \
(cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_step -o run -- python3 tools/microbench.py --step-only > $O/prof_step.log 2>&1) && \
(cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run -- python3 bench.py --steps 5 --warmup 2 > $O/prof_bench.log 2>&1) && \
python3 $R/tools/step_breakdown.py $O/prof_step/run_results.db > $O/step_breakdown.txt 2>&1 && \
python3 $R/tools/prof_summary.py $O/prof_bench/run_results.db > $O/bench_kernels.txt 2>&1 && \
rm -rf $O/prof_step $O/prof_bench
echo "exit $?"
