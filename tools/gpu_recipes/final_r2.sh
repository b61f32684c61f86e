# End-of-round check: GPU tests, RCCL self-test, bench (20 and 5 rounds), smoke, then rocprofv3 kernel
# traces of the captured step and of bench.py with their summaries.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 170 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 150 python tools/rccl_selftest.py > gpurun_out/rccl.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 200 python bench.py --force-dist --steps 20 --warmup 5 > gpurun_out/bench_rccl1.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as e; e.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step -o run -- python3 tools/gpu_probe.py --backend hip --rows 40000 --steps 40 > gpurun_out/prof_step.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof_bench.log 2>&1 && \
python3 tools/step_breakdown.py gpurun_out/prof_step/run_results.db > gpurun_out/step_breakdown.txt 2>&1 && \
python3 tools/prof_summary.py gpurun_out/prof_bench/run_results.db > gpurun_out/bench_kernels.txt 2>&1
echo "exit $?"
