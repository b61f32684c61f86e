# rocprofv3 kernel traces: the captured Intrusion step (tools/gpu_probe.py) and bench.py; summaries in gpurun_out/
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step -o run -- python3 tools/gpu_probe.py --backend hip --rows 40000 --steps 40 > gpurun_out/prof_step.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof_bench.log 2>&1 && \
python3 tools/step_breakdown.py gpurun_out/prof_step/run_results.db > gpurun_out/step_breakdown.txt 2>&1 && \
python3 tools/prof_summary.py gpurun_out/prof_step/run_results.db --timeline >> gpurun_out/step_breakdown.txt 2>&1 && \
python3 tools/prof_summary.py gpurun_out/prof_bench/run_results.db > gpurun_out/bench_kernels.txt 2>&1
echo "exit $?"
