set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step -o run -- python3 tools/gpu_probe.py --backend hip --rows 40000 --steps 40 > gpurun_out/prof_step.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof_bench.log 2>&1
echo "exit $?"
