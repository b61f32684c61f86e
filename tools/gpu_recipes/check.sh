set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 170 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 150 python tools/rccl_selftest.py > gpurun_out/rccl.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
echo "exit $?"
