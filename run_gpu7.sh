set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_ops.py tests/test_hip_engine.py tests/test_gpu_engine.py -m gpu -q -x --timeout 170 --timeout-method thread > gpurun_out/pytest_gpu7.log 2>&1 && \
timeout -k 10 300 python -u tools/microbench.py --bn-ab > gpurun_out/bn_ab.log 2>&1
echo "exit $?"
