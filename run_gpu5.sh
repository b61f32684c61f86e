set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_ops.py tests/test_hip_engine.py -m gpu -q --timeout 170 --timeout-method thread > gpurun_out/pytest_gpu5.log 2>&1 && \
timeout -k 10 300 python -u tools/microbench.py --onehot-ab > gpurun_out/onehot_ab2.log 2>&1
echo "exit $?"
