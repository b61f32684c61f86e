set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_ops.py tests/test_hip_engine.py tests/test_golden.py tests/test_vgm_parity.py -m gpu -q --timeout 170 --timeout-method thread > gpurun_out/pytest_gpu4.log 2>&1 && \
timeout -k 10 300 python -u tools/microbench.py --onehot-ab > gpurun_out/onehot_ab.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench4.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --engine onehot=0 > gpurun_out/bench4_dense.log 2>&1
echo "exit $?"
