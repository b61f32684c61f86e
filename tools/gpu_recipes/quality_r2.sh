set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/pytest_gpu2.log 2>&1 && \
timeout -k 10 900 python -u tools/real_quality.py --epochs 30 --eval-epochs 0 1 2 3 5 7 9 14 19 29 --seeds 0 1 2 3 --precisions bf16 fp32 --out gpurun_out/quality > gpurun_out/quality.log 2>&1
echo "exit $?"
