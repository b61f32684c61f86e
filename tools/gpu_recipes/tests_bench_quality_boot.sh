set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 170 --timeout-method thread > gpurun_out/pytest_gpu3.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench3.log 2>&1 && \
timeout -k 10 900 python -u tools/real_quality.py --epochs 500 --eval-epochs 0 1 2 4 9 49 99 249 499 --bootstrap-rows 20000 --only-scored-csv --seeds 0 1 2 3 --precisions bf16 fp32 --out gpurun_out/quality_boot > gpurun_out/quality_boot.log 2>&1
echo "exit $?"
