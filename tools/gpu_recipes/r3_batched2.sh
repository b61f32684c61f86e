set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3k}
mkdir -p $OUT
timeout -k 10 200 python tools/batched_diff.py --k 2 > $OUT/diff_k2.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_batched.py tests/test_hip_engine.py tests/test_gpu_federation.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/pytest_batched.log 2>&1 && \
timeout -k 10 400 python tools/batched_probe.py --streams > $OUT/batched_probe.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-eval > $OUT/bench.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-eval --phase-timer sync > $OUT/bench_sync.log 2>&1
echo "exit $?"
