# Batched multi-client engine: correctness tests, the existing engine tests (no regression from the
# client-offset prologues), and the K = 1/2/4/8 epoch-time probe.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3h}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_batched.py tests/test_hip_engine.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/pytest_batched.log 2>&1 && \
timeout -k 10 400 python tools/batched_probe.py --streams > $OUT/batched_probe.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-eval > $OUT/bench.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-eval --phase-timer sync > $OUT/bench_sync.log 2>&1
echo "exit $?"
