# XCD-aware client placement of batched GEMMs (xcd_clients 0 / 1): batched tests, K=8 epoch, per-GEMM times.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4xcd}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_batched.py tests/test_gpu_federation.py -m gpu -v --timeout 240 --timeout-method thread -k "batched or hier or dedicated" > $OUT/pytest.log 2>&1; echo "pytest rc $?" >> $OUT/pytest.log
for x in 0 1; do
  timeout -k 10 150 python tools/batched_probe.py --ks 4 8 --skip-plain --reps 4 --tuning xcd_clients=$x > $OUT/probe_x$x.log 2>&1 || break
  timeout -k 10 200 python tools/batched_ops.py --k 8 --only-planner --tuning xcd_clients=$x > $OUT/ops_x$x.jsonl 2> $OUT/ops_x$x.err || break
done
echo "exit $?"
