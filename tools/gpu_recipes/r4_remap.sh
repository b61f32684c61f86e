# XCD tile order always (gemm_xcd_remap = 2 default): GEMM / engine tests, bench (3 runs), step, batched 8.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4remap}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_hip_ops.py tests/test_hip_engine.py tests/test_batched.py tests/test_gpu_engine.py > $OUT/pytest.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 >> $OUT/bench.jsonl || exit 1
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --tuning gemm_xcd_remap=1 2>/dev/null | tail -1 >> $OUT/bench_r1.jsonl || exit 1
done
timeout -k 10 150 python tools/batched_probe.py --ks 8 --skip-plain --reps 4 > $OUT/probe.log 2>&1 || exit 1
timeout -k 10 150 python tools/batched_probe.py --ks 8 --skip-plain --reps 4 --tuning gemm_xcd_remap=1 >> $OUT/probe.log 2>&1 || exit 1
echo done
