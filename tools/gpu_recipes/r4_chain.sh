# Coalesced chain tail (chain_coalesced): tests, step A/B, bench A/B.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4chain}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_engine.py -k "chain or fused or autograd" > $OUT/pytest.log 2>&1 || exit 1
for pass in 1 2; do
  for v in "" "--tuning chain_coalesced=1"; do
    echo "== $v" >> $OUT/step.txt
    timeout -k 10 120 python tools/microbench.py --step-only $v 2>&1 | grep "full step" >> $OUT/step.txt || exit 1
  done
done
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 >> $OUT/bench.jsonl || exit 1
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --tuning chain_coalesced=1 2>/dev/null | tail -1 >> $OUT/bench_n.jsonl || exit 1
done
echo done
