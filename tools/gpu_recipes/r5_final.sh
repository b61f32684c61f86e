# Round 5 verification: RCCL pre-multiplied-sum probe, every GPU test, the smoke test, bench lines (plain x2,
# one-rank RCCL x1).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5final}
mkdir -p $OUT
cd $R
timeout -k 10 120 python tools/premul_probe.py > $OUT/premul.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 >> $OUT/bench.jsonl || exit 1
done
timeout -k 10 150 python bench.py --steps 20 --warmup 5 --force-dist 2>/dev/null | tail -1 >> $OUT/bench_dist.jsonl || exit 1
echo done
