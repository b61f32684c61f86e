# Round 5 end: the whole GPU test suite and smoke() on the final build.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5final}
mkdir -p $OUT
cd $R
timeout -k 10 1000 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 1
echo done
for i in 1 2; do timeout -k 10 150 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 >> $OUT/bench.jsonl || exit 1; done
echo done
