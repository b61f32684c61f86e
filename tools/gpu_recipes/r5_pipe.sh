# Round 5: pipelined sampling (round r's table generated on a side stream while round r + 1 trains) -- its GPU test,
# the federation GPU tests, bench A/B (two passes, alternating), one-rank RCCL bench, and a 4-epoch CLI run.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5pipe}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_federation.py > $OUT/pytest_fed.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 >> $OUT/bench_pipe.jsonl || exit 1
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --fed pipeline_sample=0 2>/dev/null | tail -1 >> $OUT/bench_nopipe.jsonl || exit 1
done
timeout -k 10 150 python bench.py --steps 20 --warmup 5 --force-dist 2>/dev/null | tail -1 >> $OUT/bench_dist.jsonl || exit 1
timeout -k 10 150 python tools/run_config.py --spec intrusion --clients 1 --epochs 6 --fed metrics_log=$OUT/m_int.jsonl > $OUT/int.log 2>&1 || exit 1
echo done
