# Round 5: round-time stalls after the CSV formatter warm-up -- the fresh-process 4-round GPU test, a 6-round
# Intrusion run with per-round host metrics, 2- and 4-epoch CLI runs (timestamp_experiment.csv), two bench lines.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5stall}
mkdir -p $OUT
cd $R
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_federation.py -k round_zero > $OUT/pytest_round0.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 150 python tools/run_config.py --spec intrusion --clients 1 --epochs 6 --fed metrics_log=$OUT/m_int$i.jsonl > $OUT/int$i.log 2>&1 || exit 1
done
C=/tmp/r5cli; rm -rf $C; mkdir -p $C $OUT/cli
(cd $C && PYTHONPATH=$R timeout -k 10 150 python -m dtds.distributed -world_size 1 -colocated -epochs 2 > $OUT/cli/cli2.log 2>&1 && cp timestamp_experiment.csv $OUT/cli/ts2.csv) || exit 1
(cd $C && PYTHONPATH=$R timeout -k 10 150 python -m dtds.distributed -world_size 1 -colocated -epochs 4 > $OUT/cli/cli4.log 2>&1 && cp timestamp_experiment.csv $OUT/cli/ts4.csv) || exit 1
rm -rf $C
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 >> $OUT/bench.jsonl || exit 1
done
echo done
