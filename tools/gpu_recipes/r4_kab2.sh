# Round-1 stall: per-round host timings (metrics_log h_wait / h_issue / h_total) at K = 1 (bench-like) and K = 8 batched,
# plus the emulated-federation GPU tests.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4kab2}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_gpu_federation.py -k "emulated or batched" > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 150 python tools/run_config.py --spec intrusion --clients 1 --epochs 6 --fed metrics_log=$OUT/m_1.jsonl > $OUT/k1.log 2>&1 || exit 1
timeout -k 10 150 python tools/run_config.py --spec intrusion --clients 8 --epochs 6 --batched on --fed metrics_log=$OUT/m_8.jsonl > $OUT/k8.log 2>&1 || exit 1
timeout -k 10 150 python tools/run_config.py --spec intrusion --clients 8 --epochs 6 --batched on --fed async_csv=0 --fed metrics_log=$OUT/m_8s.jsonl > $OUT/k8s.log 2>&1 || exit 1
echo done
for b in on off; do
  timeout -k 10 150 python tools/run_config.py --spec adult --clients 8 --shard dirichlet --alpha 0.3 --epochs 8 --rows 8000 --batched $b --fed metrics_log=$OUT/m_adult_$b.jsonl > $OUT/adult_$b.log 2>&1 || exit 1
done
timeout -k 10 200 python tools/run_config.py --spec covertype --clients 8 --shard dirichlet --alpha 0.3 --epochs 6 --rows 20000 > $OUT/cov.log 2>&1 || exit 1
echo done2
