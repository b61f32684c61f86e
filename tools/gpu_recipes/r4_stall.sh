# Round-1 stall after the pinned-copy warm-up: per-round host timings at K = 1 and 8 (batched), plus bench.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4stall}
mkdir -p $OUT
cd $R
timeout -k 10 150 python tools/run_config.py --spec intrusion --clients 1 --epochs 5 --fed metrics_log=$OUT/m_1.jsonl > $OUT/k1.log 2>&1 || exit 1
timeout -k 10 150 python tools/run_config.py --spec intrusion --clients 8 --epochs 5 --batched on --fed metrics_log=$OUT/m_8.jsonl > $OUT/k8.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 >> $OUT/bench.jsonl || exit 1
echo done
