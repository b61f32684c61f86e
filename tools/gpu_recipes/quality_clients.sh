# Real-data quality vs the number of clients (BASELINE.json: "Avg_JSD/Avg_WD on Intrusion,
# clients=1/2/4/8"): the shipped Intrusion split's 8,078 training rows divided among K clients, each
# resampled to 20,000 rows (the reference's ~40 steps per client per epoch), ROUNDS rounds (default 100),
# bf16, SEEDS seeds (default 0 1);
# ML-utility gap at the last round.  One GPU: the K clients run as threads (one HIP stream each).
set -o pipefail
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-100}
SEEDS=${SEEDS:-"0 1"}
EVAL=${EVAL:-"0 1 2 4 9 49 99"}
for K in 1 2 4 8; do
  timeout -k 10 900 python tools/real_quality.py --clients $K --epochs $ROUNDS --seeds $SEEDS --precisions bf16 \
    --bootstrap-rows 20000 --only-scored-csv --eval-epochs $EVAL --utility-workers 8 \
    --out /tmp/quality_k$K > gpurun_out/quality_k$K.log 2>&1 || exit 1
  cp /tmp/quality_k$K/real_quality.json gpurun_out/quality_k$K.json   # (the client CSVs stay on the box)
done
echo done
