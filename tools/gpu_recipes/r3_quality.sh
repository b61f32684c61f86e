# Avg_JSD / Avg_WD at epochs 0-2 on the shipped Intrusion split, 8 seeds, against the reference code's own
# 8-seed numbers (profiles/reference_quality_r3_byvalue.json): the round-3 ablations.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3q}
mkdir -p $OUT
S="--epochs 3 --seeds 0 1 2 3 4 5 6 7 --bootstrap-rows 20000 --no-utility"
timeout -k 10 300 python tools/real_quality.py $S --precisions bf16 fp32 --out $OUT/base > $OUT/base.log 2>&1 && \
timeout -k 10 300 python tools/real_quality.py $S --precisions bf16 --batched off --out $OUT/threads > $OUT/threads.log 2>&1 && \
timeout -k 10 300 python tools/real_quality.py $S --precisions bf16 --init broadcast --out $OUT/bcast > $OUT/bcast.log 2>&1
echo "exit $?"
