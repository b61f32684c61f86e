# Avg_JSD / Avg_WD at epochs 0-2 on the shipped Intrusion split, 8 seeds, against the reference code's own
# 8-seed numbers (profiles/reference_quality_r3_byvalue.json): the round-3 ablations.  Work under /tmp; only
# the summaries come back (gpurun merges at most 64 MiB of gpurun_out/).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3q}
W=/tmp/fedtgan_quality
mkdir -p $OUT $W
S="--epochs 3 --seeds 0 1 2 3 4 5 6 7 --bootstrap-rows 20000 --no-utility"
timeout -k 10 300 python tools/real_quality.py $S --precisions bf16 fp32 --out $W/base > $OUT/base.log 2>&1 && \
cp $W/base/real_quality.json $OUT/base.json && \
timeout -k 10 300 python tools/real_quality.py $S --precisions bf16 --batched off --out $W/threads > $OUT/threads.log 2>&1 && \
cp $W/threads/real_quality.json $OUT/threads.json && \
timeout -k 10 300 python tools/real_quality.py $S --precisions bf16 --init broadcast --out $W/bcast > $OUT/bcast.log 2>&1 && \
cp $W/bcast/real_quality.json $OUT/bcast.json
echo "exit $?"
