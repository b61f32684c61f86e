# This framework's quality on the shipped Intrusion split (tools/real_quality.py protocol): 16 seeds, epochs 0-20
# and 99, bf16, 2 clients resampled to 20k rows each; plus 8-client whole rounds batched vs threads.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4q}
W=/tmp/fedtgan_quality
mkdir -p $OUT $W
S="--epochs 100 --seeds $(seq 0 15 | tr '\n' ' ') --bootstrap-rows 20000 --no-utility --precisions bf16 --only-scored-csv --eval-epochs $(seq 0 20 | tr '\n' ' ') 99"
timeout -k 10 700 python tools/real_quality.py $S --out $W/q > $OUT/quality.log 2>&1 && cp $W/q/real_quality.json $OUT/quality_r4.json && \
for b in on off; do
  timeout -k 10 200 python tools/run_config.py --spec intrusion --clients 8 --epochs 6 --batched $b --n-sample 40000 > $OUT/rounds8_$b.log 2>&1 || exit 1
done
echo "exit $?"
