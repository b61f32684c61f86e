# Device (HIP) vs host (numpy) VGM encode: 24 more seeds each (8-31), epochs 0-2, bf16 -- does the encode
# move epoch-2 Avg_JSD (8-seed means: device 0.0686 +- 0.0017, host 0.0640 +- 0.0016)?
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3q3}
W=/tmp/fedtgan_quality
mkdir -p $OUT $W
SEEDS=$(seq 8 31 | tr '\n' ' ')
S="--epochs 3 --seeds $SEEDS --bootstrap-rows 20000 --no-utility --precisions bf16"
timeout -k 10 600 python tools/real_quality.py $S --host-encode --out $W/he > $OUT/host_encode.log 2>&1 && \
cp $W/he/real_quality.json $OUT/host_encode.json && \
timeout -k 10 600 python tools/real_quality.py $S --out $W/de > $OUT/device_encode.log 2>&1 && \
cp $W/de/real_quality.json $OUT/device_encode.json
echo "exit $?"
