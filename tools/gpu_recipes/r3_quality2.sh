# Avg_JSD / Avg_WD at epochs 0-2, 8 seeds: the two ablations round 3 had not run yet -- sklearn VGM fits
# (-gmm sklearn, the reference's BayesianGaussianMixture) and host VGM encode (numpy, not the HIP kernel).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3q2}
W=/tmp/fedtgan_quality
mkdir -p $OUT $W
S="--epochs 3 --seeds 0 1 2 3 4 5 6 7 --bootstrap-rows 20000 --no-utility --precisions bf16"
timeout -k 10 400 python tools/real_quality.py $S --gmm sklearn --out $W/sk > $OUT/sklearn.log 2>&1 && \
cp $W/sk/real_quality.json $OUT/sklearn.json && \
timeout -k 10 300 python tools/real_quality.py $S --host-encode --out $W/he > $OUT/host_encode.log 2>&1 && \
cp $W/he/real_quality.json $OUT/host_encode.json
echo "exit $?"
