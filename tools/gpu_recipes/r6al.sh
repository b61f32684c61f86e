# Round 6: 128x128-tile fp32 output epilogue as column-quad 16-B stores vs the previous build (ab/_C_prev.so, swapped in
# place), same box: GEMM / engine GPU tests on the new build, then the wide G.out probe and the wide epoch, alternating
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6al
mkdir -p $OUT
cd $R
cp fed_tgan_amd/_C.so ab/_C_new.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_ops.py tests/test_gemm_shortk.py tests/test_hip_engine.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2 3; do
  for arm in new prev; do
    cp ab/_C_$arm.so fed_tgan_amd/_C.so
    timeout -k 10 120 python3 tools/gout_probe.py --only-gout --reps 50 2>&1 | tail -1 | sed "s/^/[$arm] /" >> $OUT/gout.txt || exit 1
  done
done
cat $OUT/gout.txt
W="python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 4 --n-sample 10000"
for i in 1 2; do
  for arm in new prev; do
    cp ab/_C_$arm.so fed_tgan_amd/_C.so
    timeout -k 10 200 $W 2>&1 | grep '"mean_sec_per_epoch_after_first"' | sed "s/^/[$arm] /" >> $OUT/wide.jsonl || exit 1
  done
done
cp ab/_C_new.so fed_tgan_amd/_C.so
python3 -c "
import json
for l in open('$OUT/wide.jsonl'):
    t, j = l.split('] ', 1); print(t + ']', json.loads(j)['mean_sec_per_epoch_after_first'])
"
