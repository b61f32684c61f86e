# Round 6: hardware bf16 pack (v_cvt_pk_bf16_f32) + unchecked interior staging bursts in the GEMM body vs the previous
# build (ab/_C_prev.so, swapped in place), same box: GEMM / engine GPU tests on the new build first, then alternating
# Intrusion step microbench, the wide G.out probe and the Intrusion bench
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6aj
mkdir -p $OUT
cd $R
cp fed_tgan_amd/_C.so ab/_C_new.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_ops.py tests/test_gemm_shortk.py tests/test_hip_engine.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2 3; do
  for arm in new prev; do
    cp ab/_C_$arm.so fed_tgan_amd/_C.so
    timeout -k 10 120 python3 tools/microbench.py --step-only --epochs-only 2>&1 | grep "engine epoch" | sed "s/^/[$arm] /" >> $OUT/step.txt || exit 1
    timeout -k 10 120 python3 tools/gout_probe.py --only-gout --reps 50 2>&1 | tail -1 | sed "s/^/[$arm] /" >> $OUT/gout.txt || exit 1
  done
done
cat $OUT/step.txt $OUT/gout.txt
for i in 1 2; do
  for arm in new prev; do
    cp ab/_C_$arm.so fed_tgan_amd/_C.so
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 | sed "s/^/[$arm] /" >> $OUT/bench.jsonl || exit 1
  done
done
cp ab/_C_new.so fed_tgan_amd/_C.so
python3 -c "
import json
for l in open('$OUT/bench.jsonl'):
    t, j = l.split('] ', 1); d = json.loads(j); print(t + ']', d['ms_per_step'], d['phase_s']['train'], d['avg_jsd'])
"
