# Round 5: (first GPU process of the call) cold Intrusion initialisation with the three-thread kernel warm-up, then
# a warm one; GEMM op tests; wide table A/B of 128x128 tiles for the long-K D0 forward (LONG_K_128), two passes.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5cold2}
mkdir -p $OUT
cd $R
timeout -k 10 200 python tools/init_profile.py --spec intrusion --rows 40000 --cprofile --top 30 --json $OUT/init.jsonl > $OUT/init_cold.log 2>&1 || exit 1
timeout -k 10 200 python tools/init_profile.py --spec intrusion --rows 40000 --json $OUT/init.jsonl > $OUT/init_warm.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_ops.py -k gemm > $OUT/pytest_gemm.log 2>&1 || exit 1
W="python tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 2 --n-sample 10000"
for i in 1 2; do
  for v in "" "--plan LONG_K_128=1"; do
    timeout -k 10 200 $W $v 2>&1 | grep '"mean_sec_per_epoch_after_first"' >> $OUT/wide.jsonl || exit 1
  done
done
echo done
