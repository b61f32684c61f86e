# Span-parallel row kernels (tests + wide A/B), 8 clients batched vs threads after the init warm-ups, bench A/B.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4r6}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_ops.py tests/test_hip_engine.py -k "wide or onehot or activ or act_bwd or sample" > $OUT/pytest.log 2>&1 || exit 1
W="python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 2 --n-sample 10000"
for v in "--tuning act_row_mode=1" ""; do
  timeout -k 10 200 $W $v 2>&1 | grep '"mean_sec_per_epoch_after_first"' >> $OUT/wide.jsonl || exit 1
done
RC="python tools/run_config.py --spec intrusion --clients 8 --epochs 8"
timeout -k 10 150 $RC --batched on --fed metrics_log=$OUT/m_on.jsonl > $OUT/on.log 2>&1 || exit 1
timeout -k 10 150 $RC --batched off --fed metrics_log=$OUT/m_off.jsonl > $OUT/off.log 2>&1 || exit 1
for i in 1 2 3; do
  (cd $R/_basetree && timeout -k 10 150 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 >> $OUT/base_bench.jsonl) || exit 1
  (cd $R && timeout -k 10 150 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 >> $OUT/head_bench.jsonl) || exit 1
done
echo done
