# Wide rows: row-kernel + one-hot weight-gradient numerics (pytest), then the wide table: round-3 kernels
# (LDS-image row kernels, dense one-hot gradients) vs each new path.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4wide4}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_ops.py tests/test_hip_engine.py -k "wide or onehot or autograd" > $OUT/pytest.log 2>&1 || exit 1
W="python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 2 --n-sample 10000"
for v in "--tuning act_row_mode=1 --engine onehot_wgrad_min=0" "--engine onehot_wgrad_min=0" "" "--tuning gemm_pair_max_wg=2048"; do
  timeout -k 10 200 $W $v 2>&1 | grep '"mean_sec_per_epoch_after_first"' >> $OUT/wide.jsonl || exit 1
done
cd /tmp
(cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_wide -o run -- python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 2 --n-sample 10000 > $OUT/prof_wide.log 2>&1) || exit 1
python3 $R/tools/step_breakdown.py $OUT/prof_wide/run_results.db > $OUT/wide_step_breakdown.txt 2>&1 || exit 1
rm -rf $OUT/prof_wide
echo done
