# Round 5: wide 100k x 512, 5 epochs: torch oracle (eager, fp32) vs HIP fp32 vs HIP bf16, seeds 0-2 each;
# (torch oracle: seeds 0-1)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5wideq2}
mkdir -p $OUT
cd $R
W="python tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 5 --n-sample 10000 --json $OUT/wide.jsonl"
for s in 0 1 2; do
  timeout -k 10 200 $W --seed $s --precision bf16 > $OUT/w_bf16_$s.log 2>&1 || exit 1
  timeout -k 10 200 $W --seed $s --precision fp32 > $OUT/w_fp32_$s.log 2>&1 || exit 1
done
for s in 0 1; do
  timeout -k 10 600 python -X faulthandler tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 5 --n-sample 10000 --json $OUT/wide.jsonl --seed $s --precision fp32 --backend torch --fed metrics_log=$OUT/m_torch_$s.jsonl > $OUT/w_torch_$s.log 2>&1 || exit 1
done
echo done
