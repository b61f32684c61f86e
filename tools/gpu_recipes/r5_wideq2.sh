# Round 5: wide 100k x 512, 5 epochs: torch oracle (eager, fp32) vs HIP fp32 vs HIP bf16, seeds 0-2 each;
# Intrusion round 0 after init-time graph capture (metrics log) and a 2-epoch CLI run's timestamp_experiment.csv.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5wideq2}
mkdir -p $OUT
cd $R
timeout -k 10 150 python tools/run_config.py --spec intrusion --clients 1 --epochs 6 --fed metrics_log=$OUT/m_int.jsonl > $OUT/int.log 2>&1 || exit 1
mkdir -p $OUT/cli && (cd $OUT/cli && timeout -k 10 150 python -m dtds.distributed -world_size 1 -colocated -epochs 2 > cli.log 2>&1) || exit 1
(cd $OUT/cli && timeout -k 10 150 python -m dtds.distributed -world_size 1 -colocated -epochs 4 > cli4.log 2>&1 && cp timestamp_experiment.csv ts4.csv) || exit 1
W="python tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 5 --n-sample 10000 --json $OUT/wide.jsonl"
for s in 0 1 2; do
  timeout -k 10 200 $W --seed $s --precision bf16 > $OUT/w_bf16_$s.log 2>&1 || exit 1
  timeout -k 10 200 $W --seed $s --precision fp32 > $OUT/w_fp32_$s.log 2>&1 || exit 1
done
for s in 0 1 2; do
  timeout -k 10 600 python -X faulthandler tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 5 --n-sample 10000 --json $OUT/wide.jsonl --seed $s --precision fp32 --backend torch --fed metrics_log=$OUT/m_torch_$s.jsonl > $OUT/w_torch_$s.log 2>&1 || exit 1
done
echo done
