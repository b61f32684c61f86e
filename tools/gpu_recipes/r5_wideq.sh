# Round 5: wide-table (100k x 512) training three ways -- torch oracle fp32, HIP fp32, HIP bf16 -- same seed,
# 5 epochs, metrics logs (losses per round); plus the Intrusion round-1 stall with cgroup CPU accounting.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5wideq}
mkdir -p $OUT
cd $R
python -c "from fed_tgan_amd.utils.metrics import cpu_quota, cgroup_cpu_stat; print(cpu_quota(), cgroup_cpu_stat())" > $OUT/cpu.txt 2>&1
timeout -k 10 150 python tools/run_config.py --spec intrusion --clients 1 --epochs 6 --fed metrics_log=$OUT/m_int.jsonl > $OUT/int.log 2>&1 || exit 1
W="python tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 5 --n-sample 10000 --json $OUT/wide.jsonl"
timeout -k 10 300 $W --precision bf16 --fed metrics_log=$OUT/m_bf16.jsonl > $OUT/w_bf16.log 2>&1 || exit 1
timeout -k 10 300 $W --precision fp32 --fed metrics_log=$OUT/m_fp32.jsonl > $OUT/w_fp32.log 2>&1 || exit 1
timeout -k 10 900 $W --precision fp32 --backend torch --fed metrics_log=$OUT/m_torch.jsonl > $OUT/w_torch.log 2>&1 || exit 1
echo done
