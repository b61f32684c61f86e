set -o pipefail
mkdir -p gpurun_out
J=gpurun_out/configs_r2.jsonl
rm -f $J
timeout -k 10 300 python -u tools/run_config.py --spec adult --rows 8000 --clients 8 --shard dirichlet --alpha 0.3 --epochs 5 --json $J > gpurun_out/cfg_adult.log 2>&1 && \
timeout -k 10 300 python -u tools/run_config.py --spec intrusion --rows 40000 --clients 8 --epochs 4 --json $J > gpurun_out/cfg_intr8.log 2>&1 && \
timeout -k 10 300 python -u tools/run_config.py --spec covertype --rows 20000 --clients 8 --shard dirichlet --alpha 0.3 --epochs 5 --json $J > gpurun_out/cfg_cov.log 2>&1 && \
timeout -k 10 400 python -u tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 3 --n-sample 10000 --json $J > gpurun_out/cfg_wide.log 2>&1
echo "exit $?"
