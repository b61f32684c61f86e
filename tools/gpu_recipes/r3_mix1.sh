# bench with the host wait after training (default now), wide table dW0 tile A/B (planner: 128-tiles once
# clients x 128-tiles >= 256), 8-client Intrusion rounds batched vs threads, then the 8-client PMC passes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3m1}
mkdir -p $O
J=$O/configs.jsonl
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 && \
timeout -k 10 400 python -u tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 3 --n-sample 10000 --json $J > $O/wide.log 2>&1 && \
timeout -k 10 400 python -u tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 3 --n-sample 10000 --engine dw0_tile=64 --json $J > $O/wide64.log 2>&1 && \
timeout -k 10 300 python -u tools/run_config.py --spec intrusion --rows 40000 --clients 8 --epochs 6 --batched on --json $J > $O/intr8_b.log 2>&1 && \
timeout -k 10 300 python -u tools/run_config.py --spec intrusion --rows 40000 --clients 8 --epochs 6 --batched off --json $J > $O/intr8_t.log 2>&1 && \
bash tools/gpu_recipes/r3_pmc_b8.sh r3m1/pmc_b8
echo "exit $?"
