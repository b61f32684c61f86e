#!/bin/bash
# Initialisation time: 1 client via bench.py, 8 clients via run_config (batched off / auto).
set -o pipefail
mkdir -p gpurun_out/init
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/init/bench1.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/init/bench1b.log 2>&1 &&
timeout -k 10 300 python -u tools/run_config.py --clients 8 --epochs 2 --batched off > gpurun_out/init/c8.log 2>&1 &&
timeout -k 10 300 python -u tools/run_config.py --clients 4 --epochs 2 > gpurun_out/init/c4.log 2>&1
