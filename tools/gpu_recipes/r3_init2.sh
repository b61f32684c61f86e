#!/bin/bash
# Init after the device pool / warm thread changes: profile (cold), bench x2, 4 and 8 clients.
set -o pipefail
mkdir -p gpurun_out/init2
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_stats.py tests/test_vgm_parity.py > gpurun_out/init2/tests.log 2>&1 &&
timeout -k 10 200 python -u tools/init_profile.py --top 40 > gpurun_out/init2/prof.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/init2/bench1.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/init2/bench1b.log 2>&1 &&
timeout -k 10 300 python -u tools/run_config.py --clients 8 --epochs 2 --batched off > gpurun_out/init2/c8.log 2>&1 &&
timeout -k 10 300 python -u tools/run_config.py --clients 4 --epochs 2 > gpurun_out/init2/c4.log 2>&1
