#!/bin/bash
# Batched colown diff (where does a batched client first differ?), then the per-layer / full-step A/B.
set -o pipefail
mkdir -p gpurun_out/colown
timeout -k 10 200 python -u tools/batched_diff.py --k 2 --engine bn_colown=1 > gpurun_out/colown/diff.txt 2>&1 &&
timeout -k 10 200 python -u tools/batched_diff.py --k 2 > gpurun_out/colown/diff_base.txt 2>&1 &&
timeout -k 10 300 python -u tools/microbench.py --colown-ab > gpurun_out/colown/ab.txt 2>&1
