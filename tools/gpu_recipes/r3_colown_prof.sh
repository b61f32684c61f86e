#!/bin/bash
# Kernel times of the colown A/B (rocprofv3 kernel trace + stats).
set -o pipefail
mkdir -p gpurun_out/colown_prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/colown_prof/raw -o run -- python3 tools/microbench.py --colown-ab > gpurun_out/colown_prof/out.txt 2>&1 &&
find gpurun_out/colown_prof/raw -name "*kernel_stats.csv" -exec cp {} gpurun_out/colown_prof/kernel_stats.csv \; &&
rm -rf gpurun_out/colown_prof/raw
