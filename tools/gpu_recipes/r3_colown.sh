#!/bin/bash
# Column-ownership Linear+BN+ReLU: numerics tests (+ batched twins), the per-layer / full-step
# A/B, then kernel times under rocprofv3.
set -o pipefail
mkdir -p gpurun_out/colown gpurun_out/colown_prof
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_bn_colown.py tests/test_batched.py > gpurun_out/colown/tests.log 2>&1 &&
timeout -k 10 300 python -u tools/microbench.py --colown-ab > gpurun_out/colown/ab.txt 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/colown_prof/raw -o run -- python3 tools/microbench.py --colown-ab > gpurun_out/colown_prof/out.txt 2>&1 &&
find gpurun_out/colown_prof/raw -name "*kernel_stats.csv" -exec cp {} gpurun_out/colown_prof/kernel_stats.csv \; &&
rm -rf gpurun_out/colown_prof/raw
