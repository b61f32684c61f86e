#!/bin/bash
# Column-ownership Linear+BN+ReLU: numerics tests, then the per-layer / full-step A/B.
set -o pipefail
mkdir -p gpurun_out/colown
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_bn_colown.py > gpurun_out/colown/tests.log 2>&1 &&
timeout -k 10 300 python -u tools/microbench.py --colown-ab > gpurun_out/colown/ab.txt 2>&1
