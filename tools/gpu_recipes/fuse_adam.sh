# EngineConfig.fuse_g_adam / fuse_d_adam: GPU engine + op tests, then the step A/Bs (separate launches vs fused)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_engine.py tests/test_hip_ops.py -x -v --timeout 120 --timeout-method thread > gpurun_out/fuse_tests.log 2>&1 && \
timeout -k 10 300 python tools/microbench.py --cfg-ab chain_d1 > gpurun_out/chain_ab.txt 2>&1 && \
timeout -k 10 300 python tools/microbench.py --cfg-ab fuse_g_adam > gpurun_out/fuse_ab.txt 2>&1
echo "exit $?"
