# EngineConfig.g_wt A/B: GPU tests of the layout, the Intrusion step / generation microbenchmark, and the
# wide 100k x 512 config end to end with each layout (sec/epoch)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_engine.py tests/test_engine_grad.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gwt_tests.log 2>&1 && \
timeout -k 10 300 python tools/microbench.py --gwt-ab > gpurun_out/gwt_ab.txt 2>&1 && \
timeout -k 10 300 python tools/run_config.py --spec wide --rows 100000 --epochs 3 --json gpurun_out/gwt_wide.jsonl > gpurun_out/gwt_wide0.log 2>&1 && \
timeout -k 10 300 python tools/run_config.py --spec wide --rows 100000 --epochs 3 --engine g_wt=1 --json gpurun_out/gwt_wide.jsonl > gpurun_out/gwt_wide1.log 2>&1
echo "exit $?"
