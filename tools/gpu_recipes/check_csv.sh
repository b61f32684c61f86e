# GPU tests, RCCL self-test, bench (20 and 5 rounds) and the epoch-CSV write probe.  Test failures
# (pytest exit 1) still let the measurements run; a crash, abort or time limit ends the script.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 170 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
[ $rc -le 1 ] && \
timeout -k 10 150 python tools/rccl_selftest.py > gpurun_out/rccl.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 5 --warmup 2 > gpurun_out/bench5.log 2>&1 && \
timeout -k 10 200 python tools/csv_probe.py > gpurun_out/csv_probe.txt 2>&1
echo "exit $? (pytest $rc)"
