# Batched engine: tests, K sweep with planning on/off, and a kernel trace of the 8-client step.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3m}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_batched.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/pytest_batched.log 2>&1 && \
timeout -k 10 400 python tools/batched_probe.py --plan both > $OUT/batched_probe.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_b8 -o run -- python3 tools/batched_probe.py --profile-k 8 --reps 6 > $OUT/prof_b8.log 2>&1 && \
python3 tools/step_breakdown.py $OUT/prof_b8/run_results.db > $OUT/step_breakdown_b8.txt 2>&1
echo "exit $?"
