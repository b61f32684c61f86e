# Kernel trace of the 8-client batched step (current build), and the one-client bench line.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4prof8}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_b8 -o run -- python3 tools/batched_probe.py --profile-k 8 --reps 6 > $OUT/prof_b8.log 2>&1 && \
python3 tools/step_breakdown.py $OUT/prof_b8/run_results.db > $OUT/step_breakdown_b8.txt 2>&1 && rm -f $OUT/prof_b8/run_results.db && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_federation.py -m gpu -v --timeout 240 --timeout-method thread -k "broadcast_init" > $OUT/pytest.log 2>&1
echo "exit $?"
