# Round 3 re-entry: GPU tests + smoke + bench on the rebuilt .so, the colown per-layer / full-step A/B, then a
# kernel trace of the current 8-client batched step.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3s}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 170 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "pytest exit $?"
timeout -k 10 100 python -c "import __graft_entry__ as e; e.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 && \
timeout -k 10 300 python -u tools/microbench.py --colown-ab > $OUT/colown_ab.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_b8 -o run -- python3 tools/batched_probe.py --profile-k 8 --reps 6 > $OUT/prof_b8.log 2>&1 && \
python3 tools/step_breakdown.py $OUT/prof_b8/run_results.db > $OUT/step_breakdown_b8.txt 2>&1 && rm -f $OUT/prof_b8/run_results.db
echo "exit $?"
