# Round 3: GPU tests, smoke, bench (plain and over a one-rank RCCL communicator), with the new
# self-verification fields (comm record, event-timed phases).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 170 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 100 python -c "import __graft_entry__ as e; e.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 && \
timeout -k 10 200 python bench.py --force-dist --steps 20 --warmup 5 > $OUT/bench_rccl1.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench2.log 2>&1 && \
timeout -k 10 200 python bench.py --force-dist --steps 20 --warmup 5 > $OUT/bench_rccl1_2.log 2>&1
echo "exit $?"
