# bench regression diagnosis: repeat runs, in-round CSV, synchronised phase timers, per-phase round probe.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3d}
mkdir -p $OUT
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench1.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --sync-csv > $OUT/bench_sync.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --phase-timer sync > $OUT/bench_ptsync.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench2.log 2>&1 && \
timeout -k 10 200 python tools/round_probe.py > $OUT/round_probe.log 2>&1
echo "exit $?"
