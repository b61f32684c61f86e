# bench regression diagnosis 2: event timers vs a host wait after the local epoch, CSV thread counts.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3d2}
mkdir -p $OUT
B="timeout -k 10 200 python bench.py --steps 20 --warmup 5"
$B > $OUT/a_default.log 2>&1 && \
$B --fed train_sync=1 > $OUT/b_trainsync.log 2>&1 && \
$B --fed csv_threads=8 > $OUT/c_csv8.log 2>&1 && \
$B --fed csv_threads=4 > $OUT/d_csv4.log 2>&1 && \
$B --fed train_sync=1 --fed csv_threads=8 > $OUT/e_ts_csv8.log 2>&1 && \
$B --no-eval > $OUT/f_noeval.log 2>&1 && \
$B --phase-timer sync > $OUT/g_ptsync.log 2>&1
echo "exit $?"
