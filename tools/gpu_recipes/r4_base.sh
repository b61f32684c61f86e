# Round-4 starting point: batched K sweep, kernel traces of the 8-client batched step and of the wide
# 100k x 512 table, and the bench line, all from one box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4base}
mkdir -p $OUT
timeout -k 10 300 python tools/batched_probe.py --ks 1 2 4 8 --skip-plain --reps 4 > $OUT/batched_probe.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_b8 -o run -- python3 tools/batched_probe.py --profile-k 8 --reps 6 > $OUT/prof_b8.log 2>&1 && \
python3 tools/step_breakdown.py $OUT/prof_b8/run_results.db > $OUT/step_breakdown_b8.txt 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_wide -o run -- python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 3 > $OUT/prof_wide.log 2>&1 && \
python3 tools/step_breakdown.py $OUT/prof_wide/run_results.db > $OUT/step_breakdown_wide.txt 2>&1 && \
rm -f $OUT/prof_b8/run_results.db $OUT/prof_wide/run_results.db && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1
echo "exit $?"
