# Wide 100k x 512 with the current build (unrolled Adam): fused vs unfused optimizer launches, kernel trace of the
# better one.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4wide}
mkdir -p $OUT
W="python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 3"
timeout -k 10 300 $W --json $OUT/wide.jsonl > $OUT/wide_fused.log 2>&1 && \
timeout -k 10 300 $W --engine fuse_adam_max=4000000 --json $OUT/wide.jsonl > $OUT/wide_unfused.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_wide -o run -- $W --engine fuse_adam_max=4000000 > $OUT/prof_wide.log 2>&1 && \
python3 tools/step_breakdown.py $OUT/prof_wide/run_results.db > $OUT/step_breakdown_wide_unfused.txt 2>&1 && \
rm -f $OUT/prof_wide/run_results.db
echo "exit $?"
