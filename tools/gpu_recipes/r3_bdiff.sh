set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3i}
mkdir -p $OUT
timeout -k 10 200 python tools/batched_diff.py --k 1 > $OUT/diff_k1.log 2>&1 && \
timeout -k 10 200 python tools/batched_diff.py --k 2 > $OUT/diff_k2.log 2>&1 && \
timeout -k 10 200 python tools/batched_diff.py --k 2 --precision fp32 > $OUT/diff_k2_fp32.log 2>&1
echo "exit $?"
