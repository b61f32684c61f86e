# Round 5: the reduced wide table (wide:128, 2 clients x 20,000 rows, 12 epochs) with this framework -- HIP bf16 and
# fp32 with every wide-only kernel path forced, and the eager torch oracle -- for tools/wide_quality.py's comparison
# with the reference's own code (run on the CPU: profiles/wide_quality_ref_r5.jsonl).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5wideq3}
mkdir -p $OUT
cd $R
WQ="python tools/wide_quality.py --impl ours --cols 128 --rows 20000 --epochs 12 --work /tmp/wq --out $OUT/ours.jsonl"
timeout -k 10 500 $WQ --backend hip --precision bf16 --force-wide --seeds 0 1 2 3 4 5 6 7 > $OUT/hip_bf16.log 2>&1 || exit 1
timeout -k 10 300 $WQ --backend hip --precision fp32 --force-wide --seeds 0 1 2 3 > $OUT/hip_fp32.log 2>&1 || exit 1
timeout -k 10 700 $WQ --backend torch --precision fp32 --seeds 0 1 2 3 > $OUT/torch.log 2>&1 || exit 1
echo done
