# Round 5: Adult with EQUAL contiguous shards (2 clients x 8,000 rows, 4 epochs) -- is the epoch-0 gap of the Dirichlet run about unequal clients? trained by this
# framework -- HIP bf16 (8 seeds), HIP fp32 (4), the eager torch fp32 oracle (4) -- on the same client CSVs the
# reference's code trains on the CPU (tools/wide_quality.py --impl reference --spec adult --shard dirichlet).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5adulteq}
mkdir -p $OUT
cd $R
Q="python tools/wide_quality.py --impl ours --spec adult --shard contiguous --rows 8000 --clients 2 --epochs 4 --work /tmp/wqe --out $OUT/ours_adult_eq.jsonl"
timeout -k 10 300 $Q --backend hip --precision bf16 --seeds 0 1 2 3 4 5 6 7 > $OUT/bf16.log 2>&1 || exit 1
timeout -k 10 300 $Q --backend hip --precision fp32 --seeds 0 1 2 3 > $OUT/fp32.log 2>&1 || exit 1
timeout -k 10 600 $Q --backend torch --precision fp32 --seeds 0 1 2 3 > $OUT/torch.log 2>&1 || exit 1
echo done
