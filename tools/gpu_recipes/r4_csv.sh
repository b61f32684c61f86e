# Native CSV writer timings on the box (fresh process per setting): first vs later 40k-row writes, thread counts.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4csv}
mkdir -p $OUT
cd $R
for t in 0 8 4; do
  timeout -k 10 60 python tools/csv_probe.py --threads $t >> $OUT/csv.jsonl 2>&1 || exit 1
  timeout -k 10 60 python tools/csv_probe.py --threads $t --warm-rows 8192 >> $OUT/csv.jsonl 2>&1 || exit 1
done
nproc >> $OUT/csv.jsonl
echo done
