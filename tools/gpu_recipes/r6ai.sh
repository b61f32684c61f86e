# Round 6: M-fastest XCD tile order (gemm_xcd_nmajor) -- the wide table's G.out GEMM in isolation and the wide epoch,
# alternating 1 / 0 on one box; the Intrusion bench (never takes the order) as a no-change check
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6ai
mkdir -p $OUT
cd $R
for i in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 120 python3 tools/gout_probe.py --only-gout --reps 50 --tuning gemm_xcd_nmajor=$v 2>&1 | tail -1 | sed "s/^/[nmajor=$v] /" >> $OUT/gout.txt || exit 1
  done
done
cat $OUT/gout.txt
W="python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 4 --n-sample 10000"
for i in 1 2; do
  for v in 1 0; do
    timeout -k 10 200 $W --tuning gemm_xcd_nmajor=$v 2>&1 | grep '"mean_sec_per_epoch_after_first"' | sed "s/^/[nmajor=$v] /" >> $OUT/wide.jsonl || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/wide.jsonl'):
    t, j = l.split('] ', 1); print(t + ']', json.loads(j)['mean_sec_per_epoch_after_first'])
"
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 > $OUT/bench.jsonl || exit 1
cat $OUT/bench.jsonl
