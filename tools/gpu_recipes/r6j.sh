# Round 6: BN-backward pairing layouts (bnb_first x bnb_cols) vs no pairing, epoch-graph step time
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6j
mkdir -p $OUT
cd $R
for rep in 1 2; do
for cfg in "--engine bn_pair=0" "--engine bn_pair=1 --tuning bnb_first=1 --tuning bnb_cols=4" "--engine bn_pair=1 --tuning bnb_first=0 --tuning bnb_cols=4" "--engine bn_pair=1 --tuning bnb_first=1 --tuning bnb_cols=8" "--engine bn_pair=1 --tuning bnb_first=0 --tuning bnb_cols=8"; do
  timeout -k 10 120 python3 tools/microbench.py --step-only --epochs-only $cfg 2>&1 | grep "engine epoch" | sed "s/^/[$cfg] /" >> $OUT/ab.txt || exit 1
done
done
echo done
