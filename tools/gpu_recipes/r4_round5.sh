# Current build: one-client step vs the round-3 tree (same box), batched K = 4 / 8, the wide table, PMC of the
# 8-client step.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4r5}
mkdir -p $OUT
cd $R
for i in 1 2; do
  (cd $R/_basetree && timeout -k 10 150 python tools/microbench.py --step-only >> $OUT/base_step.txt 2>&1) || exit 1
  (cd $R && timeout -k 10 150 python tools/microbench.py --step-only >> $OUT/head_step.txt 2>&1) || exit 1
done
timeout -k 10 150 python tools/batched_probe.py --ks 4 8 --skip-plain --reps 4 > $OUT/probe.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 2 --n-sample 10000 > $OUT/wide.log 2>&1 || exit 1
bash tools/gpu_recipes/r3_pmc_b8.sh ${1:-r4r5}/pmc_b8 > /dev/null 2>&1
echo "exit $?"
