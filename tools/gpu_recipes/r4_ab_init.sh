# Same box: one-client step, round-3 tree vs HEAD with the global-RNG init vs HEAD with the per-engine init.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4abinit}
mkdir -p $OUT
for i in 1 2; do
  (cd $R/_basetree && timeout -k 10 150 python tools/microbench.py --step-only >> $OUT/base_step.txt 2>&1) || break
  (cd $R && timeout -k 10 150 python tools/microbench.py --step-only --init-rng global >> $OUT/head_global_step.txt 2>&1) || break
  (cd $R && timeout -k 10 150 python tools/microbench.py --step-only --init-rng engine >> $OUT/head_engine_step.txt 2>&1) || break
done
echo "exit $?"
