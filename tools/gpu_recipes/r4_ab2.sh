# Same box: one-client step + bench, round-3 tree vs HEAD; then HEAD's batched 4 / 8 clients with xcd_clients 0 / 1.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4ab2}
mkdir -p $OUT
bash $R/tools/gpu_recipes/r4_ab1.sh ${1:-r4ab2} > /dev/null 2>&1
cd $R
for x in 0 1; do
  timeout -k 10 150 python tools/batched_probe.py --ks 4 8 --skip-plain --reps 4 --tuning xcd_clients=$x > $OUT/probe_x$x.log 2>&1 || break
done
timeout -k 10 400 python -u -m pytest tests/test_batched.py tests/test_gpu_federation.py tests/test_hip_ops.py -m gpu -q -x --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
echo "exit $?"
