# Round 6: BN-backward pairing (EngineConfig.bn_pair): engine tests, step A/B, plus the exit-crash diagnostics
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6i
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_hip_engine.py tests/test_engine_grad.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || exit 1
for rep in 1 2; do
for cfg in "bn_pair=1" "bn_pair=0"; do
  timeout -k 10 120 python3 tools/microbench.py --step-only --epochs-only --engine $cfg 2>&1 | grep "engine epoch" | sed "s/^/[$cfg] /" >> $OUT/ab.txt || exit 1
done
done
bash tools/gpu_recipes/r6h.sh
echo done
