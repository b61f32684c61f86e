# Round 6: ATen-free initialisation -- cold first-process init profile first, then the init-op / VGM / federation
# tests and a bench
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6o
mkdir -p $OUT
cd $R
timeout -k 10 120 python tools/init_profile.py --cprofile --top 40 --json $OUT/init.jsonl > $OUT/init_cold.log 2>&1 || exit 1
timeout -k 10 120 python tools/init_profile.py --json $OUT/init.jsonl > $OUT/init_warm.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_init_ops.py tests/test_vgm_parity.py tests/test_gpu_federation.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit 1
echo done
