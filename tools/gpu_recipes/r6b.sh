mkdir -p gpurun_out/r6b
bash tools/gpu_session.sh \
 "300|r6b/mdtest|python -u -m pytest tests/test_hip_engine.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'multi_draw or streams or large_batches'" \
 "120|r6b/bench1|python bench.py --steps 20 --warmup 5" \
 "120|r6b/bench_nomulti|python bench.py --steps 20 --warmup 5 --engine multi_draw=0" \
 "400|r6b/vgmfit|python -u tools/vgm_fit_ab.py --seeds 30 --out gpurun_out/r6b/vgmfit.jsonl"
