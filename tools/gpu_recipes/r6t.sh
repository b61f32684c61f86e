# Round 6: after deleting the BN-fold variants -- engine / batched / checked GPU tests, the wide-table GEMM probes
# (tools/gout_probe.py) and a bench
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6t
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_hip_engine.py tests/test_batched.py tests/test_gpu_checked.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 180 python3 tools/gout_probe.py > $OUT/probe.txt 2>&1 || { cat $OUT/probe.txt; exit 1; }
cat $OUT/probe.txt
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit 1
tail -1 $OUT/bench.log
