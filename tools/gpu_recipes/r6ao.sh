# Round 6 final tree after the generation-epilogue revert: bounds-checked library tests, GEMM tests and smoke()
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6ao
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_checked.py tests/test_hip_ops.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
