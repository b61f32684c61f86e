# Round 6: after the VGM fit's plain launch -- VGM tests, bench under rocprofv3 (exit status) + per-kernel totals
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6n
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_vgm_parity.py tests/test_gpu_engine.py tests/test_gpu_federation.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || exit 1
cd /tmp
(cd $R && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/bench -o run -- python3 bench.py --steps 5 --warmup 2 > $OUT/bench_prof.log 2>&1); echo "bench under rocprofv3 --kernel-trace --stats: exit $?" >> $OUT/exit.txt
python3 $R/tools/prof_summary.py $OUT/bench/run_results.db > $OUT/bench_kernels.txt 2>&1 || true
rm -rf $OUT/bench
echo done
