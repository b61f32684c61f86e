# Round 5 end: per-kernel totals of bench.py under rocprofv3 --kernel-trace on the final build (split VGM fit).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5benchprof}
mkdir -p $OUT
cd /tmp
(cd $R && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/bench -o run -- python3 bench.py --steps 5 --warmup 2 > $OUT/bench_prof.log 2>&1) || exit 1
python3 $R/tools/prof_summary.py $OUT/bench/run_results.db > $OUT/bench_kernels.txt 2>&1 || true
rm -rf $OUT/bench
echo done
