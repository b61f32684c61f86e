# Round 6: first-process init profile (cold box), bench under rocprofv3 (exit status after the tool's finalisation),
# step breakdown of the engine's own epoch graphs (multi-step sampler draw) in kernel order
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6e
mkdir -p $OUT
cd $R
timeout -k 10 120 python tools/init_profile.py --cprofile --top 45 --json $OUT/init.jsonl > $OUT/init_cold.log 2>&1 || exit 1
timeout -k 10 120 python tools/init_profile.py --json $OUT/init.jsonl > $OUT/init_warm.log 2>&1 || exit 1
cd /tmp
(cd $R && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/bench -o run -- python3 bench.py --steps 5 --warmup 2 > $OUT/bench_prof.log 2>&1); echo "bench under rocprofv3: exit $?" >> $OUT/exit.txt
python3 $R/tools/prof_summary.py $OUT/bench/run_results.db > $OUT/bench_kernels.txt 2>&1 || true
rm -rf $OUT/bench
(cd $R && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/step -o run -- python3 tools/microbench.py --step-only --epochs-only > $OUT/step.log 2>&1) || exit 1
python3 $R/tools/step_breakdown.py $OUT/step/run_results.db --order > $OUT/step_breakdown.txt 2>&1 || exit 1
rm -rf $OUT/step
echo done
