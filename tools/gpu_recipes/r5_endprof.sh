# Round 5, end-of-round records: critical path per kernel of the captured step (final build), per-kernel totals of
# a bench run, counters of the GEMM + Adam launches (unrolled Adam), and the wide table's s/epoch.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5endprof}
mkdir -p $OUT
cd /tmp
(cd $R && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/step -o run -- python3 tools/microbench.py --step-only > $OUT/step.log 2>&1) || exit 1
python3 $R/tools/step_breakdown.py $OUT/step/run_results.db > $OUT/step_breakdown.txt 2>&1 || exit 1
rm -rf $OUT/step
(cd $R && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/bench -o run -- python3 bench.py --steps 5 --warmup 2 > $OUT/bench_prof.log 2>&1) || exit 1
python3 $R/tools/prof_summary.py $OUT/bench/run_results.db > $OUT/bench_kernels.txt 2>&1 || true
rm -rf $OUT/bench
K="gemm_adam"
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU" "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd $R && timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "$K" --output-format csv -d $OUT/p$i -o run -- python3 tools/microbench.py --step-only > $OUT/p$i.log 2>&1) || exit 1
done
python3 $R/tools/pmc_summary.py $OUT/p1 $OUT/p2 $OUT/p3 --out=$OUT/pmc_adam.txt > /dev/null 2>&1 || exit 1
rm -rf $OUT/p1 $OUT/p2 $OUT/p3
cd $R
W="python tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 3 --n-sample 10000"
for i in 1 2; do
  timeout -k 10 200 $W 2>&1 | grep '"mean_sec_per_epoch_after_first"' >> $OUT/wide.jsonl || exit 1
done
echo done
