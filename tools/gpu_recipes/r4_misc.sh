# First-use D2H costs, then a kernel-trace breakdown of the wide-table step (current kernels).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4misc}
mkdir -p $OUT
cd $R
timeout -k 10 120 python tools/d2h_probe.py > $OUT/d2h.json 2>&1 || exit 1
cd /tmp
(cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_wide -o run -- python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 2 --n-sample 10000 > $OUT/prof_wide.log 2>&1) || exit 1
python3 $R/tools/step_breakdown.py $OUT/prof_wide/run_results.db > $OUT/wide_step_breakdown.txt 2>&1 || exit 1
rm -rf $OUT/prof_wide
echo done
