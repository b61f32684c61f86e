# Round 6: wide-table GEMM probes in isolation (tools/gout_probe.py): G.out forward variants, dW0, D-phase D0 forward
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6s
mkdir -p $OUT
cd $R
timeout -k 10 180 python3 tools/gout_probe.py > $OUT/probe.txt 2>&1 || { cat $OUT/probe.txt; exit 1; }
cat $OUT/probe.txt
