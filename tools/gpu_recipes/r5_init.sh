# Round 5: federated initialisation per stage (tools/init_profile.py) -- Intrusion (first process on the box: cold,
# then warm), wide 100k x 512 from the synthetic generator and from a CSV (arrow and pandas readers).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5init}
mkdir -p $OUT
cd $R
I="python tools/init_profile.py --json $OUT/init.jsonl"
timeout -k 10 200 $I --spec intrusion --rows 40000 > $OUT/int_cold.log 2>&1 || exit 1
timeout -k 10 200 $I --spec intrusion --rows 40000 > $OUT/int_warm.log 2>&1 || exit 1
timeout -k 10 300 $I --spec wide --rows 100000 > $OUT/wide_syn.log 2>&1 || exit 1
timeout -k 10 300 $I --spec wide --rows 100000 --source csv --reader arrow > $OUT/wide_arrow.log 2>&1 || exit 1
timeout -k 10 300 $I --spec wide --rows 100000 --source csv --reader pandas > $OUT/wide_pandas.log 2>&1 || exit 1
timeout -k 10 300 $I --spec wide --rows 100000 --cprofile --top 25 > $OUT/wide_cprofile.log 2>&1 || exit 1
echo done
