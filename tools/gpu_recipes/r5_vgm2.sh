# Round 5: the split VGM fit with one exp per component in the E-step -- parity tests, fit time over splits
# (1, auto, 2, 16), the Intrusion init per stage (cold then warm).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5vgm2}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_vgm_parity.py > $OUT/tests.log 2>&1 || exit 1
I="python tools/init_profile.py --json $OUT/init.jsonl"
timeout -k 10 200 $I --spec intrusion --rows 40000 > $OUT/int_a.log 2>&1 || exit 1
timeout -k 10 200 $I --spec intrusion --rows 40000 > $OUT/int_b.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/vgm_split_bench.py --splits ${SPLITS:-1,0,2,16} > $OUT/bench_vgm.jsonl 2>&1 || exit 1
echo done
