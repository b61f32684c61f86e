# Round 5: the split VGM fit (a cluster of workgroups per column, csrc/kernels/vgm_fit.hip) -- parity tests, the
# fit-time A/B (tools/vgm_split_bench.py), the Intrusion init per stage (cold then warm) and the bench.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5vgm}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_vgm_parity.py > $OUT/tests.log 2>&1 || exit 1
I="python tools/init_profile.py --json $OUT/init.jsonl"
timeout -k 10 200 $I --spec intrusion --rows 40000 > $OUT/int_a.log 2>&1 || exit 1
timeout -k 10 200 $I --spec intrusion --rows 40000 > $OUT/int_b.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/vgm_split_bench.py > $OUT/bench_vgm.jsonl 2>&1 || exit 1
timeout -k 10 300 $I --spec wide --rows 100000 > $OUT/wide_syn.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit 1
echo done
