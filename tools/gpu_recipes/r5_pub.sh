# Round 5: BatchNorm fold with published statistics (EngineConfig.bn_fold_publish) -- fold tests, step A/B
# (fold off / fold + publish, twice; fold without publish once), per-kernel critical path of the folded step.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5pub}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_engine.py -k "bn_fold" > $OUT/pytest_fold.log 2>&1 || exit 1
timeout -k 10 200 python tools/microbench.py --cfg-ab bn_fold >> $OUT/step_ab.txt 2>&1 || exit 1
timeout -k 10 200 python tools/microbench.py --cfg-ab bn_fold >> $OUT/step_ab.txt 2>&1 || exit 1
timeout -k 10 200 python tools/microbench.py --cfg-ab bn_fold --engine bn_fold_publish=0 >> $OUT/step_ab_nopub.txt 2>&1 || exit 1
echo done
