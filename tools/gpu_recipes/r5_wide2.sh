# Round 5: wide-layout engine tests vs autograd; torch-backend wide crash (faulthandler); init stages.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5wide2}
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_hip_engine.py -k "autograd" > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 200 python tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 2 --n-sample 10000 > $OUT/w_hip.log 2>&1 || exit 1
timeout -k 10 400 python -X faulthandler tools/run_config.py --spec wide --rows 20000 --clients 1 --epochs 1 --n-sample 2000 --backend torch --precision fp32 > $OUT/w_torch.log 2>&1
echo "torch rc=$?" >> $OUT/w_torch.log
echo done
