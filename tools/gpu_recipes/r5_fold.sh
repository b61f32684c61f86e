# Round 5: BatchNorm folded into the generator GEMMs (EngineConfig.bn_fold) -- GPU tests, step A/B, bench A/B;
# round-0 cost after init-time graph capture; 2- and 4-epoch CLI runs (timestamp_experiment.csv).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5fold}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_engine.py > $OUT/pytest_engine.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
if [ $rc -ge 124 ]; then exit 1; fi      # a hang / abort / fault: nothing more on the GPU (assertion failures go on)
timeout -k 10 200 python tools/microbench.py --cfg-ab bn_fold >> $OUT/step_ab.txt 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 >> $OUT/bench_nofold.jsonl || exit 1
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --engine bn_fold=1 2>/dev/null | tail -1 >> $OUT/bench_fold.jsonl || exit 1
done
timeout -k 10 150 python tools/run_config.py --spec intrusion --clients 1 --epochs 6 --fed metrics_log=$OUT/m_int.jsonl > $OUT/int.log 2>&1 || exit 1
# (the CLI runs in a scratch directory: its epoch tables would overflow gpurun_out; logs + timestamps copied back)
C=/tmp/r5cli; rm -rf $C; mkdir -p $C $OUT/cli
(cd $C && PYTHONPATH=$R timeout -k 10 150 python -m dtds.distributed -world_size 1 -colocated -epochs 2 > $OUT/cli/cli2.log 2>&1 && cp timestamp_experiment.csv $OUT/cli/ts2.csv) || exit 1
(cd $C && PYTHONPATH=$R timeout -k 10 150 python -m dtds.distributed -world_size 1 -colocated -epochs 4 > $OUT/cli/cli4.log 2>&1 && cp timestamp_experiment.csv $OUT/cli/ts4.csv) || exit 1
rm -rf $C
echo done
