# Round 5: kernel traces of the one-rank RCCL bench with the deferred hand-off (+2 ms per round) and without, to see
# what stretches the epoch; then the pipelined-sampling identity test (deferred variant included).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5deftrace}
mkdir -p $OUT
cd /tmp
for d in 1 0; do
  (cd $R && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt$d -o run -- python3 bench.py --steps 6 --warmup 2 --force-dist --fed defer_handoff=$d > $OUT/kt$d.log 2>&1) || exit 1
done
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_federation.py -k pipelined > $OUT/pytest_pipe.log 2>&1 || exit 1
echo done
