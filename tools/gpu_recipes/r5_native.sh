# Round 5: native RCCL data plane (csrc/comm) -- its GPU tests, then bench over a one-rank communicator through
# the native plane vs torch.distributed's ProcessGroup vs plain (two passes, alternating).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5native}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_native_rccl.py > $OUT/pytest_native.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 >> $OUT/bench_plain.jsonl || exit 1
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --force-dist 2>/dev/null | tail -1 >> $OUT/bench_dist.jsonl || exit 1
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --force-dist --native-rccl 2>/dev/null | tail -1 >> $OUT/bench_native.jsonl || exit 1
done
echo done
