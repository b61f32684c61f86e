# Round 4: ragged batched clients, HierComm batching, event-ordered thread aggregation, dedicated federator
# over RCCL -- the GPU tests of those paths, then the topology timings.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4fed}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_batched.py tests/test_gpu_federation.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 && \
timeout -k 10 200 python tools/topology_probe.py --world-size 2 --epochs 8 --rows 40000 --n-sample 40000 > $OUT/topo_dedicated.log 2>&1 && \
timeout -k 10 200 python tools/topology_probe.py --world-size 1 --colocated --epochs 8 --rows 40000 --n-sample 40000 > $OUT/topo_single.log 2>&1
echo "exit $?"
