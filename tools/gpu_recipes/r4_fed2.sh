set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4fed2}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_federation.py -m gpu -x -v --timeout 240 --timeout-method thread -k "batched or hier or dedicated" > $OUT/pytest.log 2>&1; echo "pytest rc $?" >> $OUT/pytest.log
timeout -k 10 200 python tools/topology_probe.py --world-size 2 --epochs 8 --rows 40000 --n-sample 40000 > $OUT/topo_dedicated.log 2>&1 && \
timeout -k 10 200 python tools/topology_probe.py --world-size 1 --colocated --epochs 8 --rows 40000 --n-sample 40000 > $OUT/topo_single.log 2>&1
echo "exit $?"
timeout -k 10 600 python tools/batched_ops.py --k 8 > $OUT/batched_ops_k8.jsonl 2> $OUT/batched_ops_k8.err; echo "ops rc $?"
