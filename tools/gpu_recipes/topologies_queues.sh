set -o pipefail
mkdir -p gpurun_out/topo /tmp/topo
for q in 1 2; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -m dtds.distributed -world_size 3 -epochs 12 -backend hip -out_dir /tmp/topo/d$q -metrics_log gpurun_out/topo/dedicated_q$q.jsonl > gpurun_out/topo/dedicated_q$q.log 2>&1 || exit 1
done
GPU_MAX_HW_QUEUES=1 timeout -k 10 300 python -m dtds.distributed -world_size 2 -colocated -data_backend gloo -epochs 12 -backend hip -out_dir /tmp/topo/c1 -metrics_log gpurun_out/topo/colocated_q1.jsonl > gpurun_out/topo/colocated_q1.log 2>&1
echo "exit $?"
