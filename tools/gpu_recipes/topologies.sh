# Round time of the reference topology (dedicated federator + 2 clients, gloo data plane) against the
# co-located layout (2 client ranks, rank 0 also federates) and the in-process 2-client emulation,
# all on one GPU (RCCL needs a GPU per rank, so the multi-process runs use gloo here).
set -o pipefail
mkdir -p gpurun_out/topo /tmp/topo
timeout -k 10 300 python -m dtds.distributed -world_size 3 -epochs 12 -backend hip -out_dir /tmp/topo/dedicated -metrics_log gpurun_out/topo/dedicated.jsonl > gpurun_out/topo/dedicated.log 2>&1 && \
timeout -k 10 300 python -m dtds.distributed -world_size 2 -colocated -data_backend gloo -epochs 12 -backend hip -out_dir /tmp/topo/colocated -metrics_log gpurun_out/topo/colocated.jsonl > gpurun_out/topo/colocated.log 2>&1 && \
timeout -k 10 300 python -m dtds.distributed -local_clients 2 -epochs 12 -backend hip -out_dir /tmp/topo/emulated -metrics_log gpurun_out/topo/emulated.jsonl > gpurun_out/topo/emulated.log 2>&1
echo "exit $?"
