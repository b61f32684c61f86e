# Eight clients on ONE MI355X, three ways (Intrusion schema, 40,000 synthetic rows per client, 8 rounds):
#   threads : one process, 8 client threads (ThreadComm), one HIP stream each
#   hier    : 2 processes x 4 client threads (HierComm; gloo between the processes, one GPU)
#   procs   : 8 co-located client processes (gloo data plane, 2 HIP queues each)
# The round time is the mean round_s of the federator's -metrics_log over rounds 2-7.
set -o pipefail
mkdir -p gpurun_out/cpg /tmp/cpg
timeout -k 10 300 python -m dtds.distributed -local_clients 8 -epochs 8 -backend hip -out_dir /tmp/cpg/threads -metrics_log gpurun_out/cpg/threads.jsonl -quiet > gpurun_out/cpg/threads.log 2>&1 && \
timeout -k 10 300 python -m dtds.distributed -world_size 2 -local_clients 4 -data_backend gloo -epochs 8 -backend hip -out_dir /tmp/cpg/hier -metrics_log gpurun_out/cpg/hier.jsonl -quiet > gpurun_out/cpg/hier.log 2>&1 && \
timeout -k 10 400 python -m dtds.distributed -world_size 8 -colocated -data_backend gloo -epochs 8 -backend hip -out_dir /tmp/cpg/procs -metrics_log gpurun_out/cpg/procs.jsonl -quiet > gpurun_out/cpg/procs.log 2>&1
echo "exit $?"
