set -o pipefail
mkdir -p gpurun_out/topo /tmp/topo
timeout -k 10 200 python -c "
import os, sys
sys.argv=['x','-world_size','3','-epochs','6','-backend','hip','-out_dir','/tmp/topo/a','-metrics_log','gpurun_out/topo/auto.jsonl']
import fed_tgan_amd.cli as c
orig=c.run_rank
def rr(rank,args):
    print('child', rank, os.environ.get('GPU_MAX_HW_QUEUES'), flush=True)
    return orig(rank,args)
c.run_rank=rr
c.main(sys.argv[1:])
" > gpurun_out/topo/auto.log 2>&1 && \
GPU_MAX_HW_QUEUES=2 timeout -k 10 200 python -m dtds.distributed -world_size 3 -epochs 6 -backend hip -out_dir /tmp/topo/b -metrics_log gpurun_out/topo/env2.jsonl > gpurun_out/topo/env2.log 2>&1
echo "exit $?"
