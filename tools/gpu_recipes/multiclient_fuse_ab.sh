# Eight emulated Intrusion clients on one GPU: the fused launches (default) vs separate launches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/run_config.py --spec intrusion --rows 40000 --clients 8 --epochs 8 > gpurun_out/mc_fused.log 2>&1 && \
timeout -k 10 300 python -u tools/run_config.py --spec intrusion --rows 40000 --clients 8 --epochs 8 --engine fuse_g_adam=0 --engine fuse_d_adam=0 --engine chain_d1=0 > gpurun_out/mc_sep.log 2>&1 && \
timeout -k 10 300 python -u tools/run_config.py --spec intrusion --rows 40000 --clients 8 --epochs 8 > gpurun_out/mc_fused2.log 2>&1
echo "exit $?"
