# Hardware counters of the training step + generation (tools/gpu_probe.py), one rocprofv3 --pmc pass
# per counter group (gfx950 slots: <= 8 SQ, FETCH_SIZE = 3 TCC, WRITE_SIZE = 2 TCC), then a summary.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
P="python3 tools/gpu_probe.py --backend hip --rows 40000 --steps 5"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc_a -o run -- $P > gpurun_out/pmc_a.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_b -o run -- $P > gpurun_out/pmc_b.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_c -o run -- $P > gpurun_out/pmc_c.log 2>&1 && \
python3 tools/pmc_summary.py gpurun_out/pmc_a gpurun_out/pmc_b gpurun_out/pmc_c --out=gpurun_out/pmc_summary.txt > /dev/null
echo "exit $?"
