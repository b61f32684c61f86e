# Hardware counters of the 8-client batched step (tools/batched_probe.py --profile-k 8), one rocprofv3 --pmc
# pass per counter group (gfx950 slots: <= 8 SQ, FETCH_SIZE = 3 TCC, WRITE_SIZE = 2 TCC), then a summary.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_b8}
mkdir -p $O
P="python3 tools/batched_probe.py --profile-k 8 --reps 1"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/a -o run -- $P > $O/a.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/b -o run -- $P > $O/b.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/c -o run -- $P > $O/c.log 2>&1 && \
python3 tools/pmc_summary.py $O/a $O/b $O/c --out=$O/summary.txt > /dev/null && rm -rf $O/a $O/b $O/c
echo "exit $?"
