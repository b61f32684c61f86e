# Eight emulated Intrusion clients: pipelined CSV writer (current library) vs the previous one-fwrite
# writer (abtest/_C_oldcsv.so via FEDTGAN_LIB), alternating
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/run_config.py --spec intrusion --rows 40000 --clients 8 --epochs 8 > gpurun_out/csv_new1.log 2>&1 && \
FEDTGAN_LIB=abtest/_C_oldcsv.so timeout -k 10 300 python -u tools/run_config.py --spec intrusion --rows 40000 --clients 8 --epochs 8 > gpurun_out/csv_old1.log 2>&1 && \
timeout -k 10 300 python -u tools/run_config.py --spec intrusion --rows 40000 --clients 8 --epochs 8 > gpurun_out/csv_new2.log 2>&1 && \
FEDTGAN_LIB=abtest/_C_oldcsv.so timeout -k 10 300 python -u tools/run_config.py --spec intrusion --rows 40000 --clients 8 --epochs 8 > gpurun_out/csv_old2.log 2>&1
echo "exit $?"
