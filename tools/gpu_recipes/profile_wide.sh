# rocprofv3 kernel trace of the wide 100k x 512 config (1 client, 2 epochs); summary by tools/prof_summary.py
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wide -o run -- python3 tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 2 > gpurun_out/prof_wide.log 2>&1 && \
python3 tools/prof_summary.py gpurun_out/prof_wide/run_results.db --shape > gpurun_out/prof_wide_summary.txt 2>&1 && python3 tools/step_breakdown.py gpurun_out/prof_wide/run_results.db > gpurun_out/prof_wide_step.txt 2>&1
echo "exit $?"
