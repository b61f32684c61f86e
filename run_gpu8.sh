set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bn -o run -- python3 tools/microbench.py --bn-ab > gpurun_out/prof_bn.log 2>&1
echo "exit $?"
