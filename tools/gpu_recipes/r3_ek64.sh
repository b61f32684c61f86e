# EK variants for 64-tiles / batched launches: GPU tests, one-client step, batched 4 / 8 clients.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3e64}
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 170 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python tools/microbench.py --step-only > $O/head_step.txt 2>&1 && \
timeout -k 10 300 python tools/batched_probe.py --ks 4 8 --skip-plain --plan on --reps 4 > $O/batched.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
echo "exit $?"
