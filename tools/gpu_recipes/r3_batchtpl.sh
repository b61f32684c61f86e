# One-client GEMM instantiations without the batched-client prologue: step vs the round-2 tree, GPU tests, bench.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3t}
mkdir -p $O
(cd $R/_r2tree && timeout -k 10 200 python tools/microbench.py --step-only > $O/r2_step.txt 2>&1) && \
(cd $R && timeout -k 10 200 python tools/microbench.py --step-only > $O/head_step.txt 2>&1) && \
(cd $R && timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 170 --timeout-method thread > $O/pytest_gpu.log 2>&1) && \
(cd $R && timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1) && \
(cd $R && timeout -k 10 200 python tools/batched_probe.py --ks 4 8 --skip-plain --plan on --reps 4 > $O/batched.log 2>&1)
echo "exit $?"
