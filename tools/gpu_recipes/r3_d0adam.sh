# D0's weight gradient held for the D Adam launch in the batched step (EngineConfig.fuse_d0_adam): numerics
# tests, then the 8- and 4-client step A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_batched.py tests/test_hip_engine.py -m gpu -q -x --timeout 170 --timeout-method thread > $O/tests.log 2>&1 && \
P="timeout -k 10 200 python tools/batched_probe.py --ks 4 8 --skip-plain --plan on --reps 4" && \
$P > $O/on.log 2>&1 && \
$P --engine fuse_d0_adam=0 > $O/off.log 2>&1 && \
$P > $O/on2.log 2>&1
echo "exit $?"
