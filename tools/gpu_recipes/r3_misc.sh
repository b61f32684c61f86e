# Persistent-kernel probe, batched groups probe, quality ablations (one box).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3r}
mkdir -p $OUT

timeout -k 10 400 python tools/batched_probe.py --ks 4 8 --reps 4 --groups 2 4 --streams > $OUT/groups.log 2>&1 && \
bash tools/gpu_recipes/r3_quality.sh ${1:-r3r}/quality
echo "exit $?"
