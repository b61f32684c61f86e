set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3p}
mkdir -p $OUT
timeout -k 10 400 python tools/batched_probe.py --ks 4 8 --reps 4 --groups 2 4 --streams > $OUT/groups.log 2>&1 && \
timeout -k 10 400 python tools/batched_probe.py --ks 8 --reps 4 --groups 2 4 --skip-plain --engine chain_d1=0 --engine fuse_d_adam=0 > $OUT/groups_nofuse.log 2>&1
echo "exit $?"
