set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3d
mkdir -p $OUT
env | grep -i -E "nccl|rccl|hsa|hip" > $OUT/env.txt
timeout -k 10 200 python bench.py --force-dist --steps 2 --warmup 1 --no-eval > $OUT/bench_fd.log 2>&1 && \
ls -la /tmp/fedtgan_rccl_* > $OUT/ls.txt 2>&1; for f in /tmp/fedtgan_rccl_*/*; do echo "== $f"; head -80 $f; done > $OUT/rccl_logs.txt 2>&1; echo done
