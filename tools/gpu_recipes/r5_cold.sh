# Round 5: first-use cost of torch's GPU kernels on a fresh box -- 4 threads first (cold), then 1 thread, then 4
# again; then a cold-ish init profile.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r5cold}
mkdir -p $OUT
cd $R
timeout -k 10 120 python tools/cold_probe.py --threads 4 --json $OUT/cold.jsonl > $OUT/c1.log 2>&1 || exit 1
timeout -k 10 120 python tools/cold_probe.py --threads 1 --json $OUT/cold.jsonl > $OUT/c2.log 2>&1 || exit 1
timeout -k 10 120 python tools/cold_probe.py --threads 4 --json $OUT/cold.jsonl > $OUT/c3.log 2>&1 || exit 1
timeout -k 10 120 python tools/cold_probe.py --threads 1 --json $OUT/cold.jsonl > $OUT/c4.log 2>&1 || exit 1
echo done
