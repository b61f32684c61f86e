# K = 2 / 4 / 8 emulated Intrusion clients: batched vs one engine per thread (8 epochs, whole-run wall), and a
# torch.profiler trace of the batched 8-client run's epoch 1.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4kab3}
mkdir -p $OUT
cd $R
for k in 2 4 8; do
  for b in on off; do
    timeout -k 10 150 python tools/run_config.py --spec intrusion --clients $k --epochs 12 --batched $b --fed metrics_log=$OUT/m_${k}_$b.jsonl > $OUT/k${k}_$b.log 2>&1 || exit 1
  done
done
echo done
echo done
