# Round time of 1 vs 8 emulated Intrusion clients (40k rows each): batched engine vs one engine per thread.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3n}
mkdir -p $OUT
for v in "--clients 1" "--clients 8 --batched on" "--clients 8 --batched off" "--clients 8 --batched on" "--clients 1"; do
  timeout -k 10 300 python tools/run_config.py --spec intrusion --epochs 8 $v > $OUT/tmp.log 2>&1 || exit 1
  echo "[$v] $(tail -1 $OUT/tmp.log)" >> $OUT/clients.txt
done
echo ok
