# Round time of 1 / 4 / 8 emulated Intrusion clients (40k rows each): batched engine vs one engine per thread.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3u}
mkdir -p $OUT
for v in "--clients 1" "--clients 4 --batched on" "--clients 4 --batched off" "--clients 8 --batched on" "--clients 8 --batched off" "--clients 2 --batched on" "--clients 2 --batched off"; do
  timeout -k 10 300 python tools/run_config.py --spec intrusion --epochs 10 --out /tmp/rc $v > $OUT/tmp.log 2>&1 || exit 1
  echo "[$v] $(tail -1 $OUT/tmp.log)" >> $OUT/clients.txt
  rm -rf /tmp/rc
done
echo ok
