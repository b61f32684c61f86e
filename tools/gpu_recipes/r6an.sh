# Round 6: 128x128-tile bf16 output epilogue (generation GEMMs) as column-octet 16-B stores vs the previous build
# (ab/_C_prev.so swapped in place), same box: every GPU test on the new build, then the generation probe and the bench
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6an
mkdir -p $OUT
cd $R
cp fed_tgan_amd/_C.so ab/_C_new.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for i in 1 2; do
  for arm in new prev; do
    cp ab/_C_$arm.so fed_tgan_amd/_C.so
    timeout -k 10 150 python3 tools/gen_probe.py 2>&1 | tail -4 | sed "s/^/[$arm] /" >> $OUT/gen.txt || exit 1
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 | sed "s/^/[$arm] /" >> $OUT/bench.jsonl || exit 1
  done
done
cp ab/_C_new.so fed_tgan_amd/_C.so
cat $OUT/gen.txt
python3 -c "
import json
for l in open('$OUT/bench.jsonl'):
    t, j = l.split('] ', 1); d = json.loads(j); print(t + ']', d['ms_per_step'], d['phase_s'], d['avg_jsd'])
"
