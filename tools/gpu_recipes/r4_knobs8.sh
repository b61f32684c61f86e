# 8 batched clients (Intrusion, 40k rows each): existing engine / ops knobs and stream groups, one probe each.
# A probe that fails with a Python error is logged and the sweep goes on; a timeout / abort / crash stops it.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4knobs8}
mkdir -p $OUT
P="python tools/batched_probe.py --ks 8 --skip-plain --reps 3"
run() {
  echo "== $*" >> $OUT/knobs.log
  timeout -k 10 120 $P "$@" > $OUT/probe.tmp 2>&1; rc=$?
  grep '^{' $OUT/probe.tmp >> $OUT/knobs.log; tail -2 $OUT/probe.tmp | grep -i error >> $OUT/knobs.log
  case $rc in 124|134|137|139) echo "stop: rc $rc" >> $OUT/knobs.log; return 1;; esac
  return 0
}
V=(
  "--engine fuse_adam_max=0"
  "--engine fuse_g_adam=0"
  "--engine fuse_adam_max=4000000"
  "--engine bn_colown=1 --engine fuse_g_adam=0"
  "--engine fuse_d0_adam=1"
  "--engine paired=0"
  "--engine onehot_trans=1"
  "--tuning bn_cols=16"
  "--tuning bn_cols=4"
  "--tuning adam_store=0"
  "--engine dw0_tile=64"
  "--groups 2"
)
for v in "${V[@]}"; do run $v || break; done
echo "exit $?"
