# Round 6: bench.py under rocprofv3 -- bisect the exit segfault: cooperative VGM-fit launch, label-encoder helper
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6m
mkdir -p $OUT
cd /tmp
run() {
  local n=$1; shift
  (cd $R && timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/$n -o run -- python3 bench.py --steps 3 --warmup 1 "$@" > $OUT/$n.log 2>&1)
  echo "$n: exit $?" >> $OUT/exit.txt
  rm -rf $OUT/$n
}
run nocoop --tuning vgm_split=1
run noleh --fed label_encoders_early=0
run both --tuning vgm_split=1 --fed label_encoders_early=0
(cd $R && timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/micro -o run -- python3 tools/microbench.py --step-only --epochs-only > $OUT/micro.log 2>&1); echo "microbench: exit $?" >> $OUT/exit.txt
rm -rf $OUT/micro
echo done
