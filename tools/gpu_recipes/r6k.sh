# Round 6: bench.py under rocprofv3 --kernel-trace: exit status with the default teardown, with the side streams off,
# and with hipDeviceReset before interpreter exit (profiles/exit_r6.txt)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6k
mkdir -p $OUT
cd /tmp
run() {   # name, bench args
  local n=$1; shift
  (cd $R && timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/$n -o run -- python3 bench.py --steps 3 --warmup 1 "$@" > $OUT/$n.log 2>&1)
  echo "$n: exit $?" >> $OUT/exit.txt
  rm -rf $OUT/$n
}
run default
run nostreams --sync-csv --fed pipeline_sample=0
run reset --device-reset-at-exit
run reset2 --device-reset-at-exit
echo done
