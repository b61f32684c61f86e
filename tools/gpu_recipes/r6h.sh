# Round 6: symbolise the exit() segfault of bench.py under rocprofv3: the process' memory map + the crash stack
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6h
mkdir -p $OUT
cd /tmp
(cd $R && FEDTGAN_DUMP_MAPS=$OUT/maps timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/bench -o run -- python3 bench.py --steps 3 --warmup 1 > $OUT/bench_prof.log 2>&1); echo "exit $?" > $OUT/exit.txt
rm -rf $OUT/bench
(cd $R && FEDTGAN_DUMP_MAPS=$OUT/maps_noprof timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 > $OUT/bench_noprof.log 2>&1); echo "noprof exit $?" >> $OUT/exit.txt
echo done
