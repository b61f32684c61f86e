# Round 6: one-rank RCCL round vs plain, with the same sub-phase timers on both
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6p
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_federation.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "one_rank_rccl or two_ranks" > $OUT/tests.log 2>&1 || exit 1
for rep in 1 2; do
for cfg in "--fed phase_detail=1" "--force-dist" "--force-dist --native-rccl" "--force-dist --fed force_gather=1" "--fed phase_detail=1 --fed pipeline_sample=0" "--force-dist --fed pipeline_sample=0"; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 $cfg 2>/dev/null | grep '"metric"' | python3 -c "
import json,sys
r=json.loads(sys.stdin.read()); print('%-50s %7.3f ms/round plane=%s phase ms %s' % ('$cfg', r['value']*1e3, r['config']['data_plane'], {k: round(v*1e3,3) for k,v in r['phase_s'].items()}))" >> $OUT/ab.txt || exit 1
done
done
echo done
