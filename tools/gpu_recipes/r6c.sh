# Round 6: multi-draw equality test, step breakdown (kernel order) of the captured step, Adult VGM-fit bisect
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6c
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_hip_engine.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k 'multi_draw' > $OUT/mdtest.log 2>&1 || exit 1
cd /tmp
(cd $R && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/step -o run -- python3 tools/microbench.py --step-only > $OUT/step.log 2>&1) || exit 1
python3 $R/tools/step_breakdown.py $OUT/step/run_results.db --order > $OUT/step_breakdown.txt 2>&1 || exit 1
rm -rf $OUT/step
cd $R
timeout -k 10 700 python -u tools/adult_vgm_ab.py --seeds $(seq 10 39) --variants hip torchdev hip_global hip_clients --out $OUT/vgm_ab.jsonl > $OUT/vgm_ab.log 2>&1 || exit 1
echo done
