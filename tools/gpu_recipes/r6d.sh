# Round 6: Adult epoch-0, GPU pipeline variants (40 seeds each): eager torch fp32 oracle (host encode), HIP fp32,
# HIP bf16 with the host encode
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6d
mkdir -p $OUT
cd $R
S=$(seq 10 49)
timeout -k 10 300 python -u tools/adult_vgm_ab.py --seeds $S --variants hip --backend hip --precision fp32 --tag _fp32 --out $OUT/vgm_ab.jsonl > $OUT/fp32.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/adult_vgm_ab.py --seeds $S --variants hip --backend hip --fed device_encode=0 --tag _hostenc --out $OUT/vgm_ab.jsonl > $OUT/hostenc.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/adult_vgm_ab.py --seeds $S --variants torchdev --backend torch --precision fp32 --tag _torch --out $OUT/vgm_ab.jsonl > $OUT/torch.log 2>&1 || exit 1
echo done
