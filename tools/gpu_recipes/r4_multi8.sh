# 8 emulated Intrusion clients on one GPU: batched vs threads (per-phase metrics), batched without the early
# label-encoder helper; Adult 8 clients Dirichlet(0.3) (ragged -> batched); then the one-client kernel A/B.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4multi8}
mkdir -p $OUT
RC="python tools/run_config.py --spec intrusion --clients 8 --epochs 8"
for pass in 1 2; do
  timeout -k 10 150 $RC --batched on --fed metrics_log=$OUT/m_on_$pass.jsonl > $OUT/on_$pass.log 2>&1 || exit 1
  timeout -k 10 150 $RC --batched off --fed metrics_log=$OUT/m_off_$pass.jsonl > $OUT/off_$pass.log 2>&1 || exit 1
  timeout -k 10 150 $RC --batched on --fed label_encoders_early=0 --fed metrics_log=$OUT/m_onlate_$pass.jsonl > $OUT/onlate_$pass.log 2>&1 || exit 1
done
timeout -k 10 150 python tools/run_config.py --spec adult --clients 8 --shard dirichlet --alpha 0.3 --epochs 5 --rows 8000 > $OUT/adult8.log 2>&1 || exit 1
bash tools/gpu_recipes/r4_profab.sh $(basename $OUT)/profab || exit 1
echo done
