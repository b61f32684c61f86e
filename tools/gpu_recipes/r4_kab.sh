# K = 2 / 4 / 8 emulated Intrusion clients: batched vs one engine per thread (8 epochs, whole-run wall), and a
# torch.profiler trace of the batched 8-client run's epoch 1.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4kab}
mkdir -p $OUT
cd $R
for k in 2 4 8; do
  for b in on off; do
    timeout -k 10 150 python tools/run_config.py --spec intrusion --clients $k --epochs 12 --batched $b --fed metrics_log=$OUT/m_${k}_$b.jsonl > $OUT/k${k}_$b.log 2>&1 || exit 1
  done
done
timeout -k 10 200 python tools/run_config.py --spec intrusion --clients 8 --epochs 3 --batched on --fed profile_dir=$OUT/trace --fed profile_epoch=1 > $OUT/trace.log 2>&1 || exit 1
python3 - $OUT/trace <<'PY' > $OUT/trace_gaps.txt
import glob, json, sys
for path in glob.glob(sys.argv[1] + "/*.json"):
    ev = json.load(open(path)).get("traceEvents", [])
    cpu = sorted([e for e in ev if e.get("ph") == "X" and e.get("cat") in ("cpu_op", "python_function", "user_annotation", "cuda_runtime")], key=lambda e: e["ts"])
    print(path, len(ev), "events")
    tot = {}
    for e in cpu:
        tot[(e.get("cat"), e["name"][:80])] = tot.get((e.get("cat"), e["name"][:80]), 0) + e.get("dur", 0)
    for (c, n), d in sorted(tot.items(), key=lambda kv: -kv[1])[:40]:
        print(f"{d / 1000:10.2f} ms  {c:16s} {n}")
PY
rm -rf $OUT/trace
echo done
