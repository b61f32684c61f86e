# torch.profiler trace of round 1 of a one-client run (main thread only), summarised on the box.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4trace1}
mkdir -p $OUT
cd $R
timeout -k 10 200 python tools/run_config.py --spec intrusion --clients 1 --epochs 3 --fed profile_dir=$OUT/trace --fed profile_epoch=1 --fed metrics_log=$OUT/m.jsonl > $OUT/run.log 2>&1 || exit 1
python3 - $OUT/trace <<'PY' > $OUT/trace_summary.txt
import glob, json, sys
for path in glob.glob(sys.argv[1] + "/*.json"):
    ev = json.load(open(path)).get("traceEvents", [])
    xs = [e for e in ev if e.get("ph") == "X"]
    print(path.split("/")[-1], len(ev), "events")
    tot = {}
    for e in xs:
        k = (e.get("cat"), e["name"][:90])
        tot[k] = tot.get(k, 0) + e.get("dur", 0)
    for (c, n), d in sorted(tot.items(), key=lambda kv: -kv[1])[:45]:
        print(f"{d / 1000:10.2f} ms  {str(c):18s} {n}")
    print("longest single host events:")
    for e in sorted([e for e in xs if e.get("cat") in ("cpu_op", "cuda_runtime", "python_function", "user_annotation")], key=lambda e: -e.get("dur", 0))[:25]:
        print(f"{e.get('dur', 0) / 1000:10.2f} ms  {e.get('cat')} {e['name'][:100]} tid={e.get('tid')}")
PY
rm -rf $OUT/trace
echo done
