"""Round-time report of a FedRuntime metrics log (``FedConfig.metrics_log``) and of CLI ``timestamp_experiment.csv``
files against bench.py's steady round: is any round (round 0 and 1 included) slower than 1.5x the steady one?

    python tools/stall_report.py --metrics m_int.jsonl --ts ts2.csv ts4.csv --bench bench.jsonl > stall.txt

Columns per round: wall seconds, then the host's view of it (``h_wait``: entering the train phase, ``h_issue``:
issuing the epoch's graphs, ``h_agg`` / ``h_sample`` / ``h_end``: aggregation, sampling + CSV hand-off, the final
stream wait), the background writer's seconds on the previous table (``csv_wait_prev``: its device-to-host copy,
``csv_write_prev``: formatting + write), process CPU seconds and the cgroup's CFS throttling in the round.
"""
import argparse
import json
import statistics


def _load_jsonl(path):
    with open(path) as f:
        return [json.loads(line) for line in f if line.lstrip().startswith("{")]


def metrics_table(rows):
    cols = ["round_s", "t_train", "h_wait", "h_issue", "h_agg", "h_sample", "h_end", "csv_wait_prev",
            "csv_write_prev", "cpu_s", "throttled_usec"]
    steady = statistics.median([r["round_s"] for r in rows[2:]]) if len(rows) > 2 else None
    out = ["epoch " + " ".join(f"{c:>14s}" for c in cols) + "   / steady"]
    for r in rows:
        cells = []
        for c in cols:
            v = r.get(c)
            if v is None:
                cells.append(f"{'-':>14s}")
            elif c == "throttled_usec":
                cells.append(f"{v:14d}" if isinstance(v, int) else f"{v:14.0f}")
            else:
                cells.append(f"{1e3 * v:12.2f}ms")
        ratio = f"{r['round_s'] / steady:6.2f}x" if steady else "   -"
        out.append(f"{r['epoch']:5d} " + " ".join(cells) + f"   {ratio}")
    if steady:
        worst = max(r["round_s"] for r in rows) / steady
        out.append(f"steady (median of rounds >= 2): {1e3 * steady:.2f} ms; slowest round / steady = {worst:.2f}x")
    return out


def ts_table(path, bench_s):
    with open(path) as f:
        vals = [float(line.strip().split(",")[0]) for line in f if line.strip()]
    ref = f" vs bench {1e3 * bench_s:.2f} ms: " + ", ".join(f"{v / bench_s:.2f}x" for v in vals) if bench_s else ""
    return [f"{path}: " + ", ".join(f"{1e3 * v:.2f} ms" for v in vals) + ref]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--metrics", nargs="*", default=[])
    ap.add_argument("--ts", nargs="*", default=[])
    ap.add_argument("--bench", nargs="*", default=[])
    args = ap.parse_args()
    out = []
    bench_s = None
    if args.bench:
        lines = [r for p in args.bench for r in _load_jsonl(p)]
        vals = [r["value"] for r in lines]
        bench_s = statistics.median(vals)
        out.append(f"bench.py sec_per_epoch (median of {len(vals)}): {1e3 * bench_s:.2f} ms "
                   f"({', '.join(f'{1e3 * v:.2f}' for v in vals)})")
        out.append("")
    for p in args.metrics:
        out.append(f"== {p}")
        out += metrics_table(_load_jsonl(p))
        out.append("")
    if args.ts:
        out.append("== timestamp_experiment.csv entries (each includes that epoch's CSV on disk)")
        for p in args.ts:
            out += ts_table(p, bench_s)
    print("\n".join(out))


if __name__ == "__main__":
    main()
