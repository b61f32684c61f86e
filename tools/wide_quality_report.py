"""Per-epoch Avg_JSD / Avg_WD table (mean +- standard error over seeds) of tools/wide_quality.py runs, with each
implementation's z-score against the reference's own code, and the 100k x 512 three-way runs of
tools/run_config.py (torch oracle / HIP fp32 / HIP bf16).

    python tools/wide_quality_report.py --reduced profiles/wide_quality_ref_r5.jsonl profiles/wide_quality_ours_r5.jsonl \
        --full profiles/wide_full_r5.jsonl > profiles/wide_quality_r5.txt
"""
import argparse
import collections
import json

import numpy as np


def _load(paths):
    runs = []
    for p in paths:
        with open(p) as f:                               # .log files: the JSON lines among other output
            runs += [json.loads(line) for line in f if line.lstrip().startswith("{")]
    return runs


def _stats(rows, key):
    a = np.asarray([r[key] for r in rows], dtype=np.float64)
    n = len(a)
    return a.mean(0), (a.std(0, ddof=1) / np.sqrt(n)) if n > 1 else np.full(a.shape[1], np.nan), n


def reduced_table(runs):
    by = collections.defaultdict(list)
    for r in runs:
        by[r["impl"]].append(r)
    ref = by.get("reference")
    lines = []
    for key, label in (("avg_jsd", "Avg_JSD"), ("avg_wd", "Avg_WD")):
        lines.append(f"## {label} per epoch: mean +- SE (seeds); z = (impl - reference) / sqrt(SE_impl^2 + SE_ref^2)")
        impls = sorted(by, key=lambda k: (k != "reference", k))
        stats = {k: _stats(by[k], key) for k in impls}
        ne = min(len(s[0]) for s in stats.values())
        head = "epoch | " + " | ".join(f"{k} (n={stats[k][2]})" for k in impls)
        lines += [head, "-" * len(head)]
        for e in range(ne):
            cells = []
            for k in impls:
                m, se, _ = stats[k]
                cell = f"{m[e]:.4f} +- {se[e]:.4f}"
                if ref is not None and k != "reference":
                    rm, rse, _ = stats["reference"]
                    z = (m[e] - rm[e]) / np.sqrt(se[e] ** 2 + rse[e] ** 2)
                    cell += f" (z {z:+.1f})"
                cells.append(cell)
            lines.append(f"{e:5d} | " + " | ".join(cells))
        lines.append("")
    return lines


def full_table(runs):
    by = collections.defaultdict(lambda: collections.defaultdict(list))
    seen = set()
    for r in runs:
        if "epoch" not in r or "precision" not in r:     # metrics-log lines and summaries carry no per-epoch score
            continue
        key = (r.get("backend", "hip"), r["precision"], r.get("seed"), r["epoch"])
        if key in seen:                                  # the same record in a log and in the JSONL
            continue
        seen.add(key)
        tag = f"{r.get('backend', 'hip')}-{r['precision']}"
        by[tag][r["epoch"]].append(r)
    lines = ["## 100k x 512, 1 client, 5 epochs (tools/run_config.py): Avg_JSD / Avg_WD, mean +- SE over seeds (n)"]
    for tag, eps in sorted(by.items()):
        cells = []
        for e in sorted(eps):
            j = np.asarray([r["avg_jsd"] for r in eps[e]])
            w = np.asarray([r["avg_wd"] for r in eps[e]])
            n = len(j)
            se = (lambda a: a.std(ddof=1) / np.sqrt(n)) if n > 1 else (lambda a: float("nan"))
            cells.append(f"{e}: {j.mean():.4f}+-{se(j):.4f} / {w.mean():.4f}+-{se(w):.4f} (n={n})")
        lines.append(f"{tag:12s} " + "  ".join(cells))
    return lines + [""]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reduced", nargs="*", default=[])
    ap.add_argument("--full", nargs="*", default=[])
    args = ap.parse_args()
    out = []
    if args.reduced:
        out += reduced_table(_load(args.reduced))
    if args.full:
        out += full_table(_load(args.full))
    print("\n".join(out))


if __name__ == "__main__":
    main()
