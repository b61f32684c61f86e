"""Fold extra seeds of `tools/reference_quality.py` (its per-seed JSON lines, e.g. from parallel runs' logs) into
profiles/reference_quality_r3_byvalue.json: appends the runs and writes `summary_all` (mean / SEM over every seed).

    python tools/ref_quality_merge.py run_a.log run_b.log
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATH = os.path.join(ROOT, "profiles", "reference_quality_r3_byvalue.json")


def main(logs):
    d = json.load(open(PATH))
    have = {r["seed"] for r in d["runs"]}
    for lg in logs:
        for line in open(lg):
            line = line.strip()
            if not line.startswith("{"):
                continue
            try:
                r = json.loads(line)
            except ValueError:
                continue
            if "seed" in r and "avg_jsd" in r and r["seed"] not in have:
                d["runs"].append(r)
                have.add(r["seed"])
    j = np.array([r["avg_jsd"] for r in d["runs"]])
    w = np.array([r["avg_wd"] for r in d["runs"]])
    sem = lambda a: (a.std(0, ddof=1) / np.sqrt(len(a))).round(4).tolist()  # noqa: E731
    d["summary_all"] = {"epochs": d["summary"]["epochs"], "seeds": sorted(have), "n_seeds": len(have),
                        "avg_jsd_mean": j.mean(0).round(4).tolist(), "avg_jsd_sem": sem(j),
                        "avg_wd_mean": w.mean(0).round(4).tolist(), "avg_wd_sem": sem(w)}
    json.dump(d, open(PATH, "w"), indent=1)
    print(json.dumps(d["summary_all"]))


if __name__ == "__main__":
    main(sys.argv[1:])
