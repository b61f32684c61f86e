"""Build the compact Intrusion marginal profile used by the synthetic-data generator.

The reference's Intrusion *train* CSV is missing from the snapshot (only
``Server/data/raw/Intrusion_test.csv`` ships, 10,098 x 42).  This tool reads that CSV once
(plain ``pandas.read_csv``; nothing is unpickled) and writes a small JSON profile with
class frequencies, per-class categorical distributions and per-class quantile tables for
numeric columns.  ``fed_tgan_amd.data.synthetic.generate_intrusion`` samples from it.

Usage: python tools/build_intrusion_profile.py /root/reference/Server/data/raw/Intrusion_test.csv
"""
import json
import os
import sys

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from fed_tgan_amd.data.schema import INTRUSION_CATEGORICAL, INTRUSION_COLUMNS  # noqa: E402

N_Q = 65


def decimals_of(s: pd.Series) -> int:
    for d in range(0, 7):
        if np.allclose(np.round(s.to_numpy(), d), s.to_numpy()):
            return d
    return 6


def main(path: str, out: str) -> None:
    df = pd.read_csv(path)[INTRUSION_COLUMNS]
    target = "class"
    counts = df[target].value_counts()
    prof = {"columns": INTRUSION_COLUMNS, "target": target, "kinds": {}, "decimals": {},
            "classes": counts.index.tolist(), "class_p": (counts / counts.sum()).round(8).tolist(),
            "per_class": {}}
    for c in INTRUSION_COLUMNS:
        if c in INTRUSION_CATEGORICAL:
            prof["kinds"][c] = "cat_int" if df[c].dtype.kind in "iu" else "cat_str"
        else:
            prof["kinds"][c] = "int" if df[c].dtype.kind in "iu" else "float"
            prof["decimals"][c] = 0 if prof["kinds"][c] == "int" else decimals_of(df[c])
    qs = np.linspace(0, 1, N_Q)
    for cls in prof["classes"]:
        sub = df[df[target] == cls]
        entry = {"cat": {}, "num": {}}
        for c in INTRUSION_COLUMNS:
            if c == target:
                continue
            if c in INTRUSION_CATEGORICAL:
                vc = sub[c].value_counts()
                vals = [v.item() if hasattr(v, "item") else v for v in vc.index.tolist()]
                entry["cat"][c] = {"values": vals, "p": (vc / vc.sum()).round(8).tolist()}
            else:
                entry["num"][c] = np.quantile(sub[c].to_numpy(dtype=np.float64), qs).round(6).tolist()
        prof["per_class"][cls] = entry
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(prof, f, separators=(",", ":"))
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/Server/data/raw/Intrusion_test.csv"
    dst = os.path.join(os.path.dirname(__file__), "..", "fed_tgan_amd", "data", "profiles", "intrusion.json")
    main(src, dst)
