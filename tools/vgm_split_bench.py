"""Time the whole-fit VGM kernel (csrc/kernels/vgm_fit.hip) with one workgroup per column against the split
fit (a cluster of workgroups per column), at the Intrusion init shape (22 columns x 40k rows) and the wide shape
(256 x 100k).  Mixture-of-Gaussians columns, own initialisation; prints one JSON line per (shape, split).

    python tools/vgm_split_bench.py [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from fed_tgan_amd.features.vgm_fit import fit_vgm_torch  # noqa: E402
from fed_tgan_amd.ops import native  # noqa: E402


def columns(n_cols, n_rows, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n_cols):
        k = int(rng.integers(1, 6))
        mu = rng.normal(0, 10, k)
        sd = rng.uniform(0.2, 3, k)
        z = rng.integers(0, k, n_rows)
        out.append(rng.normal(mu[z], sd[z]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--splits", default="1,0", help="vgm_split values to time (0 = auto)")
    args = ap.parse_args()
    native.require()
    dev = "cuda:0"
    for n_cols, n_rows in ((22, 40000), (256, 100000)):
        cols = columns(n_cols, n_rows)
        for split in [int(v) for v in args.splits.split(",")]:
            prev = torch.ops.fedtgan.set_tuning("vgm_split", split)
            try:
                G = torch.ops.fedtgan.set_tuning("vgm_split_of", n_cols)
                ts = []
                for _ in range(args.reps + 1):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    bank = fit_vgm_torch(cols, seed=3, device=dev)
                    torch.cuda.synchronize()
                    ts.append(time.perf_counter() - t0)
                info = fit_vgm_torch.last_info
            finally:
                torch.ops.fedtgan.set_tuning("vgm_split", prev)
            print(json.dumps({"cols": n_cols, "rows": n_rows, "split": "auto" if split == 0 else split,
                              "workgroups_per_col": int(G), "fit_ms": [round(1e3 * t, 2) for t in ts[1:]],
                              "em_iters_mean": float(info[:, 0].mean()), "timeouts": int((info[:, 1] < 0).sum()),
                              "modes": int(bank.components().sum())}), flush=True)


if __name__ == "__main__":
    main()
