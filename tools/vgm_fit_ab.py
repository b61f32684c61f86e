"""Whole-fit HIP VGM kernel vs the torch-op fit vs sklearn on the Adult Dirichlet client columns, many seeds.

tools/adult_vgm_ab.py tied the Adult epoch-0 quality gap to the device VGM fit (vgm_fit_kernel): with the
torch-op fit on the same GPU the federated pipeline matches the reference.  This compares the fits themselves
per seed: final lower bound, valid-mode count and (HIP) iteration count / convergence, per client column.

    python tools/vgm_fit_ab.py --seeds 40 --out gpurun_out/vgm_fit_ab.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from wide_quality import make_wide_split  # noqa: E402


def client_columns(datapath: str, spec, k: int):
    from fed_tgan_amd.data.table import load_table
    from fed_tgan_amd.fed.stats import merge_categorical_metas
    tabs = [load_table(datapath.format(client=i), spec) for i in range(k)]
    _, vocabs, _ = merge_categorical_metas([t.local_meta() for t in tabs])
    out = []
    for t in tabs:
        enc = t.encode(vocabs)
        cat = set(t.categorical_indices())
        out.append([np.asarray(enc[:, j], dtype=np.float64) for j in range(enc.shape[1]) if j not in cat])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=40)
    ap.add_argument("--sklearn", action="store_true")
    ap.add_argument("--work", default="/tmp/fedtgan_adult_vgm")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch
    from fed_tgan_amd.features import vgm_fit
    spec, _, datapath = make_wide_split(args.work, 0, 8000, 2, spec_name="adult", shard_mode="dirichlet", alpha=0.3)
    cols = client_columns(datapath, spec, 2)
    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    variants = ["hip", "torch"] if dev.type == "cuda" else ["torch"]
    for ci, cc in enumerate(cols):
        for seed in range(args.seeds):
            for var in variants + (["sklearn"] if args.sklearn else []):
                rec = {"client": ci, "seed": seed, "variant": var}
                if var == "sklearn":
                    from sklearn.mixture import BayesianGaussianMixture
                    lbs, modes, its = [], [], []
                    for x in cc:
                        g = BayesianGaussianMixture(n_components=10, weight_concentration_prior_type="dirichlet_process",
                                                    weight_concentration_prior=0.001, n_init=1, random_state=seed)
                        g.fit(x.reshape(-1, 1))
                        lbs.append(float(g.lower_bound_))
                        modes.append(int((g.weights_ > 0.005).sum()))
                        its.append(int(g.n_iter_))
                    rec.update(lower_bound=lbs, modes=modes, iters=its)
                else:
                    b = vgm_fit.fit_vgm_torch(cc, seed=seed, device=dev, use_hip=(var == "hip"))
                    rec["lower_bound"] = [float(v) for v in vgm_fit.fit_vgm_torch.last_lower_bound]
                    rec["modes"] = [int(v) for v in b.components().sum(1)]
                    if var == "hip":
                        info = vgm_fit.fit_vgm_torch.last_info
                        rec["iters"] = [int(v) for v in info[:, 0]]
                        rec["status"] = [int(v) for v in info[:, 1]]
                        rec["refit"] = [int(v) for v in vgm_fit.fit_vgm_torch.last_refit_columns]
                    rec["weights"] = np.round(b.weights, 4).tolist()
                print(json.dumps({k: rec[k] for k in rec if k != "weights"}), flush=True)
                if args.out:
                    with open(args.out, "a") as f:
                        f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
