"""Per-column similarity after each epoch (which columns drive Avg_JSD / Avg_WD).

    python tools/quality_probe.py --epochs 2 --seeds 0 1 2

Same metric definitions as `Server/similarity_analysis.py` (fed_tgan_amd/eval/similarity.py);
the real table is the client's synthetic Intrusion-schema shard.
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np
import pandas as pd
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def per_column(real: pd.DataFrame, fake: pd.DataFrame, cat_cols):
    from scipy.spatial import distance
    from scipy.stats import wasserstein_distance
    from sklearn.preprocessing import MinMaxScaler
    out = {}
    for c in real.columns:
        if c in cat_cols:
            rv = real[c].astype(str).value_counts(normalize=True)
            fv = fake[c].astype(str).value_counts(normalize=True)
            keys = sorted(rv.index)
            p = np.array([rv.get(k, 0.0) for k in keys])
            q = np.array([fv.get(k, 0.0) for k in keys])
            out[c] = ("jsd", float(distance.jensenshannon(p, q, 2.0)) if q.sum() > 0 else 1.0)
        else:
            sc = MinMaxScaler().fit(real[[c]].values.astype(float))
            r = sc.transform(real[[c]].values.astype(float)).ravel()
            f = sc.transform(pd.to_numeric(fake[c], errors="coerce").fillna(0).values.reshape(-1, 1)).ravel()
            out[c] = ("wd", float(wasserstein_distance(r, f)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--seeds", type=int, nargs="+", default=[0])
    ap.add_argument("--rows", type=int, default=40000)
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--top", type=int, default=6)
    ap.add_argument("--gmm", default="torch", help="torch | sklearn (VGM fit backend)")
    args = ap.parse_args()
    from fed_tgan_amd.data.schema import intrusion_spec
    from fed_tgan_amd.data.synthetic import generate
    from fed_tgan_amd.eval.similarity import stat_sim
    from fed_tgan_amd.fed.runtime import FedConfig, FedRuntime
    from fed_tgan_amd.models.engine import EngineConfig
    from fed_tgan_amd.parallel.comm import Comm

    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    spec = intrusion_spec()
    for seed in args.seeds:
        out = tempfile.mkdtemp(prefix="fedtgan_q_")
        cfg = FedConfig(spec=spec, epochs=args.epochs, synthetic_rows=args.rows, out_dir=out, n_sample=40000,
                        gmm_backend=args.gmm, seed=seed, engine=EngineConfig(precision=args.precision), verbose=False,
                        async_csv=False)
        rt = FedRuntime(cfg, Comm(0, 1, [0], "gloo", device=dev), dev)
        rt.initialize()
        real = generate(spec, args.rows, seed=seed)
        for ep in range(args.epochs):
            rt.run_round(ep)
            fake = pd.read_csv(os.path.join(out, f"{spec.name}_result", f"{spec.name}_synthesis_epoch_{ep}.csv"))
            jsd, wd = stat_sim(real, fake, spec.categorical_list)
            cols = per_column(real, fake, set(spec.categorical_list))
            worst = sorted(cols.items(), key=lambda kv: -kv[1][1])[:args.top]
            print(json.dumps({"gmm": args.gmm, "seed": seed, "epoch": ep, "avg_jsd": round(jsd, 4), "avg_wd": round(wd, 4),
                              "worst": [(k, v[0], round(v[1], 4)) for k, v in worst]}), flush=True)


if __name__ == "__main__":
    main()
