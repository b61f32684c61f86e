"""Adult Dirichlet epoch-0 quality vs the VGM fit path (the follow-up of tools/adult_bisect.py).

adult_bisect.py showed that, from ONE reference initialisation, this framework's training and the reference's
give the same epoch-0 Avg_JSD (0.3247 vs 0.3249, 15-16 trials each), and that this framework's full pipeline
on the CPU (torch-op VGM fits) matches the reference too (0.3250 vs 0.3255).  The round-5 gap (0.318-0.3195)
was measured on the GPU, where every backend shares the device VGM fit (csrc/kernels/vgm_fit.hip).  This tool
runs the full federated pipeline on the GPU for several seeds with the VGM fit on

* ``hip``      : the whole-fit kernel (vgm_fit_kernel; the default on a GPU),
* ``torchdev`` : the torch-op fit on the GPU (fit_vgm_torch(use_hip=False)),
* ``passes``   : HIP data passes + torch M-step (fused=False),
* ``hip_global`` / ``hip_clients``: the whole-fit kernel only for the federator's pooled fit / the clients' fits,

and records epoch-0 Avg_JSD / Avg_WD plus every fit's valid-mode counts.

    python tools/adult_vgm_ab.py --seeds 0 1 2 3 4 5 6 7 --variants hip torchdev --out gpurun_out/vgm_ab.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from wide_quality import make_wide_split  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", default=list(range(8)))
    ap.add_argument("--variants", nargs="+", default=["hip", "torchdev"])
    ap.add_argument("--backend", default="hip")
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--work", default="/tmp/fedtgan_adult_vgm")
    ap.add_argument("--out", default=None)
    ap.add_argument("--fed", action="append", default=[], metavar="KEY=VALUE", help="FedConfig override (bool/int)")
    ap.add_argument("--tag", default="", help="suffix of the recorded variant name")
    args = ap.parse_args()
    import torch
    from fed_tgan_amd.eval.similarity import stat_sim_normalize
    from fed_tgan_amd.features import vgm_fit
    from fed_tgan_amd.fed.local import run_local_emulation
    from fed_tgan_amd.fed.runtime import FedConfig
    from fed_tgan_amd.models.engine import EngineConfig
    spec, train_path, datapath = make_wide_split(args.work, 0, 8000, 2, spec_name="adult", shard_mode="dirichlet",
                                                 alpha=0.3)
    orig = vgm_fit.fit_vgm_torch
    fits = []

    def patched(variant):
        def f(columns, *a, **k):
            is_global = isinstance(columns, torch.Tensor)      # the federator's pooled re-fit (a device tensor)
            if variant == "torchdev" or (variant == "hip_clients" and is_global) or \
                    (variant == "hip_global" and not is_global):
                k["use_hip"] = False
            elif variant == "passes":
                k["fused"] = False
            b = orig(columns, *a, **k)
            fits.append([int(x) for x in b.components().sum(1)])
            return b
        return f
    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    for seed in args.seeds:
        for var in args.variants:
            fits.clear()
            vgm_fit.fit_vgm_torch = patched(var)
            work = os.path.join(args.work, f"{var}_s{seed}")
            shutil.rmtree(work, ignore_errors=True)
            cfg = FedConfig(spec=spec, epochs=args.epochs, datapath=datapath, out_dir=work, n_sample=40000, seed=seed,
                            engine=EngineConfig(precision=args.precision), verbose=False, backend=args.backend)
            for kv in args.fed:
                key, val = kv.split("=", 1)
                setattr(cfg, key, type(getattr(cfg, key))(int(val)) if val.isdigit() else val)
            rt = run_local_emulation(cfg, 2, backend=args.backend, device=dev)
            res_dir = os.path.join(work, f"{spec.name}_result")
            res = [stat_sim_normalize(train_path, os.path.join(res_dir, f"{spec.name}_synthesis_epoch_{ep}.csv"),
                                      list(spec.categorical_list)) for ep in range(args.epochs)]
            tr = rt.transformer
            r = {"variant": var + args.tag, "seed": seed, "backend": args.backend, "precision": args.precision,
                 "avg_jsd": [float(x[0]) for x in res],
                 "avg_wd": [float(x[1]) for x in res], "fits_modes": list(fits),
                 "global_modes": [int(c.sum()) for c in tr.components], "n_opt": int(tr.layout.n_opt),
                 "global_weights": np.round(tr.bank.weights, 4).tolist(),
                 "global_means": np.round(tr.bank.means, 4).tolist(),
                 "global_stds": np.round(tr.bank.stds, 4).tolist()}
            print(json.dumps({k: r[k] for k in ("variant", "seed", "avg_jsd", "avg_wd", "global_modes", "n_opt")}),
                  flush=True)
            if args.out:
                with open(args.out, "a") as f:
                    f.write(json.dumps(r) + "\n")
            shutil.rmtree(work, ignore_errors=True)
    vgm_fit.fit_vgm_torch = orig


if __name__ == "__main__":
    main()
