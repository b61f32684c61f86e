"""Real-data quality: Avg_JSD / Avg_WD per epoch and the ML-utility gap on the shipped Intrusion split.

The only real table that ships with the reference is `Server/data/raw/Intrusion_test.csv`
(10,098 x 42, vendored as ``data/raw/Intrusion_test.csv``).  Protocol:

* a fixed 80 / 20 split (permutation seed 2024): 8,078 training rows, 2,020 held-out rows;
* the training rows split into 2 client CSVs (first / second half of the training rows) -- the
  README's 2-client federation (`R/README.md:7-25`);
* a 2-client federation (in-process emulation: 2 clients on one GPU, one HIP stream each) with the
  reference defaults (batch 500, 40,000 sampled rows per epoch), ``--epochs`` rounds, per precision
  and seed;
* Avg_JSD / Avg_WD of every epoch CSV against the 8,078 real training rows, with the reference
  evaluator definitions (`Server/similarity_analysis.py:15-82`) -- the published numbers are
  0.19 / 0.08 after epoch 0 and 0.082 / 0.04 after epoch 1 (`R/README.md:53-54`, 2 clients on the
  ~40k-row train split: ~40 steps per client per epoch; here 8 steps per client per epoch);
* ML utility of the final epoch CSV: `Server/utility_analysis.py` protocol (LR / DT / RF / MLP,
  random_state 69) trained on real vs synthetic rows, tested on the 2,020 held-out rows; the
  published gap is a weighted-F1 difference of 0.0849 at epoch 499 (`R/README.md:67`).

    python tools/real_quality.py --epochs 10 --seeds 0 1 2 3 --precisions bf16 fp32 --out gpurun_out/quality
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np
import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
DATA = os.path.join(ROOT, "data", "raw", "Intrusion_test.csv")


def make_split(out: str, n_clients: int = 2, seed: int = 2024, bootstrap_rows: int = 0):
    df = pd.read_csv(DATA)
    perm = np.random.default_rng(seed).permutation(len(df))
    n_tr = int(round(0.8 * len(df)))
    train, hold = df.iloc[perm[:n_tr]].reset_index(drop=True), df.iloc[perm[n_tr:]].reset_index(drop=True)
    d = os.path.join(out, "data")
    os.makedirs(d, exist_ok=True)
    train.to_csv(os.path.join(d, "train.csv"), index=False)
    hold.to_csv(os.path.join(d, "holdout.csv"), index=False)
    bounds = np.linspace(0, len(train), n_clients + 1).astype(int)
    rng = np.random.default_rng(seed + 1)
    for i in range(n_clients):
        part = train.iloc[bounds[i]:bounds[i + 1]]
        if bootstrap_rows:   # resample with replacement to the reference's per-client size (steps/epoch)
            part = part.iloc[rng.integers(0, len(part), bootstrap_rows)]
        part.to_csv(os.path.join(d, f"client{i}.csv"), index=False)
    return os.path.join(d, "train.csv"), os.path.join(d, "holdout.csv"), os.path.join(d, "client{client}.csv")


def train_run(out: str, datapath: str, precision: str, seed: int, epochs: int, clients: int, gmm: str,
              csv_epochs=None, batched: str = "auto", init: str = "independent", host_encode: bool = False):
    import torch
    from fed_tgan_amd.data.schema import intrusion_spec
    from fed_tgan_amd.fed.local import run_local_emulation
    from fed_tgan_amd.fed.runtime import FedConfig
    from fed_tgan_amd.models.engine import EngineConfig
    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    cfg = FedConfig(spec=intrusion_spec(), epochs=epochs, datapath=datapath, out_dir=out, n_sample=40000,
                    gmm_backend=gmm, seed=seed, engine=EngineConfig(precision=precision), verbose=False,
                    batched_clients=batched, init=init, device_encode=not host_encode)
    if csv_epochs is not None:      # long runs: only the scored epochs' tables are written
        cfg.csv_epochs = sorted(set(csv_epochs))
    t0 = time.time()
    rt = run_local_emulation(cfg, clients, backend="auto", device=dev)
    return {"rows": rt.rows, "steps": rt.steps, "weights": [float(w) for w in rt.weights],
            "batched": bool(getattr(rt, "batched", False)),
            "wall_s": time.time() - t0, "round_s": [float(x) for x in rt.round_times]}


def similarity(train_path: str, run_dir: str, epochs):
    from fed_tgan_amd.data.schema import intrusion_spec
    from fed_tgan_amd.eval.similarity import stat_sim_normalize
    cats = intrusion_spec().categorical_list
    res = []
    for ep in epochs:
        p = os.path.join(run_dir, "Intrusion_result", f"Intrusion_synthesis_epoch_{ep}.csv")
        jsd, wd = stat_sim_normalize(train_path, p, cats)
        res.append((float(jsd), float(wd)))
    return res


def utility(train_path: str, hold_path: str, fake_path: str):
    import warnings
    warnings.simplefilter("ignore")
    from fed_tgan_amd.data.schema import intrusion_spec
    from fed_tgan_amd.eval.utility import utility_difference
    spec = intrusion_spec()
    train, hold, fake = pd.read_csv(train_path), pd.read_csv(hold_path), pd.read_csv(fake_path)
    diff, f1_gap = utility_difference(train, hold, fake, spec.target_column, spec.categorical_list, verbose=False)
    return {"diff": diff.tolist(), "f1_gap": f1_gap}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1, 2, 3])
    ap.add_argument("--precisions", nargs="+", default=["bf16", "fp32"])
    ap.add_argument("--clients", type=int, default=2)
    ap.add_argument("--gmm", default="torch")
    ap.add_argument("--out", default="gpurun_out/quality")
    ap.add_argument("--utility-workers", type=int, default=8)
    ap.add_argument("--keep-csv", action="store_true")
    ap.add_argument("--eval-epochs", type=int, nargs="*", default=None, help="epochs to score (default: all)")
    ap.add_argument("--bootstrap-rows", type=int, default=0,
                    help="resample every client's rows (with replacement) to this many: 20000 gives the "
                         "reference's ~40 steps per client per epoch")
    ap.add_argument("--only-scored-csv", action="store_true", help="write only the scored epochs' CSVs")
    ap.add_argument("--init", default="independent", choices=["independent", "broadcast"])
    ap.add_argument("--no-utility", action="store_true", help="skip the ML-utility evaluation of the last epoch")
    ap.add_argument("--batched", default="auto", choices=["auto", "on", "off"],
                    help="FedConfig.batched_clients: the clients' steps as one batched engine, or one per thread")
    ap.add_argument("--host-encode", action="store_true",
                    help="FedConfig.device_encode off: VGM-encode the rows on the host (numpy) instead of the HIP kernel")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    train_path, hold_path, datapath = make_split(args.out, args.clients, bootstrap_rows=args.bootstrap_rows)
    eval_epochs = [e for e in (args.eval_epochs or range(args.epochs)) if e < args.epochs]
    runs = []
    for prec in args.precisions:
        for seed in args.seeds:
            rd = os.path.join(args.out, f"run_{prec}_s{seed}")
            info = train_run(rd, datapath, prec, seed, args.epochs, args.clients, args.gmm,
                             eval_epochs if args.only_scored_csv else None, args.batched, args.init,
                             args.host_encode)
            sims = similarity(train_path, rd, eval_epochs)
            rec = {"precision": prec, "seed": seed, **info, "eval_epochs": eval_epochs, "avg_jsd": [s[0] for s in sims],
                   "avg_wd": [s[1] for s in sims]}
            runs.append(rec)
            print(json.dumps({k: rec[k] for k in ("precision", "seed", "avg_jsd", "avg_wd", "steps")}), flush=True)
    # ML utility of each run's final epoch (CPU, parallel processes)
    last = args.epochs - 1
    fakes = [os.path.join(args.out, f"run_{r['precision']}_s{r['seed']}", "Intrusion_result",
                          f"Intrusion_synthesis_epoch_{last}.csv") for r in runs]
    if args.no_utility:
        utils = [{"diff": None, "f1_gap": float("nan")} for _ in fakes]
    else:
        with ProcessPoolExecutor(max_workers=args.utility_workers) as ex:
            utils = list(ex.map(utility, [train_path] * len(fakes), [hold_path] * len(fakes), fakes))
    for r, u in zip(runs, utils):
        r["utility_final"] = u
        print(json.dumps({"precision": r["precision"], "seed": r["seed"], "f1_gap": u["f1_gap"]}), flush=True)
    summary = {}
    for prec in args.precisions:
        rs = [r for r in runs if r["precision"] == prec]
        summary[prec] = {"avg_jsd_mean": np.mean([r["avg_jsd"] for r in rs], axis=0).round(4).tolist(),
                         "avg_jsd_sem": (np.std([r["avg_jsd"] for r in rs], axis=0, ddof=1) /
                                         np.sqrt(len(rs))).round(4).tolist() if len(rs) > 1 else None,
                         "avg_wd_mean": np.mean([r["avg_wd"] for r in rs], axis=0).round(4).tolist(),
                         "f1_gap_mean": float(np.mean([r["utility_final"]["f1_gap"] for r in rs])),
                         "avg_wd_sem": (np.std([r["avg_wd"] for r in rs], axis=0, ddof=1) /
                                        np.sqrt(len(rs))).round(4).tolist() if len(rs) > 1 else None,
                         "eval_epochs": eval_epochs, "bootstrap_rows": args.bootstrap_rows,
                         "gmm": args.gmm, "init": args.init, "batched": args.batched,
                         "host_encode": args.host_encode,
                         "seeds": [r["seed"] for r in rs]}
    with open(os.path.join(args.out, "real_quality.json"), "w") as f:
        json.dump({"protocol": __doc__, "runs": runs, "summary": summary}, f, indent=1)
    print(json.dumps(summary), flush=True)
    if not args.keep_csv:
        import shutil
        for r in runs:
            shutil.rmtree(os.path.join(args.out, f"run_{r['precision']}_s{r['seed']}", "Intrusion_result"),
                          ignore_errors=True)


if __name__ == "__main__":
    main()
