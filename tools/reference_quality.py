"""Quality of the REFERENCE implementation on exactly the data `tools/real_quality.py` uses.

The reference's README numbers (Avg_JSD / Avg_WD 0.19 / 0.08 after epoch 0, 0.082 / 0.04 after
epoch 1, `R/README.md:53-54`) come from one run on the 40k-row train split, which is not shipped.
This tool runs the reference's own federated code offline, on the CPU, on the same 2-client split of
the shipped `Intrusion_test.csv` (80 / 20 split, clients resampled to 20,000 rows each: ~40 steps per
client per epoch, like the README run), so the comparison with this framework is like for like:

* `MDGANClient` / `MDGANServer` from `Server/dtds/distributed.py`, driven through the same in-process
  RRef stand-ins as `tools/make_goldens.py` (the PyTorch RPC layer cannot run on torch 2.10),
  including the server's `fit()` round loop, weighted `average_model`, `sample_data` and CSV dump;
* the server's sampling `Cond` is built from the clients' encoded rows (`models/Intrusion_train.npz`,
  as the reference expects);
* every epoch CSV is scored with the reference's `stat_sim_normalize` against the 8,078 real rows.

Nothing is imported from the reference at test time; this writes `profiles/reference_quality_r2.json`.

    python tools/reference_quality.py --epochs 3 --seeds 0 1 2 3
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import shutil
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from make_goldens import CATEGORICAL, NONNEG, PROBLEM, SELECTED, TARGET, FakeRRef  # noqa: E402
from real_quality import make_split  # noqa: E402  (imported before the reference goes on sys.path)


def _by_value(x):
    """What an RPC peer receives: a copy (PyTorch RPC pickles every argument and return value)."""
    return copy.deepcopy(x)


class _ByValue:
    """Method proxy with RPC by-value semantics: arguments and the result are copied.

    The in-process stand-ins of `make_goldens.py` hand back the client's live objects.  Under those,
    `MDGANServer.fit()` (`Server/dtds/distributed.py:789`) takes client 0's OWN generator as the
    server's, and `sample()` (`:161`) then calls `generator.eval()` on it -- client 0 would train every
    later round with eval-mode BatchNorm (running statistics, never updated).  Over real RPC the
    server holds a pickled copy, and client 0 keeps training in train mode."""

    def __init__(self, obj, wrap, copy: bool = True):
        self.obj, self.wrap, self.copy = obj, wrap, copy

    def __getattr__(self, name):
        f = getattr(self.obj, name)
        if not self.copy:
            return lambda *a, **k: self.wrap(f(*a, **k))
        return lambda *a, **k: self.wrap(_by_value(f(*_by_value(a), **_by_value(k))))


class _Fut:
    def __init__(self, v):
        self.v = v

    def to_here(self):
        return self.v

    def wait(self):
        return self.v


class FakeRRefAsync(FakeRRef):
    """RRef stand-in; ``by_value`` (default) gives RPC copy semantics, False the live-object aliasing
    of the round-2 tool (kept to reproduce `profiles/reference_quality_r2.json`)."""

    def __init__(self, obj, by_value: bool = True):
        super().__init__(obj)
        self.by_value = by_value

    def remote(self):
        return _ByValue(self.obj, _Fut, self.by_value)

    def rpc_sync(self):
        return _ByValue(self.obj, lambda v: v, self.by_value)

    def rpc_async(self):
        return _ByValue(self.obj, _Fut, self.by_value)


def run_seed(ref_dir: str, work: str, seed: int, epochs: int, bootstrap: int, csv_epochs=None,
             utility: bool = False, by_value: bool = True) -> dict:
    import pandas as pd
    import torch
    os.makedirs(work)
    os.chdir(work)
    for d in ("models", "Intrusion_result"):
        os.makedirs(d)
    train_path, _, datapath = make_split(work, 2, bootstrap_rows=bootstrap)
    np.random.seed(seed)
    torch.manual_seed(seed)
    import dtds.distributed as rdist        # (reference)
    assert os.path.abspath(rdist.__file__).startswith(os.path.abspath(ref_dir)), rdist.__file__
    import similarity_analysis as rsim      # (reference)
    t0 = time.time()
    clients = [rdist.MDGANClient(datapath.format(client=i), list(SELECTED), list(CATEGORICAL), list(NONNEG), {},
                                 TARGET, PROBLEM, epochs) for i in range(2)]
    server = rdist.MDGANServer([FakeRRefAsync(c, by_value) for c in clients], epochs)
    server.uniform_meta_category()
    server.uniform_continuous_gmm()
    server.refit_local_transformer()
    server.calculate_final_weights_for_aggregation()
    np.savez(os.path.join("models", "Intrusion_train.npz"), train=np.concatenate([c.train for c in clients]))
    server.server_local_synthesizer_initialization()
    t_init = time.time() - t0
    if csv_epochs is not None:      # long runs: the reference's sample_data only on the scored epochs
        keep = set(csv_epochs) | {epochs - 1}
        orig = server.sample_data
        server.sample_data = lambda i: orig(i) if i in keep else None
    server.fit()
    times = pd.read_csv("timestamp_experiment.csv", header=None).iloc[:, 0].tolist()
    res = []
    scored = sorted(set(csv_epochs) | {epochs - 1}) if csv_epochs is not None else list(range(epochs))
    for ep in scored:
        jsd, wd = rsim.stat_sim_normalize(train_path, f"Intrusion_result/Intrusion_synthesis_epoch_{ep}.csv",
                                          list(CATEGORICAL))
        res.append((float(jsd), float(wd)))
    out = {"seed": seed, "init_s": t_init, "round_s": times, "epochs": scored, "avg_jsd": [r[0] for r in res],
           "avg_wd": [r[1] for r in res], "weights": np.asarray(server.weights_con_cat_combination).tolist(),
           "steps_per_epoch": [int(c.steps_per_epoch) for c in clients]}
    if utility:     # the reference's utility_analysis protocol on the last epoch (real vs synthetic rows)
        import utility_analysis as rutil    # (reference)
        real, hold = pd.read_csv(train_path), pd.read_csv(os.path.join(os.path.dirname(train_path), "holdout.csv"))
        fake = pd.read_csv(f"Intrusion_result/Intrusion_synthesis_epoch_{epochs - 1}.csv")
        orig_real = pd.concat([real, hold])
        ru = rutil.real_res(orig_real, real, hold, TARGET, list(CATEGORICAL))
        fu = rutil.real_res(orig_real, fake, hold, TARGET, list(CATEGORICAL))
        diff = np.asarray(ru) - np.asarray(fu)
        out["utility_final"] = {"diff": diff.tolist(), "f1_gap": float(diff.mean(axis=0)[1])}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference/Server")
    ap.add_argument("--work", default="/tmp/fedtgan_refq")
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1, 2, 3])
    ap.add_argument("--bootstrap-rows", type=int, default=20000)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "reference_quality_r2.json"))
    ap.add_argument("--csv-epochs", type=int, nargs="*", default=None, help="only these epochs' CSVs (+ the last)")
    ap.add_argument("--utility", action="store_true", help="ML-utility gap of the last epoch")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--aliased", action="store_true",
                    help="round-2 harness: RRef stand-ins hand back live objects (client 0's generator is the "
                         "server's and is switched to eval mode by the first sample_data)")
    args = ap.parse_args()
    shutil.rmtree(args.work, ignore_errors=True)
    shim = os.path.join(args.work, "shim")
    os.makedirs(shim)
    with open(os.path.join(shim, "pickle5.py"), "w") as f:
        f.write("from pickle import *  # noqa\nfrom pickle import HIGHEST_PROTOCOL, dump, dumps, load, loads  # noqa\n")
    sys.dont_write_bytecode = True
    sys.path[:0] = [shim, args.reference]      # ahead of this repo's own `dtds` shim
    import torch
    torch.set_num_threads(args.threads or os.cpu_count() or 8)
    runs = []
    for seed in args.seeds:
        r = run_seed(args.reference, os.path.join(args.work, f"s{seed}"), seed, args.epochs, args.bootstrap_rows,
                     args.csv_epochs, args.utility, by_value=not args.aliased)
        runs.append(r)
        print(json.dumps(r), flush=True)
    summary = {"epochs": runs[0]["epochs"],
               "avg_jsd_mean": np.mean([r["avg_jsd"] for r in runs], axis=0).round(4).tolist(),
               "avg_wd_mean": np.mean([r["avg_wd"] for r in runs], axis=0).round(4).tolist(),
               "avg_jsd_sem": (np.std([r["avg_jsd"] for r in runs], axis=0, ddof=1) / np.sqrt(len(runs))).round(4).tolist()
               if len(runs) > 1 else None,
               "rpc_semantics": "aliased" if args.aliased else "by_value",
               "round_s_mean": float(np.mean([np.mean(r["round_s"]) for r in runs]))}
    if args.utility:
        summary["f1_gap_mean"] = float(np.mean([r["utility_final"]["f1_gap"] for r in runs]))
    with open(args.out, "w") as f:
        json.dump({"protocol": __doc__, "bootstrap_rows": args.bootstrap_rows, "runs": runs, "summary": summary}, f,
                  indent=1)
    print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
