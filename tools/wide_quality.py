"""Training quality on a reduced WIDE table (or a built-in spec, --spec adult / covertype, optionally with
Dirichlet non-IID shards): the reference's own code vs this framework, same data.

BASELINE config 5 (100k rows x 512 columns) has no published reference number, and the reference's
CPU code cannot train it in reasonable time.  This tool builds a reduced wide table the reference CAN
run (``wide:<n_cols>`` from ``fed_tgan_amd.data.synthetic.generate_wide``: half continuous columns
with 1-4 latent modes, half categorical columns of 2-31 values, all tied to one latent class), splits
it over ``--clients`` client CSVs, and trains it

* ``--impl reference``: with the reference's federated code (``MDGANClient`` / ``MDGANServer`` of
  `Server/dtds/distributed.py`, sklearn VGMs, PyTorch autograd on the CPU), driven offline through the
  RPC stand-ins of `tools/reference_quality.py` (by-value semantics).  Every epoch CSV is scored with the
  reference's ``stat_sim_normalize`` (`Server/similarity_analysis.py:15-82`).
* ``--impl ours``: with this framework (``run_local_emulation``: the same clients on one device), on the
  HIP backend (``--backend hip``, GPU) or the eager torch oracle (``--backend torch``, ``ops/ref.py``).
  ``--force-wide`` forces the kernel paths only the 512-column table takes by default: the scattered
  one-hot weight gradients (``EngineConfig.onehot_wgrad_min = 1``), the register-resident activation row
  kernels and the chunk-split gradient-penalty scale (their thresholds are below this table's widths).
  Every epoch CSV is scored with ``fed_tgan_amd.eval.similarity.stat_sim_normalize`` (byte-compatible
  with the reference's, `tests/test_golden.py`).

Both sample 40,000 rows per epoch (the reference's literal, `Server/dtds/distributed.py:583`) and score
against the union of the client shards.  One JSON line per seed; ``--out`` collects them.

    python tools/wide_quality.py --impl reference --cols 128 --seeds 0 1 2 3 4 5 --epochs 8      # CPU
    python tools/wide_quality.py --impl ours --backend hip --force-wide --cols 128 --seeds 0 ... # GPU
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from fed_tgan_amd.data.schema import get_spec, wide_spec  # noqa: E402
from fed_tgan_amd.data.synthetic import generate, shard  # noqa: E402


def make_wide_split(out: str, n_cols: int, rows: int, clients: int, seed: int = 2025, spec_name: str | None = None,
                    shard_mode: str = "contiguous", alpha: float = 0.3):
    """``rows`` per client of the ``wide:<n_cols>`` table (or of a built-in spec: ``spec_name`` = adult /
    covertype / intrusion); train.csv = the union of the shards.  shard_mode "dirichlet": label-skewed
    Dirichlet(alpha) shards of the spec's target column (``data.synthetic.shard``), the non-IID config-4 split."""
    spec = get_spec(spec_name) if spec_name else wide_spec(n_cols)
    df = generate(spec, rows * clients, seed=seed)
    d = os.path.join(out, "data")
    os.makedirs(d, exist_ok=True)
    train = os.path.join(d, "train.csv")
    if not os.path.exists(train):
        df.to_csv(train, index=False)
        if shard_mode == "dirichlet":
            parts = shard(df, clients, "dirichlet", seed=seed, target=spec.target_column, alpha=alpha)
        else:
            parts = [df.iloc[p] for p in np.array_split(np.arange(len(df)), clients)]
        for i, part in enumerate(parts):
            part.to_csv(os.path.join(d, f"client{i}.csv"), index=False)
    return spec, train, os.path.join(d, "client{client}.csv")


def run_reference(ref_dir: str, work: str, spec, train_path: str, datapath: str, clients: int, seed: int,
                  epochs: int) -> dict:
    import pandas as pd
    import torch
    from reference_quality import FakeRRefAsync     # (imported in main, before the reference's path)
    shutil.rmtree(work, ignore_errors=True)
    os.makedirs(work)
    os.chdir(work)
    for d in ("models", "Intrusion_result"):
        os.makedirs(d)
    np.random.seed(seed)
    torch.manual_seed(seed)
    import dtds.distributed as rdist        # (reference)
    assert os.path.abspath(rdist.__file__).startswith(os.path.abspath(ref_dir)), rdist.__file__
    import similarity_analysis as rsim      # (reference)
    t0 = time.time()
    cs = [rdist.MDGANClient(datapath.format(client=i), list(spec.selected_variables), list(spec.categorical_list),
                            list(spec.nonnegative_list), dict(spec.date_dic), spec.target_column, spec.problem_type,
                            epochs) for i in range(clients)]
    server = rdist.MDGANServer([FakeRRefAsync(c) for c in cs], epochs)
    server.uniform_meta_category()
    server.uniform_continuous_gmm()
    server.refit_local_transformer()
    server.calculate_final_weights_for_aggregation()
    np.savez(os.path.join("models", "Intrusion_train.npz"), train=np.concatenate([c.train for c in cs]))
    server.server_local_synthesizer_initialization()
    t_init = time.time() - t0
    server.fit()
    times = pd.read_csv("timestamp_experiment.csv", header=None).iloc[:, 0].tolist()
    res = [rsim.stat_sim_normalize(train_path, f"Intrusion_result/Intrusion_synthesis_epoch_{ep}.csv",
                                   list(spec.categorical_list)) for ep in range(epochs)]
    shutil.rmtree(os.path.join(work, "Intrusion_result"), ignore_errors=True)
    return {"impl": "reference", "seed": seed, "init_s": t_init, "round_s": times,
            "avg_jsd": [float(r[0]) for r in res], "avg_wd": [float(r[1]) for r in res],
            "weights": np.asarray(server.weights_con_cat_combination).tolist(),
            "data_dim": int(cs[0].train.shape[1]), "steps_per_epoch": [int(c.steps_per_epoch) for c in cs]}


def run_ours(work: str, spec, train_path: str, datapath: str, clients: int, seed: int, epochs: int,
             backend: str, precision: str, force_wide: bool) -> dict:
    import torch
    from fed_tgan_amd.eval.similarity import stat_sim_normalize
    from fed_tgan_amd.fed.local import run_local_emulation
    from fed_tgan_amd.fed.runtime import FedConfig
    from fed_tgan_amd.models.engine import EngineConfig
    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    shutil.rmtree(work, ignore_errors=True)
    ecfg = EngineConfig(precision=precision)
    if force_wide:
        ecfg.onehot_wgrad_min = 1
    cfg = FedConfig(spec=spec, epochs=epochs, datapath=datapath, out_dir=work, n_sample=40000, seed=seed,
                    engine=ecfg, verbose=False, backend=backend)
    t0 = time.time()
    rt = run_local_emulation(cfg, clients, backend=backend, device=dev)
    wall = time.time() - t0
    res_dir = os.path.join(work, f"{spec.name}_result")
    res = [stat_sim_normalize(train_path, os.path.join(res_dir, f"{spec.name}_synthesis_epoch_{ep}.csv"),
                              list(spec.categorical_list)) for ep in range(epochs)]
    shutil.rmtree(res_dir, ignore_errors=True)
    return {"impl": f"ours-{backend}-{precision}" + ("-forcewide" if force_wide else ""), "seed": seed,
            "wall_s": wall, "round_s": [float(x) for x in rt.round_times],
            "avg_jsd": [float(r[0]) for r in res], "avg_wd": [float(r[1]) for r in res],
            "weights": [float(w) for w in rt.weights], "steps": rt.steps}


def summarize(runs):
    out = {}
    for impl in sorted({r["impl"] for r in runs}):
        rs = [r for r in runs if r["impl"] == impl]
        j, w = np.asarray([r["avg_jsd"] for r in rs]), np.asarray([r["avg_wd"] for r in rs])
        n = len(rs)
        out[impl] = {"n": n, "avg_jsd_mean": j.mean(0).round(4).tolist(), "avg_wd_mean": w.mean(0).round(4).tolist(),
                     "avg_jsd_sem": (j.std(0, ddof=1) / np.sqrt(n)).round(4).tolist() if n > 1 else None,
                     "avg_wd_sem": (w.std(0, ddof=1) / np.sqrt(n)).round(4).tolist() if n > 1 else None}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--impl", choices=["reference", "ours"], required=True)
    ap.add_argument("--reference", default="/root/reference/Server")
    ap.add_argument("--cols", type=int, default=128)
    ap.add_argument("--spec", default=None, help="a built-in spec (adult, covertype, intrusion) instead of wide:<cols>")
    ap.add_argument("--shard", default="contiguous", choices=["contiguous", "dirichlet"])
    ap.add_argument("--alpha", type=float, default=0.3, help="Dirichlet concentration of --shard dirichlet")
    ap.add_argument("--rows", type=int, default=10000, help="rows per client")
    ap.add_argument("--clients", type=int, default=2)
    ap.add_argument("--epochs", type=int, default=8)
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1, 2, 3, 4, 5])
    ap.add_argument("--backend", default="hip", choices=["hip", "torch", "auto"])
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--force-wide", action="store_true")
    ap.add_argument("--tuning", action="append", default=[], metavar="KEY=VALUE", help="native set_tuning knob")
    ap.add_argument("--work", default="/tmp/fedtgan_wideq")
    ap.add_argument("--out", default=None, help="append one JSON line per seed to this file")
    ap.add_argument("--threads", type=int, default=0)
    args = ap.parse_args()
    spec, train_path, datapath = make_wide_split(args.work, args.cols, args.rows, args.clients, spec_name=args.spec,
                                                 shard_mode=args.shard, alpha=args.alpha)
    if args.impl == "reference":
        import reference_quality  # noqa: F401  (it puts this repo first on sys.path: import it before the reference)
        shim = os.path.join(args.work, "shim")
        os.makedirs(shim, exist_ok=True)
        with open(os.path.join(shim, "pickle5.py"), "w") as f:
            f.write("from pickle import *  # noqa\nfrom pickle import HIGHEST_PROTOCOL, dump, dumps, load, loads  # noqa\n")
        sys.dont_write_bytecode = True
        sys.path[:0] = [shim, args.reference]      # ahead of this repo's own `dtds` shim
    import torch
    if args.threads:
        torch.set_num_threads(args.threads)
    if args.tuning:
        from fed_tgan_amd.ops import native
        for kv in args.tuning:
            k, v = kv.split("=", 1)
            native.require().set_tuning(k, int(v))
    runs = []
    for seed in args.seeds:
        work = os.path.join(args.work, f"{args.impl}_s{seed}")
        if args.impl == "reference":
            r = run_reference(args.reference, work, spec, train_path, datapath, args.clients, seed, args.epochs)
        else:
            r = run_ours(work, spec, train_path, datapath, args.clients, seed, args.epochs, args.backend,
                         args.precision, args.force_wide)
        r.update({"spec": spec.name, "shard": args.shard, "cols": args.cols, "rows_per_client": args.rows,
                  "clients": args.clients, "tuning": args.tuning})
        runs.append(r)
        print(json.dumps(r), flush=True)
        if args.out:
            with open(args.out, "a") as f:
                f.write(json.dumps(r) + "\n")
    print(json.dumps(summarize(runs)), flush=True)


if __name__ == "__main__":
    main()
