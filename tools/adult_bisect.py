"""Bisect the Adult unequal-client epoch-0 quality gap with artefacts, not seeds.

The reference's own federated code (`Server/dtds/distributed.py`, `Client/.../dtds/distributed.py`) and this
framework give different epoch-0 Avg_JSD on the Dirichlet(0.3) Adult split (2 clients, 11 / 20 steps):
0.3246 (reference) vs 0.318-0.3195 (ours, all three backends; profiles/quality_configs_r5.txt).  This tool
fixes everything that can be fixed -- ONE reference initialisation (its sklearn VGMs, label encoders, encoded
client matrices, the server's generation ``Cond`` and transformer) -- and then swaps one stage at a time:

* ``ref``     : reference train_model on both clients -> reference average_model -> reference sample_data
* ``ours``    : this framework's CTGANEngine (eager torch oracle, fp32, CPU) trained on the SAME encoded client
                matrices -> reference-layout state dicts -> reference average_model -> reference sample_data
* ``ref_bn0`` : as ``ref`` but every client's G BatchNorm running statistics reset to (0, 1) before aggregation
* ``ours_seq``: as ``ours`` with the unpaired (reference-order) step: D step, then G step, each drawing its own batch

Every arm's epoch-0 CSV is scored with the reference's ``stat_sim_normalize`` against the union of the shards;
diagnostics of the aggregated generator (BN running statistics, output-logit scale) are recorded per trial.

    python tools/adult_bisect.py --trials 8 --arms ref ours --out profiles/adult_epoch0_r6.jsonl
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import pickle
import shutil
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from wide_quality import make_wide_split  # noqa: E402


def ref_init(spec, datapath: str, clients: int, seed: int):
    import torch
    from reference_quality import FakeRRefAsync
    import dtds.distributed as rdist        # (reference)
    np.random.seed(seed)
    torch.manual_seed(seed)
    cs = [rdist.MDGANClient(datapath.format(client=i), list(spec.selected_variables), list(spec.categorical_list),
                            list(spec.nonnegative_list), dict(spec.date_dic), spec.target_column, spec.problem_type,
                            1) for i in range(clients)]
    server = rdist.MDGANServer([FakeRRefAsync(c) for c in cs], 1)
    server.uniform_meta_category()
    server.uniform_continuous_gmm()
    server.refit_local_transformer()
    server.calculate_final_weights_for_aggregation()
    np.savez(os.path.join("models", "Intrusion_train.npz"), train=np.concatenate([c.train for c in cs]))
    server.server_local_synthesizer_initialization()
    return cs, server


def fresh_modules(c):
    """What `Client/.../distributed.py:156-168` builds in refit_transformer (new random init, new Adam)."""
    import torch.optim as optim
    from dtds.synthesizers import ctgan     # (reference)
    c.generator = ctgan.Generator(c.embedding_dim + c.cond_generator.n_opt, c.gen_dim, c.transformer.output_dim)
    c.discriminator = ctgan.Discriminator(input_dim=c.data_dim + c.cond_generator.n_opt, dis_dims=c.dis_dim)
    c.optG = optim.Adam(c.generator.parameters(), lr=2e-4, betas=(0.5, 0.9), weight_decay=c.l2scale)
    c.optD = optim.Adam(c.discriminator.parameters(), lr=2e-4, betas=(0.5, 0.9))


def ours_train(c, seed: int, paired: bool = True):
    """This framework's engine (eager torch oracle, fp32) on the reference client's encoded matrix."""
    from fed_tgan_amd.features.transformer import SpanLayout
    from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig
    lay = SpanLayout.from_output_info(c.out_info)
    eng = CTGANEngine(lay, EngineConfig(precision="fp32", paired=paired), "cpu", backend="torch", seed=seed)
    eng.set_training_data(np.asarray(c.sampler.data, dtype=np.float32))
    assert eng.steps_per_epoch == c.steps_per_epoch, (eng.steps_per_epoch, c.steps_per_epoch)
    eng.train_steps(c.steps_per_epoch, use_graph=False)
    return eng.g_state_dict(), eng.d_state_dict()


def gen_diag(server, n: int = 4000) -> dict:
    """Aggregated generator: BN running statistics and the scale of the output logits (eval mode)."""
    import torch
    g = server.generator
    g.eval()
    sd = g.state_dict()
    out = {}
    for k, v in sd.items():
        if k.endswith("running_mean"):
            out[k] = float(v.abs().mean())
        elif k.endswith("running_var"):
            out[k] = float(v.mean())
    with torch.no_grad():
        z = torch.randn(n, server.embedding_dim)
        c1 = torch.from_numpy(server.cond_generator.sample_zero(n))
        logits = g(torch.cat([z, c1], 1))
    out["logit_std"] = float(logits.std())
    return out


def run_trial(arm: str, cs, server, trial: int, train_path: str, cat_cols) -> dict:
    import torch
    import dtds.distributed as rdist        # (reference)
    import similarity_analysis as rsim      # (reference)
    np.random.seed(10007 * trial + 11)
    torch.manual_seed(10007 * trial + 11)
    g_dicts, d_dicts = [], []
    for i, c in enumerate(cs):
        if arm.startswith("ref"):
            fresh_modules(c)
            g, d = copy.deepcopy(c.train_model(1))
            if arm == "ref_bn0":
                for k in g:
                    if k.endswith("running_mean"):
                        g[k].zero_()
                    elif k.endswith("running_var"):
                        g[k].fill_(1.0)
        else:
            g, d = ours_train(c, seed=7919 * trial + 31 * i + 5, paired=(arm != "ours_seq"))
        g_dicts.append(g)
        d_dicts.append(d)
    w = server.weights_con_cat_combination
    if server.generator is None:
        server.generator = copy.deepcopy(cs[0].generator)
    server.generator.load_state_dict(rdist.average_model(g_dicts, w))
    np.random.seed(5003 * trial + 3)
    torch.manual_seed(5003 * trial + 3)
    server.sample_data(trial)
    csv = f"Intrusion_result/Intrusion_synthesis_epoch_{trial}.csv"
    jsd, wd = rsim.stat_sim_normalize(train_path, csv, list(cat_cols))
    os.remove(csv)
    rec = {"arm": arm, "trial": trial, "avg_jsd": float(jsd), "avg_wd": float(wd)}
    rec.update(gen_diag(server))
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference/Server")
    ap.add_argument("--work", default="/tmp/fedtgan_adult_bisect")
    ap.add_argument("--seed", type=int, default=0, help="reference initialisation seed (sklearn VGMs, encode)")
    ap.add_argument("--trials", type=int, default=6)
    ap.add_argument("--first-trial", type=int, default=0)
    ap.add_argument("--arms", nargs="+", default=["ref", "ours"])
    ap.add_argument("--threads", type=int, default=2)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    spec, train_path, datapath = make_wide_split(args.work, 0, 8000, 2, spec_name="adult", shard_mode="dirichlet",
                                                 alpha=0.3)
    import reference_quality  # noqa: F401  (puts this repo first on sys.path: import it before the reference)
    shim = os.path.join(args.work, "shim")
    os.makedirs(shim, exist_ok=True)
    with open(os.path.join(shim, "pickle5.py"), "w") as f:
        f.write("from pickle import *  # noqa\nfrom pickle import HIGHEST_PROTOCOL, dump, dumps, load, loads  # noqa\n")
    sys.dont_write_bytecode = True
    sys.path[:0] = [shim, args.reference]
    import torch
    torch.set_num_threads(args.threads)
    work = os.path.join(args.work, f"init_s{args.seed}")
    cache = os.path.join(work, "init.pkl")      # written by this tool (own file)
    os.makedirs(work, exist_ok=True)
    os.chdir(work)
    for d in ("models", "Intrusion_result"):
        os.makedirs(d, exist_ok=True)
    t0 = time.time()
    if os.path.exists(cache):
        import dtds.distributed  # noqa: F401  (classes for the unpickler)
        with open(cache, "rb") as f:
            cs, server = pickle.load(f)
    else:
        cs, server = ref_init(spec, datapath, 2, args.seed)
        server.generator = None
        with open(cache + ".tmp", "wb") as f:
            pickle.dump((cs, server), f)
        os.replace(cache + ".tmp", cache)
    print(f"[init] {time.time() - t0:.1f}s steps={[c.steps_per_epoch for c in cs]} "
          f"weights={list(server.weights_con_cat_combination)}", flush=True)
    for t in range(args.first_trial, args.first_trial + args.trials):
        for arm in args.arms:
            t1 = time.time()
            r = run_trial(arm, cs, server, t, train_path, spec.categorical_list)
            r.update({"init_seed": args.seed, "secs": round(time.time() - t1, 1)})
            print(json.dumps(r), flush=True)
            if args.out:
                with open(args.out, "a") as f:
                    f.write(json.dumps(r) + "\n")
    shutil.rmtree(os.path.join(work, "dtds"), ignore_errors=True)


if __name__ == "__main__":
    main()
