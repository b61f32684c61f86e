"""Golden fixture of the reference's unequal-client aggregation: tests/golden/unequal_agg.npz.

Made with the reference's OWN code on the CPU (`Server/dtds/distributed.py`, `Client/.../dtds/distributed.py`,
driven by the by-value RPC stand-ins of tools/reference_quality.py) on the Adult Dirichlet(0.3) split that shows
the unequal clients (11 / 20 steps per epoch, tools/wide_quality.py --spec adult --shard dirichlet):

* the federator's normalised categorical JS distances d_hat, continuous W1 distances e_hat, client row counts
  and final aggregation weights (`calculate_final_weights_for_aggregation`, `:767-783`);
* each client's generator / discriminator state dict after ONE local epoch (`train_model(1)`, `C:179-269`) --
  with the reference modules at (32, 32) hidden widths so the file stays small (the aggregation rule does not
  depend on the widths) -- including the BatchNorm running statistics after 2 x 11 and 2 x 20 updates and
  ``num_batches_tracked``;
* the federator's aggregate (`average_model`, `:86-106`) as loaded into its generator (`:811`): the float
  average cast back into the int64 ``num_batches_tracked`` buffer.

Everything is stored as plain arrays (np.load with allow_pickle=False reads it).  The test
(tests/test_stats.py::test_unequal_client_aggregate_matches_reference) runs this framework's aggregation on the
per-client states and compares.

    python tools/make_unequal_fixture.py            # ~40 s
"""
from __future__ import annotations

import copy
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from wide_quality import make_wide_split  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "unequal_agg.npz")
DIMS = (32, 32)


def main():
    work = "/tmp/fedtgan_unequal_fixture"
    spec, _, datapath = make_wide_split(work, 0, 8000, 2, spec_name="adult", shard_mode="dirichlet", alpha=0.3)
    import reference_quality  # noqa: F401  (this repo first on sys.path, before the reference)
    from adult_bisect import fresh_modules, ref_init      # (before the reference goes on sys.path)
    shim = os.path.join(work, "shim")
    os.makedirs(shim, exist_ok=True)
    with open(os.path.join(shim, "pickle5.py"), "w") as f:
        f.write("from pickle import *  # noqa\nfrom pickle import HIGHEST_PROTOCOL, dump, dumps, load, loads  # noqa\n")
    sys.dont_write_bytecode = True
    sys.path[:0] = [shim, "/root/reference/Server"]
    import torch
    torch.set_num_threads(4)
    os.chdir(work)
    for d in ("models", "Intrusion_result"):
        os.makedirs(d, exist_ok=True)
    import dtds.distributed as rdist          # (reference)
    assert rdist.__file__.startswith("/root/reference"), rdist.__file__
    cs, server = ref_init(spec, datapath, 2, seed=0)
    for c in cs:
        c.gen_dim, c.dis_dim = DIMS, DIMS
    np.random.seed(11)
    torch.manual_seed(11)
    g_dicts, d_dicts = [], []
    for c in cs:
        fresh_modules(c)
        g, d = copy.deepcopy(c.train_model(1))      # by value, as over RPC
        g_dicts.append(g)
        d_dicts.append(d)
    w = np.asarray(server.weights_con_cat_combination, dtype=np.float64)
    gen = copy.deepcopy(cs[0].generator)
    dis = copy.deepcopy(cs[0].discriminator)
    gen.load_state_dict(rdist.average_model(copy.deepcopy(g_dicts), w))
    dis.load_state_dict(rdist.average_model(copy.deepcopy(d_dicts), w))
    arrays = {
        "d_hat": np.asarray(server.distribution_similarity_vector, dtype=np.float64),
        "e_hat": np.asarray(server.distribution_similarity_vector_continuous, dtype=np.float64),
        "rows": np.asarray([c.rows for c in cs], dtype=np.int64),
        "steps": np.asarray([c.steps_per_epoch for c in cs], dtype=np.int64),
        "weights": w,
        "span_width": np.asarray([int(x[0]) for x in cs[0].out_info], dtype=np.int64),
        "span_kind": np.asarray([0 if x[1] == "tanh" else 1 for x in cs[0].out_info], dtype=np.int64),
        "dims": np.asarray(DIMS, dtype=np.int64),
    }
    for tag, dicts, agg in (("G", g_dicts, gen.state_dict()), ("D", d_dicts, dis.state_dict())):
        keys = list(agg.keys())
        arrays[f"{tag}_keys"] = np.asarray(keys)
        for k in keys:
            for i, dct in enumerate(dicts):
                arrays[f"{tag}{i}|{k}"] = dct[k].detach().cpu().numpy()
            arrays[f"{tag}agg|{k}"] = agg[k].detach().cpu().numpy()
    np.savez_compressed(OUT, **arrays)
    print(f"wrote {OUT}: steps {arrays['steps'].tolist()} weights {w.tolist()} "
          f"num_batches_tracked {[int(dct['seq.0.bn.num_batches_tracked']) for dct in g_dicts]} -> "
          f"{int(gen.state_dict()['seq.0.bn.num_batches_tracked'])}")


if __name__ == "__main__":
    main()
