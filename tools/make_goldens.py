"""Generate the golden parity fixtures in ``tests/golden/`` by running the REFERENCE code offline.

This is the oracle of SURVEY §4.1: the reference's math modules (server copy) are imported with a
one-line ``pickle5`` shim from a scratch directory and driven on the shipped Intrusion test split
(``data/raw/Intrusion_test.csv``, vendored from `Server/data/raw/Intrusion_test.csv`).  The RPC
layer cannot run on torch 2.10, so the federator (``MDGANServer``) is driven through in-process
stand-ins for the RRef API that call the reference ``MDGANClient`` methods directly.

Outputs are plain JSON / NPZ / CSV (no pickles).  The tests never import the reference; they only
read these files.  Run once (CPU, ~1-2 min):

    python tools/make_goldens.py [--reference /root/reference/Server]

What is pinned (reference file:line -> golden):
  * FileGenerator meta of the full split          file_generator.py:191-231    meta_full.json
  * 2-client split (rows [0,5000) / [5000,N)):
      merged vocab, JSD distances d_hat            distributed.py:592-687        fed_two_clients.json
      client VGMs -> pooled samples, W1 e_hat,
      global VGM, final softmax weights            distributed.py:689-783        fed_two_clients.json,
                                                                                 fed_gmm_samples.npz, global_bgm.npz
  * VGM encode posterior / decode given the
    global VGM; reference-encoded client-0 rows    transformers.py:385-464       vgm_codec.npz
  * Transform.inverse + to_csv bytes               transform.py:10-69            transform_inverse.csv
  * cond_loss / slerp / GP (dropout off) /
    G (train BN) and D forward on fixed tensors    ctgan.py:15-64, 174-258       model_ops.npz
  * stat_sim_normalize on a fixed CSV pair         similarity_analysis.py:15-82  evaluators.json
  * real_res (4 classifiers) on a fixed split      utility_analysis.py:15-91     evaluators.json
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "golden")
DATA = os.path.join(ROOT, "data", "raw", "Intrusion_test.csv")
SPLIT = 5000

SELECTED = ['duration', 'protocol_type', 'service', 'flag', 'src_bytes', 'dst_bytes', 'land', 'wrong_fragment',
            'urgent', 'hot', 'num_failed_logins', 'logged_in', 'num_compromised', 'root_shell', 'su_attempted',
            'num_root', 'num_file_creations', 'num_shells', 'num_access_files', 'num_outbound_cmds', 'is_host_login',
            'is_guest_login', 'count', 'srv_count', 'serror_rate', 'srv_serror_rate', 'rerror_rate',
            'srv_rerror_rate', 'same_srv_rate', 'diff_srv_rate', 'srv_diff_host_rate', 'dst_host_count',
            'dst_host_srv_count', 'dst_host_same_srv_rate', 'dst_host_diff_srv_rate', 'dst_host_same_src_port_rate',
            'dst_host_srv_diff_host_rate', 'dst_host_serror_rate', 'dst_host_srv_serror_rate',
            'dst_host_rerror_rate', 'dst_host_srv_rerror_rate', 'class']
CATEGORICAL = ['protocol_type', 'service', 'flag', 'land', 'wrong_fragment', 'urgent', 'hot', 'num_failed_logins',
               'logged_in', 'num_compromised', 'root_shell', 'su_attempted', 'num_root', 'num_file_creations',
               'num_shells', 'num_access_files', 'num_outbound_cmds', 'is_host_login', 'is_guest_login', 'class']
NONNEG = ['dst_bytes', 'src_bytes']
TARGET, PROBLEM = "class", "binary_classification"


def _jsonable(o):
    if isinstance(o, dict):
        return {str(k): _jsonable(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return [_jsonable(v) for v in o]
    if isinstance(o, np.ndarray):
        return _jsonable(o.tolist())
    if isinstance(o, np.integer):
        return int(o)
    if isinstance(o, np.floating):
        return float(o)
    if isinstance(o, np.bool_):
        return bool(o)
    return o


# ------------------------------------------------------------------ RRef stand-ins
class _Fut:
    def __init__(self, v):
        self.v = v

    def to_here(self):
        return self.v


class _Remote:
    def __init__(self, obj):
        self.obj = obj

    def __getattr__(self, name):
        f = getattr(self.obj, name)
        return lambda *a, **k: _Fut(f(*a, **k))


class FakeRRef:
    def __init__(self, obj):
        self.obj = obj

    def remote(self):
        return _Remote(self.obj)

    def rpc_sync(self):
        return self.obj


def _bgm_params(models, comps):
    keep = [(m, c) for m, c in zip(models, comps) if m is not None]
    st = lambda f: np.stack([f(m) for m, _ in keep])  # noqa: E731
    return {"wc_a": st(lambda m: m.weight_concentration_[0]), "wc_b": st(lambda m: m.weight_concentration_[1]),
            "mean_precision": st(lambda m: m.mean_precision_), "means": st(lambda m: m.means_.reshape(-1)),
            "dof": st(lambda m: m.degrees_of_freedom_), "covariances": st(lambda m: m.covariances_.reshape(-1)),
            "weights": st(lambda m: m.weights_), "components": np.stack([np.asarray(c, bool) for _, c in keep])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference/Server")
    ap.add_argument("--work", default="/tmp/fedtgan_golden")
    args = ap.parse_args()
    work = args.work
    shutil.rmtree(work, ignore_errors=True)
    shim = os.path.join(work, "shim")
    os.makedirs(shim)
    with open(os.path.join(shim, "pickle5.py"), "w") as f:
        f.write("from pickle import *  # noqa\nfrom pickle import HIGHEST_PROTOCOL, dump, dumps, load, loads  # noqa\n")
    sys.dont_write_bytecode = True
    sys.path[:0] = [shim, args.reference]
    os.chdir(work)
    for d in ("models", "Intrusion_result", "data"):
        os.makedirs(d)
    os.makedirs(OUT, exist_ok=True)

    import pandas as pd
    import torch

    np.random.seed(0)
    torch.manual_seed(0)
    import dtds.distributed as rdist                         # noqa: E402  (reference)
    import dtds.synthesizers.ctgan as rctgan                 # noqa: E402
    from dtds.data.load import prepare_data                  # noqa: E402
    from dtds.data.utils.transform import Transform          # noqa: E402

    df = pd.read_csv(DATA)
    paths = []
    for i, part in enumerate((df.iloc[:SPLIT], df.iloc[SPLIT:])):
        p = os.path.join(work, "data", f"client{i}.csv")
        part.to_csv(p, index=False)
        paths.append(p)

    # ---- FileGenerator meta of the whole split
    meta_full = prepare_data(DATA, list(SELECTED), list(CATEGORICAL), list(NONNEG), {}, TARGET, PROBLEM)
    with open(os.path.join(OUT, "meta_full.json"), "w") as f:
        json.dump(_jsonable(meta_full), f, indent=1)   # key order kept: i2s follows value_counts order

    # ---- federated initialisation over two in-process clients
    np.random.seed(1)
    clients = [rdist.MDGANClient(p, list(SELECTED), list(CATEGORICAL), list(NONNEG), {}, TARGET, PROBLEM, 1)
               for p in paths]
    client_metas = [_jsonable(c.get_meta()) for c in clients]
    server = rdist.MDGANServer([FakeRRef(c) for c in clients], 1)
    server.uniform_meta_category()
    captured = []
    real_wd = rdist.wasserstein_distance

    def wd_capture(u, v):
        captured.append((np.asarray(u, dtype=np.float64).copy(), np.asarray(v, dtype=np.float64).copy()))
        return real_wd(u, v)

    rdist.wasserstein_distance = wd_capture
    np.random.seed(2)
    server.uniform_continuous_gmm()
    rdist.wasserstein_distance = real_wd
    server.calculate_final_weights_for_aggregation()
    np.random.seed(3)
    server.refit_local_transformer()
    with open(os.path.join(work, "models", "Intrusion.json")) as f:
        merged = json.load(f)
    le_classes = {d["column_name"]: [str(x) for x in d["label_encoder"].classes_] for d in server.label_encoder}
    fed = {"split": SPLIT, "client_metas": client_metas, "merged_meta": merged, "le_classes": le_classes,
           "d_hat": np.asarray(server.distribution_similarity_vector),
           "e_hat": np.asarray(server.distribution_similarity_vector_continuous),
           "rows": [int(c.rows) for c in clients], "share": server.model_weights_by_number,
           "weights": np.asarray(server.weights_con_cat_combination)}
    with open(os.path.join(OUT, "fed_two_clients.json"), "w") as f:
        json.dump(_jsonable(fed), f, indent=1)
    # pooled / per-client GMM samples in the order the reference measured them (per column: client 0, 1)
    k = len(clients)
    n_cont = len(captured) // k
    samples = {}
    for j in range(n_cont):
        # the pooled sample is the concatenation of the clients' draws (`distributed.py:731-735`)
        assert np.array_equal(captured[j * k][0], np.concatenate([captured[j * k + i][1] for i in range(k)]))
        for i in range(k):
            samples[f"client{i}_{j}"] = captured[j * k + i][1]
    np.savez_compressed(os.path.join(OUT, "fed_gmm_samples.npz"), n_cont=n_cont, k=k, **samples)
    c0 = clients[0]
    gb = _bgm_params(c0.model, c0.components)
    np.savez_compressed(os.path.join(OUT, "global_bgm.npz"), **gb)

    # ---- VGM codec given the global VGM (client 0's refit transformer)
    tr = c0.transformer
    n_codec = 1500
    x = np.asarray(c0.train[:n_codec], dtype=np.float64)
    cont_cols = [j for j, m in enumerate(tr.meta) if m["type"] == "continuous"]
    post = np.stack([tr.model[j].predict_proba(x[:, j].reshape(-1, 1)) for j in cont_cols], axis=1)
    enc = np.asarray(c0.sampler.data[:n_codec], dtype=np.float64)      # the reference's own encode (mode sampled)
    dec = tr.inverse_transform(enc, None)
    np.savez_compressed(os.path.join(OUT, "vgm_codec.npz"), x=x, posterior=post, encoded=enc, decoded=dec,
                        cont_cols=np.asarray(cont_cols), output_dim=int(tr.output_dim))

    # ---- Transform.inverse + to_csv bytes of the decoded rows
    inv_df, _, _ = Transform.inverse(dec, os.path.join(work, "models", "Intrusion.json"), server.label_encoder)
    inv_df.to_csv(os.path.join(OUT, "transform_inverse.csv"), index=False)

    # ---- model-level math on fixed tensors
    g = torch.Generator().manual_seed(7)
    ops = {}
    out_info = [(1, "tanh"), (3, "softmax"), (1, "tanh"), (2, "softmax"), (4, "softmax")]
    n_opt = 9
    B, dim = 20, sum(w for w, _ in out_info)
    logits = torch.randn(B, dim, generator=g, dtype=torch.float64)
    col = torch.randint(0, 3, (B,), generator=g)
    opt = torch.tensor([int(torch.randint(0, w, (1,), generator=g)) for w in np.array([3, 2, 4])[col.numpy()]])
    offs = np.array([0, 3, 5])
    c = torch.zeros(B, n_opt, dtype=torch.float64)
    c[torch.arange(B), torch.as_tensor(offs)[col] + opt] = 1.0
    m = torch.zeros(B, 3, dtype=torch.float64)
    m[torch.arange(B), col] = 1.0
    ops.update(cl_logits=logits.numpy(), cl_c=c.numpy(), cl_m=m.numpy(),
               cl_loss=rctgan.cond_loss(logits, out_info, c, m).numpy())
    val = torch.rand(B, 1, generator=g, dtype=torch.float64)
    low = torch.randn(B, 30, generator=g, dtype=torch.float64)
    high = torch.randn(B, 30, generator=g, dtype=torch.float64)
    ops.update(sl_val=val.numpy(), sl_low=low.numpy(), sl_high=high.numpy(),
               sl_out=rctgan.slerp(val, low, high).numpy())
    torch.manual_seed(11)
    D = rctgan.Discriminator(12, (16, 8), pack=10).double()
    D.eval()                                            # dropout off: the penalty is deterministic
    real = torch.randn(B, 12, generator=g, dtype=torch.float64)
    # (in the reference the fake rows come from G, so the interpolates require grad)
    fake = torch.randn(B, 12, generator=g, dtype=torch.float64).requires_grad_(True)
    for n_, p_ in D.state_dict().items():
        ops[f"D_{n_}"] = p_.numpy().copy()
    torch.manual_seed(12)
    pen = rctgan.calc_gradient_penalty(D, real, fake, device="cpu", pac=10, lambda_=10)
    # calc_gradient_penalty draws alpha in fp32 (torch.rand default dtype): record the alpha it used
    torch.manual_seed(12)
    alpha32 = torch.rand(B, 1).double()
    D.zero_grad()
    yr, yf = D(real), D(fake)
    loss_d = -(torch.mean(yr) - torch.mean(yf))
    (loss_d + pen).backward()
    ops.update(gp_real=real.numpy(), gp_fake=fake.detach().numpy(), gp_alpha=alpha32.numpy(), gp_pen=pen.detach().numpy(),
               gp_loss_d=loss_d.detach().numpy(), gp_y_real=yr.detach().numpy())
    for n_, p_ in D.named_parameters():
        ops[f"Dgrad_{n_}"] = p_.grad.numpy()
    torch.manual_seed(13)
    G = rctgan.Generator(10, (16, 16), 7).double()
    G.train()
    for n_, p_ in G.state_dict().items():
        ops[f"G_{n_}"] = p_.numpy().copy()   # (state_dict tensors alias the module: copy before forward)
    gin = torch.randn(B, 10, generator=g, dtype=torch.float64)
    ops.update(g_in=gin.numpy(), g_out=G(gin).detach().numpy())
    for n_, p_ in G.state_dict().items():
        if "running" in n_:
            ops[f"Gafter_{n_}"] = p_.numpy().copy()
    np.savez_compressed(os.path.join(OUT, "model_ops.npz"), **ops)

    # ---- evaluators
    import similarity_analysis as rsim
    import utility_analysis as rutil
    real_path = paths[0]
    fake_path = os.path.join(OUT, "transform_inverse.csv")
    jsd, wd = rsim.stat_sim_normalize(real_path, fake_path, list(CATEGORICAL))
    full = pd.read_csv(DATA)
    tr_df, te_df = full.iloc[:1500].copy(), full.iloc[SPLIT:SPLIT + 1000].copy()
    fake_df = pd.read_csv(fake_path).iloc[:1500].copy()
    ru = rutil.real_res(full, tr_df, te_df, TARGET, list(CATEGORICAL))
    fu = rutil.real_res(full, fake_df, te_df, TARGET, list(CATEGORICAL))
    ev = {"stat_sim": {"real": "client0 rows [0,5000)", "fake": "transform_inverse.csv", "avg_jsd": jsd, "avg_wd": wd},
          "real_res": {"train": "rows [0,1500)", "test": f"rows [{SPLIT},{SPLIT + 1000})", "real": ru,
                       "fake_train": "transform_inverse.csv rows [0,1500)", "fake": fu}}
    with open(os.path.join(OUT, "evaluators.json"), "w") as f:
        json.dump(_jsonable(ev), f, indent=1)
    print("goldens written to", OUT)
    for fn in sorted(os.listdir(OUT)):
        print(f"  {fn}: {os.path.getsize(os.path.join(OUT, fn))} bytes")


if __name__ == "__main__":
    main()
