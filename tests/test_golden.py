"""Golden parity against the REFERENCE's own code.

The fixtures in ``tests/golden/`` were produced offline by ``tools/make_goldens.py``, which ran the
reference modules (`Server/dtds/...`, `Server/similarity_analysis.py`, `Server/utility_analysis.py`)
on the shipped Intrusion test split (``data/raw/Intrusion_test.csv``).  Nothing here imports the
reference; every comparison is against those stored outputs, so a misreading shared by this
package's own oracle (``models/ctgan.py``, ``ops/ref.py``) and its kernels would fail here.
"""
import json
import os

import numpy as np
import pandas as pd
import pytest
import torch

from fed_tgan_amd.data.decode import csv_columns, decode_frame
from fed_tgan_amd.data.table import TablePreprocessor
from fed_tgan_amd.features.gmm import VGMBank
from fed_tgan_amd.features.transformer import VGMTransformer
from fed_tgan_amd.fed.stats import aggregation_weights, continuous_client_distances, merge_categorical_metas

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
DATA = os.path.join(ROOT, "data", "raw", "Intrusion_test.csv")

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


def _json(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def _npz(name):
    return np.load(os.path.join(GOLD, name))     # allow_pickle=False (default): plain arrays only


def _table(frame, name="Intrusion_test"):
    return TablePreprocessor(frame[SELECTED], name, "binary_classification", "class", list(CATEGORICAL),
                             list(NONNEG), {})


def _plain(o):
    """JSON round trip: numpy scalars -> Python, dict key order kept."""
    return json.loads(json.dumps(o, default=lambda v: v.item() if hasattr(v, "item") else v))


@pytest.fixture(scope="module")
def fed():
    g = _json("fed_two_clients.json")
    df = pd.read_csv(DATA)
    parts = (df.iloc[:g["split"]].reset_index(drop=True), df.iloc[g["split"]:].reset_index(drop=True))
    tables = [_table(p, f"client{i}") for i, p in enumerate(parts)]
    metas = [t.local_meta() for t in tables]
    merged, vocabs, d_hat = merge_categorical_metas(metas)
    return g, parts, tables, metas, merged, vocabs, d_hat


def _cmp_meta(ours, gold):
    ours = _plain(ours)
    for key in ("integer_info", "non_negative_cols", "problem_type", "target", "date_info"):
        assert ours[key] == gold[key], key
    assert len(ours["columns"]) == len(gold["columns"])
    for a, b in zip(ours["columns"], gold["columns"]):
        assert a == b, (a.get("column_name"), a, b)
        if isinstance(b.get("i2s"), dict):          # value_counts order decides frequency ties later
            assert list(a["i2s"]) == list(b["i2s"]), a["column_name"]


def test_filegenerator_meta_full_split():
    """`Server/dtds/data/utils/file_generator.py:191-231` on the whole split: types ("continous"),
    min/max after log1p of the non-negative columns, value counts in value_counts order, integer
    detection."""
    _cmp_meta(_table(pd.read_csv(DATA)).local_meta(), _json("meta_full.json"))


def test_client_metas_and_merged_vocab(fed):
    """`Server/dtds/distributed.py:592-687`: per-client metas, global vocab sorted by summed frequency
    (ties in client order), LabelEncoder classes, normalised JS distances d_hat."""
    g, _, _, metas, merged, vocabs, d_hat = fed
    for ours, gold in zip(metas, g["client_metas"]):
        _cmp_meta(ours, gold)
    for a, b in zip(merged["columns"], g["merged_meta"]["columns"]):
        if b["type"] == "categorical":
            assert a["i2s"] == b["i2s"], b["column_name"]
    for v in vocabs:
        assert [str(x) for x in v.to_sklearn().classes_] == g["le_classes"][v.column_name]
    np.testing.assert_allclose(d_hat, np.asarray(g["d_hat"]), rtol=1e-10, atol=1e-12)


def test_continuous_distances_and_final_weights(fed):
    """`Server/dtds/distributed.py:731-783`: W1 of every client's GMM sample to the pooled sample,
    normalised over clients (no zero fallback), then (1 - S_i / sum S) n_i / N and softmax."""
    g = fed[0]
    s = _npz("fed_gmm_samples.npz")
    k, n_cont = int(s["k"]), int(s["n_cont"])
    per = [[s[f"client{i}_{j}"] for j in range(n_cont)] for i in range(k)]
    pooled = [np.concatenate([per[i][j] for i in range(k)]) for j in range(n_cont)]
    e_hat = continuous_client_distances(pooled, per)
    np.testing.assert_allclose(e_hat, np.asarray(g["e_hat"]), rtol=1e-9, atol=1e-12)
    w = aggregation_weights(np.asarray(g["d_hat"]), np.asarray(g["e_hat"]), g["rows"])
    np.testing.assert_allclose(w, np.asarray(g["weights"]), rtol=1e-12)
    assert g["rows"] == [len(p) for p in fed[1]]


def _global_transformer(fed):
    g, _, tables, _, merged, vocabs, _ = fed
    gb = _npz("global_bgm.npz")
    bank = VGMBank(gb["wc_a"], gb["wc_b"], gb["mean_precision"], gb["means"], gb["dof"], gb["covariances"])
    enc0 = tables[0].encode(vocabs)
    cat_idx = [j for j, c in enumerate(merged["columns"]) if c["type"] == "categorical"]
    tr = VGMTransformer().refit(enc0, merged, vocabs, cat_idx, (), bank, gb["components"])
    return tr, enc0, bank, gb


def test_vgm_weights_components_and_posterior(fed):
    """The stored sklearn posterior reproduces ``weights_`` (valid modes = weights_ > 0.005) and
    ``predict_proba`` (digamma stick-breaking + Student-t-free Gaussian terms) of the reference's
    global BayesianGaussianMixtures (`Server/dtds/features/transformers.py:334-342, 400`)."""
    tr, enc0, bank, gb = _global_transformer(fed)
    np.testing.assert_allclose(bank.weights, gb["weights"], rtol=1e-10, atol=1e-14)
    assert np.array_equal(bank.components(), gb["components"])
    v = _npz("vgm_codec.npz")
    n = len(v["x"])
    # our label-encoded client-0 rows are the reference's encoded training matrix
    np.testing.assert_allclose(enc0[:n].astype(np.float64), v["x"], rtol=0, atol=1e-9)
    post = bank.predict_proba(v["x"][:, v["cont_cols"]])
    np.testing.assert_allclose(post, v["posterior"], rtol=1e-7, atol=1e-10)


def test_vgm_encode_layout_alpha_and_mode_frequencies(fed):
    """Encode (`transformers.py:385-428`): same output width and span layout; categorical one-hots
    identical; for the mode the reference SAMPLED, alpha = clip((x - mu)/(4 sd), +-0.99) exactly; our
    sampled mode frequencies match the reference's (both draw from posterior[valid] + 1e-6)."""
    tr, enc0, bank, gb = _global_transformer(fed)
    v = _npz("vgm_codec.npz")
    ref = v["encoded"]
    n = len(ref)
    assert tr.output_dim == int(v["output_dim"]) == ref.shape[1]
    ours = tr.transform(enc0[:n], np.random.default_rng(0))
    pos = 0
    c = 0
    freq_err = []
    for j, m in enumerate(tr.meta):
        if m["type"] == "continuous":
            nv = int(gb["components"][c].sum())
            mode = ref[:, pos + 1:pos + 1 + nv].argmax(axis=1)
            valid = np.nonzero(gb["components"][c])[0]
            mu = bank.means[c][valid][mode]
            sd = np.sqrt(bank.covariances[c][valid][mode])
            alpha = np.clip((v["x"][:, j] - mu) / (4 * sd), -0.99, 0.99)
            np.testing.assert_allclose(ref[:, pos], alpha, rtol=1e-6, atol=1e-6)
            # frequencies over 1500 rows: both are draws from the same categorical per row
            f_ref = ref[:, pos + 1:pos + 1 + nv].mean(axis=0)
            f_our = ours[:, pos + 1:pos + 1 + nv].mean(axis=0)
            freq_err.append(np.abs(f_ref - f_our).max())
            pos += 1 + nv
            c += 1
        else:
            w = int(m["size"])
            np.testing.assert_array_equal(ours[:, pos:pos + w], ref[:, pos:pos + w])
            pos += w
    assert max(freq_err) < 0.06, freq_err     # 1500 rows: sd of a frequency difference <= 0.018


def test_vgm_decode_matches_reference(fed):
    """Decode (`transformers.py:430-464`): argmax over valid modes, clip(alpha, +-1) * 4 sd + mu;
    categorical argmax -> global label code."""
    tr, _, _, _ = _global_transformer(fed)
    v = _npz("vgm_codec.npz")
    dec = tr.inverse_transform(v["encoded"])
    np.testing.assert_allclose(dec, v["decoded"], rtol=1e-12, atol=1e-9)


def test_transform_inverse_csv_bytes(fed, tmp_path):
    """`Server/dtds/data/utils/transform.py:10-69` + ``to_csv(index=False)``: label decoding,
    exp(x)-1 with ceil below zero on the non-negative columns, ' ' for empties -- byte-identical,
    through the pandas path and the native C++ writer."""
    _, _, _, _, merged, vocabs, _ = fed
    v = _npz("vgm_codec.npz")
    with open(os.path.join(GOLD, "transform_inverse.csv"), "rb") as f:
        want = f.read()
    got = decode_frame(v["decoded"], merged, vocabs).to_csv(index=False).encode()
    assert got == want
    from fed_tgan_amd.utils import csvio
    if csvio.available():
        names, kinds, vocab_lists = csv_columns(merged, vocabs)
        p = tmp_path / "native.csv"
        csvio.write_table(str(p), v["decoded"], names, kinds, vocab_lists, threads=4)
        assert p.read_bytes() == want


def test_model_math_matches_reference():
    """`Server/dtds/synthesizers/ctgan.py`: cond_loss (:174-194), slerp (:231-237), gradient penalty
    with the reference's alpha and dropout off, and the D-step gradients of loss_d + pen (:240-258,
    `Client/.../distributed.py:225-231`), Generator forward with train-mode BN (:33-64)."""
    from fed_tgan_amd.models.ctgan import Discriminator, Generator, calc_gradient_penalty, cond_loss, slerp
    o = _npz("model_ops.npz")
    out_info = [(1, "tanh"), (3, "softmax"), (1, "tanh"), (2, "softmax"), (4, "softmax")]
    t = lambda k: torch.from_numpy(np.array(o[k]))  # noqa: E731
    cl = cond_loss(t("cl_logits"), out_info, t("cl_c"), t("cl_m"))
    assert abs(float(cl) - float(o["cl_loss"])) < 1e-12
    torch.testing.assert_close(slerp(t("sl_val"), t("sl_low"), t("sl_high")), t("sl_out"), rtol=1e-12, atol=1e-12)
    D = Discriminator(12, (16, 8), pack=10).double()
    D.load_state_dict({k[2:]: t(k) for k in o.files if k.startswith("D_")})
    D.eval()
    real, fake = t("gp_real"), t("gp_fake").requires_grad_(True)
    pen = calc_gradient_penalty(D, real, fake, pac=10, lambda_=10, alpha=t("gp_alpha"))
    yr, yf = D(real), D(fake)
    loss_d = -(yr.mean() - yf.mean())
    assert abs(float(pen.detach()) - float(o["gp_pen"])) < 1e-10 * max(1.0, abs(float(o["gp_pen"])))
    assert abs(float(loss_d) - float(o["gp_loss_d"])) < 1e-12
    D.zero_grad()
    (loss_d + pen).backward()
    for n, p in D.named_parameters():
        torch.testing.assert_close(p.grad, t(f"Dgrad_{n}"), rtol=1e-9, atol=1e-12)
    G = Generator(10, (16, 16), 7).double()
    G.load_state_dict({k[2:]: t(k) for k in o.files if k.startswith("G_")})
    G.train()
    torch.testing.assert_close(G(t("g_in")), t("g_out"), rtol=1e-10, atol=1e-12)
    sd = G.state_dict()
    for k in o.files:
        if k.startswith("Gafter_"):
            torch.testing.assert_close(sd[k[7:]], t(k), rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("backend", ["torch", pytest.param("hip", marks=pytest.mark.gpu)])
def test_engine_gradient_penalty_chain_matches_reference(backend):
    """The engine's own D update (explicit WGAN + hand-derived GP double backward, ``_d_update``) on
    the reference's discriminator, rows and alpha with dropout off: WGAN value, penalty and every D
    gradient of loss_d + pen.  torch: the TorchOps mirror on the CPU; hip: the HIP kernels (exact-fp32
    MFMA GEMMs) on the GPU."""
    from fed_tgan_amd.features.transformer import SpanLayout
    from fed_tgan_amd.models.ctgan import slerp
    from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig
    o = _npz("model_ops.npz")
    dev = torch.device("cuda:0" if backend == "hip" else "cpu")
    if backend == "hip":
        from fed_tgan_amd.ops import native
        native.require()
    t = lambda k: torch.from_numpy(np.array(o[k])).float().to(dev)  # noqa: E731
    lay = SpanLayout.from_output_info([(1, "tanh"), (3, "softmax"), (1, "tanh"), (2, "softmax")])  # 7 + 5 = 12
    eng = CTGANEngine(lay, EngineConfig(batch_size=20, pack=10, dis_dims=(16, 8), gen_dims=(8,), dropout_p=0.0,
                                        precision="fp32"), dev, backend=backend, seed=0)
    assert eng.Din == 12
    for i, k in enumerate(("seq.0", "seq.3")):
        eng.p[f"D.{i}.W"].copy_(t(f"D_{k}.weight"))
        eng.p[f"D.{i}.b"].copy_(t(f"D_{k}.bias"))
    eng.p["D.out.W"].copy_(t("D_seq.6.weight"))
    eng.p["D.out.b"].copy_(t("D_seq.6.bias"))
    real, fake = t("gp_real"), t("gp_fake")
    eng.X_real.copy_(real)
    eng.X_fake.copy_(fake)
    eng.X_interp.copy_(slerp(t("gp_alpha"), real, fake))
    eng.metrics.zero_()
    if not getattr(eng.ops, "adam_counts_steps", True):
        # HIP: the D-phase sampler launch bumps the Adam step counter (skipped here); at t = 0 Adam's bias
        # correction divides by zero, and the WGAN value's e-term could read D.out.b after that update
        eng.stepD.fill_(1.0)
    eng._d_update()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    wgan, pen = float(eng.metrics[0]), float(eng.metrics[1])
    assert abs(pen - float(o["gp_pen"])) < 1e-4 * max(1.0, abs(float(o["gp_pen"])))
    assert abs(wgan - float(o["gp_loss_d"])) < 1e-5
    rel = lambda a, b: float((a - b).norm() / b.norm().clamp_min(1e-12))  # noqa: E731
    for i, k in enumerate(("seq.0", "seq.3")):
        assert rel(eng.g[f"D.{i}.W"], t(f"Dgrad_{k}.weight")) < 1e-4, k
        assert rel(eng.g[f"D.{i}.b"], t(f"Dgrad_{k}.bias")) < 1e-4, k
    assert rel(eng.g["D.out.W"].view(-1), t("Dgrad_seq.6.weight").view(-1)) < 1e-4
    assert abs(float(o["Dgrad_seq.6.bias"][0])) < 1e-12      # d(loss)/d(e) = 0: the engine never updates it


def test_similarity_evaluator_matches_reference(tmp_path):
    """`Server/similarity_analysis.py:15-82` on (client-0 rows, the reference's decoded CSV)."""
    from fed_tgan_amd.eval.similarity import stat_sim_normalize
    g = _json("evaluators.json")["stat_sim"]
    real = tmp_path / "real.csv"
    pd.read_csv(DATA).iloc[:5000].to_csv(real, index=False)
    jsd, wd = stat_sim_normalize(str(real), os.path.join(GOLD, "transform_inverse.csv"), list(CATEGORICAL))
    assert abs(jsd - g["avg_jsd"]) < 1e-12 and abs(wd - g["avg_wd"]) < 1e-12


@pytest.mark.slow
def test_utility_evaluator_matches_reference():
    """`Server/utility_analysis.py:15-91`: LR / DT / RF / MLP accuracy + weighted F1 (random_state 69)."""
    from fed_tgan_amd.eval.utility import real_res
    g = _json("evaluators.json")["real_res"]
    full = pd.read_csv(DATA)
    tr, te = full.iloc[:1500].copy(), full.iloc[5000:6000].copy()
    fake = pd.read_csv(os.path.join(GOLD, "transform_inverse.csv")).iloc[:1500].copy()
    np.testing.assert_allclose(real_res(full, tr, te, "class", CATEGORICAL, verbose=False), g["real"], atol=1e-12)
    np.testing.assert_allclose(real_res(full, fake, te, "class", CATEGORICAL, verbose=False), g["fake"], atol=1e-12)
