"""VGM banks, the VGM transformer, samplers and the alternative transformers."""
import numpy as np
from sklearn.mixture import BayesianGaussianMixture

from fed_tgan_amd.features.alt_transformers import (DiscretizeTransformer, GeneralTransformer, GMMTransformer,
                                                    TableganTransformer)
from fed_tgan_amd.features.gmm import bank_from_sklearn, fit_vgm
from fed_tgan_amd.features.transformer import SpanLayout
from fed_tgan_amd.models.samplers import CondTables, RowIndex

from helpers import small_table


def _bimodal(n=3000, seed=0):
    rng = np.random.default_rng(seed)
    return np.concatenate([rng.normal(0, 1, n // 2), rng.normal(8, 0.5, n - n // 2)])


def test_bank_predict_proba_equals_sklearn():
    x = _bimodal()
    gm = BayesianGaussianMixture(n_components=10, weight_concentration_prior_type="dirichlet_process",
                                 weight_concentration_prior=0.001, n_init=1, random_state=0).fit(x.reshape(-1, 1))
    bank = bank_from_sklearn([gm])
    ours = bank.predict_proba(x.reshape(-1, 1))[:, 0, :]
    assert np.allclose(ours, gm.predict_proba(x.reshape(-1, 1)), atol=1e-9)
    assert np.allclose(bank.weights[0], gm.weights_, atol=1e-12)


def test_torch_vgm_fit_quality_matches_sklearn():
    cols = [_bimodal(4000, 1), np.random.default_rng(2).exponential(2.0, 3000)]
    sk = fit_vgm(cols, "sklearn", seed=0)
    th = fit_vgm(cols, "torch", seed=0)
    for j, x in enumerate(cols):
        def ll(b):
            lp = b.log_prob_consts()[j][None] - 0.5 * ((x[:, None] - b.means[j][None]) * b.prec_chol[j][None]) ** 2
            m = lp.max(1, keepdims=True)
            return float((m[:, 0] + np.log(np.exp(lp - m).sum(1))).mean())
        assert abs(ll(th) - ll(sk)) < 0.05
    assert th.components()[0].sum() >= 2


def test_bank_sampling_matches_mixture():
    x = _bimodal(6000, 3)
    bank = fit_vgm([x], "sklearn", seed=0)
    s = bank.sample_column(0, 20000, np.random.default_rng(0))
    assert abs(s.mean() - x.mean()) < 0.15 and abs(s.std() - x.std()) < 0.15


def test_transformer_layout_roundtrip_and_mode_stats():
    spec, df, tp, meta, vocabs, enc, tr, X = small_table()
    lay = tr.layout
    assert lay.data_dim == X.shape[1] == tr.output_dim
    assert lay.n_col == len(tp.categorical_indices()) + len(tr.cont_index)
    # one-hot spans are exactly one-hot, alpha in [-0.99, 0.99]
    for s, w, k in zip(lay.start, lay.width, lay.kind):
        if k == 1:
            assert np.all(X[:, s:s + w].sum(1) == 1)
        else:
            assert np.all(np.abs(X[:, s]) <= 0.99)
    dec = tr.inverse_transform(X)
    cat = tp.categorical_indices()
    assert np.array_equal(dec[:, cat], enc[:, cat])
    # un-clipped continuous values come back exactly
    c0 = tr.cont_index[3]
    s0 = lay.start[list(lay.kind).index(0)]
    ok = np.abs(X[:, s0]) < 0.98
    assert np.allclose(dec[ok, tr.cont_index[0]], enc[ok, tr.cont_index[0]], rtol=1e-4, atol=1e-4)
    # sampled modes follow the renormalised posterior
    probs = tr.mode_probs(enc)[:, 0, :]
    w0 = int(tr.components[0].sum())
    counts = X[:, s0 + 1:s0 + 1 + w0].mean(0)
    assert np.allclose(counts, probs[:, tr.components[0]].mean(0), atol=0.03)


def test_cond_tables_and_row_index():
    spec, df, tp, meta, vocabs, enc, tr, X = small_table()
    lay = tr.layout
    ct = CondTables.from_encoded(X, lay)
    for c in range(lay.n_col):
        s, w = lay.cond_start[c], lay.cond_width[c]
        cnt = X[:, s:s + w].sum(0)
        lp = np.log1p(cnt) / np.log1p(cnt).sum()
        assert np.allclose(ct.p_log[c, :w], lp) and np.allclose(ct.p_emp[c, :w], cnt / cnt.sum())
    rng = np.random.default_rng(0)
    c1, m1, col, opt = ct.sample(20000, rng)
    assert np.all(c1.sum(1) == 1) and np.all(m1.sum(1) == 1)
    assert abs(np.bincount(col, minlength=lay.n_col).std() / (20000 / lay.n_col)) < 0.1
    ri = RowIndex(X, lay)
    rows = ri.sample_rows(col[:500], opt[:500], rng)
    for r, c, o in zip(rows, col[:500], opt[:500]):
        assert X[r, lay.cond_start[c] + o] == 1


def test_alternative_transformers():
    spec, df, tp, meta, vocabs, enc, tr, X = small_table()
    cat = tp.categorical_indices()
    small = enc[:400]
    g = GeneralTransformer("tanh").fit(small, cat)
    t = g.transform(small)
    assert t.shape[1] == g.output_dim
    back = g.inverse_transform(t)
    assert np.array_equal(back[:, cat], small[:, cat])
    d = DiscretizeTransformer(5).fit(small, cat)
    assert d.transform(small).max() <= max(4, small[:, cat].max())
    gm = GMMTransformer(3).fit(small[:, :3], [1, 2])
    assert gm.transform(small[:, :3]).shape[1] == gm.output_dim
    tg = TableganTransformer(7).fit(small, cat)
    img = tg.transform(small)
    assert img.shape == (400, 1, 7, 7)
    assert np.array_equal(tg.inverse_transform(img)[:, cat], small[:, cat])


def test_span_layout():
    lay = SpanLayout.from_output_info([(1, "tanh"), (3, "softmax"), (5, "softmax")])
    assert lay.data_dim == 9 and lay.n_opt == 8 and lay.n_col == 2
    assert list(lay.cond_start) == [1, 4] and list(lay.cond_offset) == [0, 3]
