"""VGM fit parity with sklearn's BayesianGaussianMixture on every Intrusion continuous column.

The reference fits ``BayesianGaussianMixture(n_components=10, weight_concentration_prior_type=
"dirichlet_process", weight_concentration_prior=0.001, n_init=1)`` per continuous column
(`Server/dtds/features/transformers.py:334-342`) and again at the federator on the pooled GMM
samples (`Server/dtds/distributed.py:725-745`); the valid modes (``weights_ > 0.005``) decide the
encoded width (``data_dim`` / ``n_opt``).

* Same initialisation: sklearn's k-means centres (``KMeans(10, n_init=1)`` with the RandomState the
  BGM itself would hand it) are passed as ``init_centers``; from there the fit is deterministic, so
  ours must reproduce sklearn's variational posterior -- weights, means, covariances, valid-mode
  count -- on all 22 columns of the shipped split (CPU torch path; the fused HIP kernel on a GPU).
* Own initialisation (k-means++ + Lloyd on the device RNG): the valid-mode count of every column
  lies within the range sklearn itself produces over seeds, and the fitted mixture's average
  log-likelihood is within 0.05 nats of sklearn's best.
"""
import os
import warnings

import numpy as np
import pandas as pd
import pytest
import torch

from fed_tgan_amd.data.table import TablePreprocessor
from fed_tgan_amd.features.gmm import VGMBank, bank_from_sklearn
from fed_tgan_amd.features.vgm_fit import fit_vgm_torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "data", "raw", "Intrusion_test.csv")
N_ROWS = 5000


@pytest.fixture(scope="module")
def columns():
    from fed_tgan_amd.data.schema import intrusion_spec
    spec = intrusion_spec()
    df = pd.read_csv(DATA).iloc[:N_ROWS]
    tp = TablePreprocessor(df[spec.selected_variables], "Intrusion_test", spec.problem_type, spec.target_column,
                           list(spec.categorical_list), list(spec.nonnegative_list), {})
    from fed_tgan_amd.fed.stats import merge_categorical_metas
    _, vocabs, _ = merge_categorical_metas([tp.local_meta()])
    enc = tp.encode(vocabs)
    cat = set(tp.categorical_indices())
    return [np.asarray(enc[:, j], dtype=np.float64) for j in range(enc.shape[1]) if j not in cat]


def _sklearn(x, seed):
    from sklearn.cluster import KMeans
    from sklearn.mixture import BayesianGaussianMixture
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        gm = BayesianGaussianMixture(n_components=10, weight_concentration_prior_type="dirichlet_process",
                                     weight_concentration_prior=0.001, n_init=1, random_state=seed)
        gm.fit(x.reshape(-1, 1))
        km = KMeans(n_clusters=10, n_init=1, random_state=np.random.RandomState(seed)).fit(x.reshape(-1, 1))
    return gm, km.cluster_centers_.reshape(-1)


@pytest.fixture(scope="module")
def sk(columns):
    return [_sklearn(x, 0) for x in columns]


def _check_same_init(bank: VGMBank, sk, tag):
    ref = bank_from_sklearn([g for g, _ in sk])
    bad = []
    for j, (g, _) in enumerate(sk):
        if not np.array_equal(bank.components()[j], g.weights_ > 0.005):
            bad.append((j, "components"))
            continue
        ok = (np.allclose(bank.weights[j], g.weights_, rtol=1e-5, atol=1e-8)
              and np.allclose(bank.means[j], ref.means[j], rtol=1e-5, atol=1e-6 * (1 + np.abs(ref.means[j]).max()))
              and np.allclose(bank.covariances[j], ref.covariances[j], rtol=1e-4, atol=1e-9))
        if not ok:
            bad.append((j, "params"))
    assert not bad, (tag, bad)


def test_same_init_matches_sklearn_cpu(columns, sk):
    bank = fit_vgm_torch(columns, seed=0, device="cpu", init_centers=np.stack([c for _, c in sk]))
    _check_same_init(bank, sk, "torch")


@pytest.mark.gpu
def test_same_init_matches_sklearn_fused_kernel(columns, sk):
    from fed_tgan_amd.ops import native
    native.require()
    bank = fit_vgm_torch(columns, seed=0, device="cuda:0", init_centers=np.stack([c for _, c in sk]))
    _check_same_init(bank, sk, "hip")


def _avg_loglik(bank: VGMBank, j: int, x: np.ndarray) -> float:
    w = bank.weights[j]
    sd = np.sqrt(bank.covariances[j])
    lp = np.log(np.maximum(w, 1e-300))[None] - 0.5 * np.log(2 * np.pi) - np.log(sd)[None] \
        - 0.5 * ((x[:, None] - bank.means[j][None]) / sd[None]) ** 2
    m = lp.max(1, keepdims=True)
    return float(np.mean(m[:, 0] + np.log(np.exp(lp - m).sum(1))))


def _own_init_checks(bank: VGMBank, columns, seeds=(0, 1, 2, 3)):
    sks = [[_sklearn(x, s)[0] for s in seeds] for x in columns]
    for j, x in enumerate(columns):
        counts = [int((g.weights_ > 0.005).sum()) for g in sks[j]]
        ours = int(bank.components()[j].sum())
        assert min(counts) - 1 <= ours <= max(counts) + 1, (j, ours, counts)
        best = max(_avg_loglik(bank_from_sklearn([g]), 0, x) for g in sks[j])
        assert _avg_loglik(bank, j, x) >= best - 0.05 * (1 + abs(best)), (j, _avg_loglik(bank, j, x), best)


@pytest.mark.slow
def test_own_init_statistically_equivalent_cpu(columns):
    _own_init_checks(fit_vgm_torch(columns, seed=3, device="cpu"), columns)


@pytest.mark.gpu
def test_own_init_statistically_equivalent_fused_kernel(columns):
    from fed_tgan_amd.ops import native
    native.require()
    _own_init_checks(fit_vgm_torch(columns, seed=3, device="cuda:0"), columns)
    info = fit_vgm_torch.last_info
    assert (info[:, 0] >= 1).all() and (info[:, 0] <= 100).all()


@pytest.mark.gpu
@pytest.mark.parametrize("split", [4, 11])
def test_split_fit_matches_sklearn_and_is_deterministic(columns, sk, split):
    """set_tuning("vgm_split"): a cluster of workgroups per column (E-step rows split, the partial records summed in
    workgroup order behind a per-column arrival counter) still reproduces sklearn from the same initialisation,
    every barrier completes, and two fits give the same bits."""
    from fed_tgan_amd.ops import native
    native.require()
    prev = torch.ops.fedtgan.set_tuning("vgm_split", split)
    try:
        assert torch.ops.fedtgan.set_tuning("vgm_split_of", len(columns)) == split
        ic = np.stack([c for _, c in sk])
        a = fit_vgm_torch(columns, seed=0, device="cuda:0", init_centers=ic)
        info = fit_vgm_torch.last_info.copy()
        b = fit_vgm_torch(columns, seed=0, device="cuda:0", init_centers=ic)
    finally:
        torch.ops.fedtgan.set_tuning("vgm_split", prev)
    assert (info[:, 1] >= 0).all(), info          # -1: a cluster barrier timed out
    for f in ("means", "covariances", "weights"):
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f))
    _check_same_init(a, sk, f"hip split {split}")
