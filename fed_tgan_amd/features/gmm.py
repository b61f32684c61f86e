"""Variational Dirichlet-process Gaussian mixtures for 1-D columns (the VGM of CTGAN).

The reference fits one ``sklearn.mixture.BayesianGaussianMixture(n_components=10,
weight_concentration_prior_type="dirichlet_process", weight_concentration_prior=0.001,
n_init=1)`` per continuous column (`Server/dtds/features/transformers.py:334-340`) and a
global one per column at the federator (`Server/dtds/distributed.py:725-745`).

``VGMBank`` stores the fitted variational posteriors of *all* continuous columns as dense
``[n_cols, K]`` arrays so that encode (`predict_proba`), sampling and decode run batched
over columns (numpy here; ``fed_tgan_amd.ops`` has the torch/HIP versions).  The
posterior predictive used for responsibilities reproduces sklearn's
``_estimate_weighted_log_prob`` for 1-D data exactly:

    log w_k  = psi(a_k) - psi(a_k+b_k) + sum_{l<k} [psi(b_l) - psi(a_l+b_l)]
    log p_k  = -0.5 log(2 pi) + log(pc_k) - 0.5 ((x-mu_k) pc_k)^2 - 0.5 log(nu_k)
               + 0.5 (log 2 + psi(nu_k / 2) - 1 / beta_k)

``fit_vgm`` dispatches to sklearn (the oracle, default) or to the batched torch VI fit in
:mod:`fed_tgan_amd.features.vgm_fit` (runs on the GPU, all columns at once).
"""
from __future__ import annotations

import dataclasses
from typing import List, Sequence

import numpy as np
from scipy.special import digamma

N_CLUSTERS = 10
EPS_WEIGHT = 0.005
WEIGHT_PRIOR = 0.001


@dataclasses.dataclass
class VGMBank:
    """Variational posteriors of ``n`` 1-D DP-GMMs with ``K`` components each."""

    wc_a: np.ndarray          # [n, K] stick-breaking Beta a (weight_concentration_[0])
    wc_b: np.ndarray          # [n, K] stick-breaking Beta b (weight_concentration_[1])
    mean_precision: np.ndarray  # [n, K] beta_k
    means: np.ndarray         # [n, K]
    dof: np.ndarray           # [n, K] nu_k
    covariances: np.ndarray   # [n, K] (1-D "full" covariance)

    @property
    def n(self) -> int:
        return self.means.shape[0]

    @property
    def k(self) -> int:
        return self.means.shape[1]

    @property
    def prec_chol(self) -> np.ndarray:
        return 1.0 / np.sqrt(self.covariances)

    @property
    def stds(self) -> np.ndarray:
        return np.sqrt(self.covariances)

    @property
    def weights(self) -> np.ndarray:
        """Expected stick-breaking weights (sklearn ``weights_``)."""
        tot = self.wc_a + self.wc_b
        frac = self.wc_b / tot
        w = self.wc_a / tot * np.concatenate([np.ones((self.n, 1)), np.cumprod(frac[:, :-1], axis=1)], axis=1)
        return w / w.sum(axis=1, keepdims=True)

    def components(self, eps: float = EPS_WEIGHT) -> np.ndarray:
        return self.weights > eps

    def column(self, j: int) -> "VGMBank":
        return VGMBank(*(getattr(self, f.name)[j:j + 1] for f in dataclasses.fields(self)))

    @staticmethod
    def concat(banks: Sequence["VGMBank"]) -> "VGMBank":
        return VGMBank(*(np.concatenate([getattr(b, f.name) for b in banks], axis=0)
                         for f in dataclasses.fields(VGMBank)))

    def to_dict(self) -> dict:
        return {f.name: getattr(self, f.name).tolist() for f in dataclasses.fields(self)}

    @classmethod
    def from_dict(cls, d: dict) -> "VGMBank":
        return cls(**{f.name: np.asarray(d[f.name], dtype=np.float64) for f in dataclasses.fields(cls)})

    # ----------------------------------------------------------------- responsibilities
    def log_weights(self) -> np.ndarray:
        dsum = digamma(self.wc_a + self.wc_b)
        da = digamma(self.wc_a)
        db = digamma(self.wc_b)
        prefix = np.concatenate([np.zeros((self.n, 1)), np.cumsum(db - dsum, axis=1)[:, :-1]], axis=1)
        return da - dsum + prefix

    def log_prob_consts(self) -> np.ndarray:
        """Per-component constant part of the weighted log prob, [n, K]."""
        pc = self.prec_chol
        return (self.log_weights() - 0.5 * np.log(2 * np.pi) + np.log(pc) - 0.5 * np.log(self.dof)
                + 0.5 * (np.log(2.0) + digamma(0.5 * self.dof) - 1.0 / self.mean_precision))

    def log_resp(self, x: np.ndarray) -> np.ndarray:
        """x: [N, n] (column j evaluated under model j) -> normalised log responsibilities [N, n, K]."""
        pc = self.prec_chol
        y = (x[:, :, None] - self.means[None]) * pc[None]
        lp = self.log_prob_consts()[None] - 0.5 * y * y
        mx = lp.max(axis=2, keepdims=True)
        return lp - (mx + np.log(np.exp(lp - mx).sum(axis=2, keepdims=True)))

    def predict_proba(self, x: np.ndarray) -> np.ndarray:
        return np.exp(self.log_resp(x))

    # ----------------------------------------------------------------- sampling
    def sample_column(self, j: int, n: int, rng: np.random.Generator) -> np.ndarray:
        """sklearn ``BayesianGaussianMixture.sample`` for one column (component counts ~ multinomial)."""
        counts = rng.multinomial(n, self.weights[j])
        out = [rng.normal(self.means[j, k], np.sqrt(self.covariances[j, k]), c) for k, c in enumerate(counts)]
        return np.concatenate(out) if out else np.zeros(0)


def sample_pool(banks: Sequence[VGMBank], n_per_client: Sequence[int], rng: np.random.Generator, device,
                seed: int):
    """Every client's VGM sampled into one pooled tensor on ``device``: [n_cont, sum(n_per_client)],
    client i's ``n_per_client[i]`` draws of column j in columns ``off[i]:off[i+1]`` of row j, grouped
    by component like ``sklearn``'s ``sample`` / :meth:`VGMBank.sample_column`.

    Component counts are multinomial draws on the host (``n_cont x K x 10`` numbers); the normals are
    drawn on the device from a generator seeded with ``seed``.  Returns (pool, offsets)."""
    import torch
    n_cont = banks[0].n
    nk = banks[0].k
    off = np.concatenate([[0], np.cumsum(n_per_client)]).astype(np.int64)
    counts = np.zeros((n_cont, len(banks), nk), dtype=np.int64)
    for j in range(n_cont):
        for i, b in enumerate(banks):
            counts[j, i] = rng.multinomial(int(n_per_client[i]), b.weights[j])
    mean = np.stack([b.means for b in banks], axis=1)                      # [n_cont, K, nk]
    std = np.sqrt(np.stack([b.covariances for b in banks], axis=1))
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if dev.type == "cuda":
        # one launch of this library's pool_sample kernel (csrc/kernels/init_ops.hip): segment (j, i, k) of the
        # row-major pool is [seg_off[s], seg_off[s + 1]) -- the flattened counts' prefix sums, as row j holds every
        # client's draws of column j back to back.  Its normals are Philox keyed on (seed, element), not torch's
        # generator (no ATen kernel on the initialisation path)
        from ..ops import native
        seg_off = np.concatenate([[0], np.cumsum(counts.reshape(-1))]).astype(np.int64)
        pool = torch.empty(n_cont, int(off[-1]), dtype=torch.float64, device=dev)
        native.require().pool_sample(pool, torch.as_tensor(seg_off, device=dev),
                                     torch.as_tensor(np.ascontiguousarray(mean.reshape(-1)), device=dev),
                                     torch.as_tensor(np.ascontiguousarray(std.reshape(-1)), device=dev),
                                     int(seed) & ((1 << 62) - 1))
        return pool, off.tolist()
    seg = torch.arange(n_cont * len(banks) * nk, device=dev)
    idx = torch.repeat_interleave(seg, torch.as_tensor(counts.reshape(-1), device=dev),
                                  output_size=int(n_cont * off[-1]))
    gen = torch.Generator(device=dev)
    gen.manual_seed(int(seed))
    z = torch.randn(int(n_cont * off[-1]), generator=gen, dtype=torch.float64, device=dev)
    m = torch.as_tensor(mean.reshape(-1), device=dev)
    sd = torch.as_tensor(std.reshape(-1), device=dev)
    pool = (m[idx] + sd[idx] * z).view(n_cont, int(off[-1]))
    return pool, off.tolist()


def bank_from_sklearn(models: Sequence) -> VGMBank:
    return VGMBank(
        wc_a=np.stack([m.weight_concentration_[0] for m in models]),
        wc_b=np.stack([m.weight_concentration_[1] for m in models]),
        mean_precision=np.stack([m.mean_precision_ for m in models]),
        means=np.stack([m.means_.reshape(-1) for m in models]),
        dof=np.stack([m.degrees_of_freedom_ for m in models]),
        covariances=np.stack([m.covariances_.reshape(-1) for m in models]),
    )


def fit_vgm_sklearn(columns: List[np.ndarray], n_clusters: int = N_CLUSTERS, seed: int | None = None) -> VGMBank:
    import warnings
    from sklearn.exceptions import ConvergenceWarning
    from sklearn.mixture import BayesianGaussianMixture
    models = []
    for x in columns:
        gm = BayesianGaussianMixture(n_components=n_clusters, weight_concentration_prior_type="dirichlet_process",
                                     weight_concentration_prior=WEIGHT_PRIOR, n_init=1, random_state=seed)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", ConvergenceWarning)
            gm.fit(np.asarray(x, dtype=np.float64).reshape(-1, 1))
        models.append(gm)
    return bank_from_sklearn(models)


def fit_vgm(columns, backend: str = "sklearn", n_clusters: int = N_CLUSTERS,
            seed: int | None = None, device=None) -> VGMBank:
    """columns: a list of 1-D samples, one per column, or (torch backend) a [n_cols, n] tensor."""
    if len(columns) == 0:
        z = np.zeros((0, n_clusters))
        return VGMBank(z, z, z, z, z, z)
    if backend == "sklearn":
        return fit_vgm_sklearn(columns, n_clusters, seed)
    if backend == "torch":
        from .vgm_fit import fit_vgm_torch
        return fit_vgm_torch(columns, n_clusters=n_clusters, seed=seed, device=device)
    raise ValueError(f"unknown VGM fit backend {backend!r}")
