"""Federated table statistics: vocabulary merge, client distances, aggregation weights.

Parity map (all `Server/dtds/distributed.py`):

* :func:`merge_categorical_metas` — ``uniform_meta_category`` (`:592-687`): per categorical
  column the clients' value counts are summed (dict insertion order = first appearance
  over clients in rank order), the vocabulary is sorted by global frequency (descending,
  stable), a label vocabulary is fitted, and every client gets the Jensen-Shannon
  *distance* (natural log) between the global and its own count vector; distances are
  normalised over clients per column, with ``1/K`` for all-zero columns (`:642-657`).
* :func:`continuous_client_distances` — the Wasserstein-1 part of ``uniform_continuous_gmm``
  (`:731-760`): normalised over clients, left unchanged when the sum is 0.
* :func:`aggregation_weights` — ``calculate_final_weights_for_aggregation`` (`:767-783`):
  ``S_i = sum_j e_ij + sum_j d_ij``; ``w~_i = (1 - S_i / sum_k S_k) * n_i / N``;
  ``w = softmax(w~)``.
* :func:`uniform_weights` — the ``average_model_ordinary`` ablation (`:111-132`).

``jensenshannon`` and ``wasserstein_1d`` are re-statements of the SciPy functions the
reference calls (tests pin them against SciPy).
"""
from __future__ import annotations

import copy
from typing import List, Sequence, Tuple

import numpy as np

from ..data.constants import CATEGORICAL
from ..data.vocab import CategoryVocab


def jensenshannon(p: np.ndarray, q: np.ndarray, base: float | None = None) -> float:
    p = np.asarray(p, dtype=np.float64)
    q = np.asarray(q, dtype=np.float64)
    p = p / p.sum()
    q = q / q.sum()
    m = 0.5 * (p + q)

    def kl(a, b):
        nz = a > 0
        return float(np.sum(a[nz] * np.log(a[nz] / b[nz])))

    js = 0.5 * (kl(p, m) + kl(q, m))
    if base is not None:
        js /= np.log(base)
    return float(np.sqrt(max(js, 0.0)))


def wasserstein_1d(u: np.ndarray, v: np.ndarray) -> float:
    """W1 distance between two empirical 1-D distributions (unit weights)."""
    u = np.sort(np.asarray(u, dtype=np.float64))
    v = np.sort(np.asarray(v, dtype=np.float64))
    allv = np.concatenate([u, v])
    allv.sort(kind="mergesort")
    deltas = np.diff(allv)
    cu = np.searchsorted(u, allv[:-1], side="right") / len(u)
    cv = np.searchsorted(v, allv[:-1], side="right") / len(v)
    return float(np.sum(np.abs(cu - cv) * deltas))


def wasserstein_1d_rows(u, v, u_sorted: bool = False):
    """Row-wise W1 on the device: ``u`` [R, N], ``v`` [R, M] torch tensors (one empirical
    distribution per row, unit weights) -> [R] float64.  The same CDF-difference integral as
    :func:`wasserstein_1d`, batched over rows (sort + merged grid + two ``searchsorted``)."""
    import torch
    u = u.double() if u_sorted else torch.sort(u.double(), dim=1).values
    v = torch.sort(v.double(), dim=1).values
    allv = torch.sort(torch.cat([u, v], dim=1), dim=1).values
    grid = allv[:, :-1].contiguous()
    cu = torch.searchsorted(u, grid, right=True).double() / u.shape[1]
    cv = torch.searchsorted(v, grid, right=True).double() / v.shape[1]
    return ((cu - cv).abs() * torch.diff(allv, dim=1)).sum(1)


def continuous_client_distances_device(pooled, offsets: Sequence[int]) -> np.ndarray:
    """:func:`continuous_client_distances` for a device pool: ``pooled`` [n_cont, N] holds client i's
    samples in columns ``offsets[i]:offsets[i+1]`` of every row."""
    import torch
    k = len(offsets) - 1
    if pooled.shape[0] == 0:
        return np.zeros((k, 0))
    if k == 1:      # one client: the pool IS its sample, W1 = 0 exactly (normalised: 0 as well)
        return np.zeros((1, int(pooled.shape[0])))
    us = torch.sort(pooled, dim=1).values
    e = torch.stack([wasserstein_1d_rows(us, pooled[:, offsets[i]:offsets[i + 1]], u_sorted=True)
                     for i in range(k)])
    return normalise_over_clients(e.cpu().numpy(), zero_fill_uniform=False)


def normalise_over_clients(dist: np.ndarray, zero_fill_uniform: bool) -> np.ndarray:
    """dist: [K, n_cols]. Divide each column by its sum over clients."""
    out = dist.astype(np.float64).copy()
    s = out.sum(axis=0)
    nz = s != 0
    out[:, nz] /= s[nz]
    if zero_fill_uniform:
        out[:, ~nz] = 1.0 / out.shape[0]
    return out


def merge_categorical_metas(metas: Sequence[dict]) -> Tuple[dict, List[CategoryVocab], np.ndarray]:
    """Returns (global meta with frequency-sorted ``i2s`` lists, vocabularies, d_hat [K, n_cat])."""
    k = len(metas)
    merged = copy.deepcopy(metas[0])
    vocabs: List[CategoryVocab] = []
    dists: List[np.ndarray] = []
    for j, col in enumerate(merged["columns"]):
        if col["type"] != CATEGORICAL:
            continue
        totals: dict = {}
        for m in metas:
            for key, cnt in m["columns"][j]["i2s"].items():
                totals[key] = totals.get(key, 0) + cnt
        order = sorted(totals.items(), key=lambda kv: kv[1], reverse=True)
        col["i2s"] = [kv[0] for kv in order]
        vocab = CategoryVocab(col["i2s"], col["column_name"])
        vocabs.append(vocab)
        glob = np.zeros(len(vocab))
        keys = list(totals.keys())
        glob[vocab.transform(keys)] = [totals[x] for x in keys]
        d = np.zeros(k)
        for i, m in enumerate(metas):
            local = np.zeros(len(vocab))
            ck = list(m["columns"][j]["i2s"].keys())
            if ck:
                local[vocab.transform(ck)] = [m["columns"][j]["i2s"][x] for x in ck]
            d[i] = jensenshannon(glob, local)
        dists.append(d)
    dmat = np.stack(dists, axis=1) if dists else np.zeros((k, 0))
    return merged, vocabs, normalise_over_clients(dmat, zero_fill_uniform=True)


def continuous_client_distances(pooled: Sequence[np.ndarray], per_client: Sequence[Sequence[np.ndarray]]) -> np.ndarray:
    """pooled[j]: all samples of column j; per_client[i][j]: client i's samples. -> e_hat [K, n_cont]."""
    k = len(per_client)
    n_cont = len(pooled)
    e = np.zeros((k, n_cont))
    for j in range(n_cont):
        for i in range(k):
            e[i, j] = wasserstein_1d(pooled[j], per_client[i][j])
    return normalise_over_clients(e, zero_fill_uniform=False)


def softmax(v: np.ndarray) -> np.ndarray:
    e = np.exp(v)
    return e / e.sum()


def aggregation_weights(d_hat: np.ndarray, e_hat: np.ndarray, rows: Sequence[int]) -> np.ndarray:
    rows = np.asarray(rows, dtype=np.float64)
    share = rows / rows.sum()
    s = e_hat.sum(axis=1) + d_hat.sum(axis=1)
    tot = s.sum()
    raw = (1.0 - s / tot) * share if tot != 0 else share * 0.0 + share
    return softmax(raw)


def uniform_weights(k: int) -> np.ndarray:
    return np.full(k, 1.0 / k)
