"""Mode-specific normalisation (VGM) transformer and the span layout the kernels consume.

Parity: ``BGM_CTGAN_Transformer`` (`Server/dtds/features/transformers.py:310-464`), the
transformer the Fed-TGAN path actually uses, including ``get_metadata`` /
``get_metadata_refit`` (`:14-71`):

* continuous column -> ``[alpha (tanh span of width 1), one-hot mode (softmax span of
  width = #valid modes)]`` where valid modes are ``weights_ > 0.005``;
  ``alpha = clip((x - mu_m) / (4 sigma_m), -0.99, 0.99)`` and the mode ``m`` is *sampled*
  from ``normalise(predict_proba[valid] + 1e-6)`` (`:391-420`);
* categorical / ordinal column -> one-hot at the position of the value in ``i2s``
  (`:423-426`); after a federated ``refit`` ``i2s`` holds global label codes ordered by
  global frequency (`:41-71, 359-375`);
* decode: ``x = clip(alpha, -1, 1) * 4 sigma_m + mu_m`` with ``m`` the argmax over valid
  modes; categorical argmax -> ``i2s`` (`:430-464`).

The reference samples modes with a per-row Python loop (`:406-410`); here encode and
decode are vectorised over rows *and* columns (numpy on the host; the GPU versions live
in :mod:`fed_tgan_amd.ops`).
"""
from __future__ import annotations

import dataclasses
from typing import List, Sequence

import numpy as np
import pandas as pd

from ..data.constants import CATEGORICAL, CONTINUOUS, ORDINAL
from .gmm import EPS_WEIGHT, N_CLUSTERS, VGMBank, fit_vgm

TANH = "tanh"
SOFTMAX = "softmax"


@dataclasses.dataclass
class SpanLayout:
    """Flat description of ``output_info`` for kernels.

    spans:  ``start[s], width[s], kind[s]`` (kind 0 = tanh, 1 = softmax) for every span.
    cond :  the softmax spans (the conditional-vector "columns" of ``Cond``, which cover
            continuous-mode indicators *and* categoricals, `ctgan.py:107-118`):
            ``cond_start[c]`` (position in the data row), ``cond_offset[c]`` (position in
            the ``n_opt`` conditional vector), ``cond_width[c]``.
    """

    start: np.ndarray
    width: np.ndarray
    kind: np.ndarray
    cond_start: np.ndarray
    cond_offset: np.ndarray
    cond_width: np.ndarray
    data_dim: int
    n_opt: int

    @property
    def n_span(self) -> int:
        return len(self.start)

    @property
    def n_col(self) -> int:
        return len(self.cond_start)

    @property
    def max_width(self) -> int:
        return int(self.width.max()) if len(self.width) else 0

    @classmethod
    def from_output_info(cls, output_info: Sequence) -> "SpanLayout":
        start, width, kind = [], [], []
        cs, co, cw = [], [], []
        pos = 0
        opt = 0
        for w, act in output_info:
            w = int(w)
            start.append(pos)
            width.append(w)
            if act == TANH:
                kind.append(0)
            elif act == SOFTMAX:
                kind.append(1)
                cs.append(pos)
                co.append(opt)
                cw.append(w)
                opt += w
            else:
                raise ValueError(f"unknown activation {act!r}")
            pos += w
        i32 = lambda v: np.asarray(v, dtype=np.int32)  # noqa: E731
        return cls(i32(start), i32(width), i32(kind), i32(cs), i32(co), i32(cw), pos, opt)


def metadata_from_data(data: np.ndarray, categorical_columns=(), ordinal_columns=()) -> List[dict]:
    """``Transformer.get_metadata`` (`transformers.py:14-40`)."""
    meta = []
    df = pd.DataFrame(data)
    for j in df.columns:
        col = df[j]
        if j in categorical_columns:
            vals = col.value_counts().index.tolist()
            meta.append({"name": j, "type": CATEGORICAL, "size": len(vals), "i2s": vals})
        elif j in ordinal_columns:
            vc = sorted(col.value_counts().items(), key=lambda kv: -kv[1])
            vals = [k for k, _ in vc]
            meta.append({"name": j, "type": ORDINAL, "size": len(vals), "i2s": vals})
        else:
            meta.append({"name": j, "type": CONTINUOUS, "min": col.min(), "max": col.max()})
    return meta


def metadata_from_global(data: np.ndarray, global_meta: dict, vocabs, categorical_columns=(), ordinal_columns=()):
    """``Transformer.get_metadata_refit`` (`transformers.py:41-71`): i2s = global codes by frequency."""
    meta = []
    if data is None:   # a dataless federator: only the schema is known
        df = pd.DataFrame(np.zeros((0, len(global_meta["columns"]))))
    else:
        df = pd.DataFrame(data)
    cursor = 0
    for j in df.columns:
        col = df[j]
        if j in categorical_columns:
            gl = global_meta["columns"][j]["i2s"]
            codes = vocabs[cursor].transform(gl).tolist()
            cursor += 1
            meta.append({"name": j, "type": CATEGORICAL, "size": len(gl), "i2s": codes})
        elif j in ordinal_columns:
            vc = sorted(col.value_counts().items(), key=lambda kv: -kv[1])
            vals = [k for k, _ in vc]
            meta.append({"name": j, "type": ORDINAL, "size": len(vals), "i2s": vals})
        else:
            meta.append({"name": j, "type": CONTINUOUS, "min": col.min() if len(col) else None,
                         "max": col.max() if len(col) else None})
    return meta


class VGMTransformer:
    """Fit / refit / transform / inverse_transform of the reference VGM transformer."""

    def __init__(self, n_clusters: int = N_CLUSTERS, eps: float = EPS_WEIGHT):
        self.n_clusters = n_clusters
        self.eps = eps
        self.meta: List[dict] | None = None
        self.bank: VGMBank | None = None
        self.components: np.ndarray | None = None   # [n_cont, K] bool
        self.cont_index: List[int] = []
        self.output_info: list = []
        self.output_dim = 0
        self.layout: SpanLayout | None = None

    # --------------------------------------------------------------------- fitting
    def _build_info(self) -> None:
        self.cont_index = [j for j, m in enumerate(self.meta) if m["type"] == CONTINUOUS]
        info = []
        c = 0
        for m in self.meta:
            if m["type"] == CONTINUOUS:
                info += [(1, TANH), (int(self.components[c].sum()), SOFTMAX)]
                c += 1
            else:
                info.append((int(m["size"]), SOFTMAX))
        self.output_info = info
        self.output_dim = int(sum(w for w, _ in info))
        self.layout = SpanLayout.from_output_info(info)
        self._code_pos = {}
        for j, m in enumerate(self.meta):
            if m["type"] != CONTINUOUS:
                self._code_pos[j] = {v: i for i, v in enumerate(m["i2s"])}

    def fit(self, data: np.ndarray, categorical_columns=(), ordinal_columns=(), backend: str = "sklearn",
            seed: int | None = None, device=None) -> "VGMTransformer":
        self.meta = metadata_from_data(data, categorical_columns, ordinal_columns)
        cont = [j for j, m in enumerate(self.meta) if m["type"] == CONTINUOUS]
        self.bank = fit_vgm([np.asarray(data[:, j], dtype=np.float64) for j in cont], backend=backend,
                            n_clusters=self.n_clusters, seed=seed, device=device)
        self.components = self.bank.components(self.eps)
        self._build_info()
        return self

    def refit(self, data: np.ndarray, global_meta: dict, vocabs, categorical_columns=(), ordinal_columns=(),
              bank: VGMBank | None = None, components: np.ndarray | None = None) -> "VGMTransformer":
        self.meta = metadata_from_global(data, global_meta, vocabs, categorical_columns, ordinal_columns)
        self.bank = bank
        self.components = np.asarray(components, dtype=bool)
        self._build_info()
        return self

    def get_information(self):
        return self.bank, self.components, self.meta

    # --------------------------------------------------------------------- persistence
    def to_dict(self) -> dict:
        """Plain-Python state (loadable with ``torch.load(..., weights_only=True)`` / JSON)."""
        def py(v):
            if isinstance(v, (list, tuple)):
                return [py(x) for x in v]
            if isinstance(v, np.generic):
                return v.item()
            return v
        meta = [{k: py(v) for k, v in m.items()} for m in self.meta]
        return {"n_clusters": self.n_clusters, "eps": self.eps, "meta": meta, "bank": self.bank.to_dict(),
                "components": np.asarray(self.components, dtype=bool).tolist()}

    @classmethod
    def from_dict(cls, d: dict) -> "VGMTransformer":
        t = cls(int(d["n_clusters"]), float(d["eps"]))
        t.meta = [dict(m) for m in d["meta"]]
        t.bank = VGMBank.from_dict(d["bank"])
        t.components = np.asarray(d["components"], dtype=bool)
        t._build_info()
        return t

    def set_model(self, bank: VGMBank, components: np.ndarray) -> None:
        self.bank = bank
        self.components = np.asarray(components, dtype=bool)
        self._build_info()

    # --------------------------------------------------------------------- encode
    def mode_probs(self, data: np.ndarray) -> np.ndarray:
        """Responsibilities over valid modes, +1e-6, renormalised: [N, n_cont, K] (invalid = 0)."""
        x = np.asarray(data[:, self.cont_index], dtype=np.float64)
        pr = self.bank.predict_proba(x) + 1e-6
        pr = pr * self.components[None]
        return pr / pr.sum(axis=2, keepdims=True)

    def transform(self, data: np.ndarray, rng: np.random.Generator | None = None) -> np.ndarray:
        rng = rng if rng is not None else np.random.default_rng()
        n = len(data)
        out = np.zeros((n, self.output_dim), dtype=np.float32)
        if self.cont_index:
            probs = self.mode_probs(data)
            u = rng.random((n, len(self.cont_index), 1))
            mode = (np.cumsum(probs, axis=2) > u).argmax(axis=2)          # index into the K components
            x = np.asarray(data[:, self.cont_index], dtype=np.float64)
            mu = np.take_along_axis(np.broadcast_to(self.bank.means[None], probs.shape), mode[:, :, None], 2)[:, :, 0]
            sd = np.take_along_axis(np.broadcast_to(self.bank.stds[None], probs.shape), mode[:, :, None], 2)[:, :, 0]
            alpha = np.clip((x - mu) / (4 * sd), -0.99, 0.99)
            # position of the mode among the valid ones
            valid_rank = np.cumsum(self.components, axis=1) - 1            # [n_cont, K]
            mpos = valid_rank[np.arange(len(self.cont_index))[None, :], mode]
        pos = 0
        c = 0
        for j, m in enumerate(self.meta):
            if m["type"] == CONTINUOUS:
                out[:, pos] = alpha[:, c]
                out[np.arange(n), pos + 1 + mpos[:, c]] = 1.0
                pos += 1 + int(self.components[c].sum())
                c += 1
            else:
                lut = self._code_pos[j]
                idx = np.fromiter((lut[v] for v in data[:, j].tolist()), dtype=np.int64, count=n) \
                    if n else np.zeros(0, np.int64)
                out[np.arange(n), pos + idx] = 1.0
                pos += int(m["size"])
        return out

    # --------------------------------------------------------------------- decode
    def inverse_transform(self, enc: np.ndarray, sigmas=None) -> np.ndarray:
        enc = np.asarray(enc)
        n = len(enc)
        out = np.zeros((n, len(self.meta)))
        pos = 0
        c = 0
        for j, m in enumerate(self.meta):
            if m["type"] == CONTINUOUS:
                nv = int(self.components[c].sum())
                u = enc[:, pos].astype(np.float64)
                if sigmas is not None:
                    u = np.random.normal(u, sigmas[pos])
                u = np.clip(u, -1, 1)
                logits = np.full((n, self.n_clusters), -100.0)
                logits[:, self.components[c]] = enc[:, pos + 1: pos + 1 + nv]
                k = logits.argmax(axis=1)
                out[:, j] = u * 4 * self.bank.stds[c][k] + self.bank.means[c][k]
                pos += 1 + nv
                c += 1
            else:
                w = int(m["size"])
                idx = enc[:, pos: pos + w].argmax(axis=1)
                out[:, j] = np.asarray(m["i2s"], dtype=np.float64)[idx] if m["type"] == CATEGORICAL else \
                    np.asarray(m["i2s"], dtype=object)[idx]
                pos += w
        return out

    # --------------------------------------------------------------------- kernel tables
    def decode_tables(self):
        """Dense tables for the GPU decode kernel: per continuous column its valid-mode means/stds
        (padded with 0) and per categorical column its i2s codes (padded)."""
        n_cont = len(self.cont_index)
        k = self.n_clusters
        mu = np.zeros((n_cont, k), dtype=np.float32)
        sd = np.ones((n_cont, k), dtype=np.float32)
        for c in range(n_cont):
            valid = np.nonzero(self.components[c])[0]
            mu[c, :len(valid)] = self.bank.means[c][valid]
            sd[c, :len(valid)] = self.bank.stds[c][valid]
        return mu, sd
