"""Conditional-vector sampler (``Cond``) and real-row sampler (``Sampler``).

Parity: ``Cond`` `Server/dtds/synthesizers/ctgan.py:85-172`, ``Sampler`` `:197-228`.

* Conditional "columns" are **all** softmax spans of ``output_info`` (continuous-mode
  indicators and categoricals), unlike upstream CTGAN (`ctgan.py:107-118`).
* training draw (``sample``): span ``col ~ U{0..n_col-1}``; option ``opt`` from
  ``log(1 + count) / sum`` over that span (`:133-137, 147-161`).
* generation draw (``sample_zero``): ``col ~ U``; option = the argmax of a uniformly
  drawn training row in that span, i.e. the empirical option frequency (`:163-172`).
* real rows: uniform among training rows whose span ``col`` has option ``opt`` hot
  (`:221-228`).

The reference builds these with Python loops over the batch and NumPy on the host, then
copies them to the device every step (`Client/.../distributed.py:190-214`).  Here the
tables are flat arrays (CDFs padded to the widest span; row lists in CSR form) that
the fused GPU sampler kernel reads directly; the host NumPy version below is the
CPU/oracle path and the statistical test reference.
"""
from __future__ import annotations

import numpy as np

from ..features.transformer import SpanLayout


class CondTables:
    """Per-span option statistics of a (possibly federated) encoded table."""

    def __init__(self, layout: SpanLayout, counts: np.ndarray):
        """counts: [n_col, max_width] one-hot column sums (padded with 0)."""
        self.layout = layout
        self.counts = np.asarray(counts, dtype=np.float64)
        w = layout.cond_width
        n_col = layout.n_col
        maxw = self.counts.shape[1] if n_col else 0
        valid = np.arange(maxw)[None, :] < w[:, None]
        logf = np.where(valid, np.log1p(self.counts), 0.0)
        self.p_log = logf / np.maximum(logf.sum(1, keepdims=True), 1e-300)
        emp = np.where(valid, self.counts, 0.0)
        self.p_emp = emp / np.maximum(emp.sum(1, keepdims=True), 1e-300)
        # CDFs padded with 1.0 beyond the span width so an inverse-CDF search stays in range
        self.cdf_log = np.where(valid, np.cumsum(self.p_log, 1), 1.0)
        self.cdf_emp = np.where(valid, np.cumsum(self.p_emp, 1), 1.0)
        self.max_width = maxw

    @staticmethod
    def span_counts(encoded: np.ndarray, layout: SpanLayout) -> np.ndarray:
        maxw = int(layout.cond_width.max()) if layout.n_col else 0
        out = np.zeros((layout.n_col, maxw))
        sums = np.asarray(encoded, dtype=np.float64).sum(0)
        for c in range(layout.n_col):
            s, w = layout.cond_start[c], layout.cond_width[c]
            out[c, :w] = sums[s:s + w]
        return out

    @classmethod
    def from_encoded(cls, encoded: np.ndarray, layout: SpanLayout) -> "CondTables":
        return cls(layout, cls.span_counts(encoded, layout))

    # ------------------------------------------------------------------ host draws
    def _draw(self, cdf: np.ndarray, batch: int, rng: np.random.Generator):
        col = rng.integers(0, self.layout.n_col, batch)
        u = rng.random(batch)
        opt = (cdf[col] > u[:, None]).argmax(1)
        opt = np.minimum(opt, self.layout.cond_width[col] - 1)
        return col, opt

    def one_hot(self, col: np.ndarray, opt: np.ndarray):
        b = len(col)
        c1 = np.zeros((b, self.layout.n_opt), dtype=np.float32)
        c1[np.arange(b), self.layout.cond_offset[col] + opt] = 1.0
        m1 = np.zeros((b, self.layout.n_col), dtype=np.float32)
        m1[np.arange(b), col] = 1.0
        return c1, m1

    def sample(self, batch: int, rng: np.random.Generator):
        """-> (c1 [B, n_opt], m1 [B, n_col], col, opt); None if there is no softmax span."""
        if self.layout.n_col == 0:
            return None
        col, opt = self._draw(self.cdf_log, batch, rng)
        c1, m1 = self.one_hot(col, opt)
        return c1, m1, col, opt

    def sample_zero(self, batch: int, rng: np.random.Generator):
        if self.layout.n_col == 0:
            return None
        col, opt = self._draw(self.cdf_emp, batch, rng)
        return self.one_hot(col, opt)[0]


class RowIndex:
    """CSR lists of training rows per (span, option)."""

    def __init__(self, encoded: np.ndarray, layout: SpanLayout):
        n = len(encoded)
        self.n_rows = n
        self.layout = layout
        maxw = int(layout.cond_width.max()) if layout.n_col else 0
        self.offset = np.zeros((layout.n_col, maxw), dtype=np.int64)
        self.count = np.zeros((layout.n_col, maxw), dtype=np.int64)
        perms = []
        base = 0
        for c in range(layout.n_col):
            s, w = layout.cond_start[c], layout.cond_width[c]
            opt = np.asarray(encoded[:, s:s + w]).argmax(1)
            order = np.argsort(opt, kind="stable")
            cnt = np.bincount(opt, minlength=w)
            self.count[c, :w] = cnt
            self.offset[c, :w] = base + np.concatenate([[0], np.cumsum(cnt)[:-1]])
            perms.append(order)
            base += n
        self.rows = np.concatenate(perms).astype(np.int64) if perms else np.zeros(0, np.int64)

    def sample_rows(self, col, opt, rng: np.random.Generator) -> np.ndarray:
        if col is None:
            return rng.integers(0, self.n_rows, len(opt))
        cnt = self.count[col, opt]
        pick = np.floor(rng.random(len(col)) * np.maximum(cnt, 1)).astype(np.int64)
        return self.rows[self.offset[col, opt] + np.minimum(pick, np.maximum(cnt - 1, 0))]

    def sample_uniform(self, n: int, rng: np.random.Generator) -> np.ndarray:
        return rng.integers(0, self.n_rows, n)
