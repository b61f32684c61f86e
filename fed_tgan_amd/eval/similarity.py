"""Statistical-similarity evaluator (Avg_JSD / Avg_WD).

Output-compatible with ``stat_sim_normalize`` (`Server/similarity_analysis.py:15-82`):

* categorical column: base-2 Jensen-Shannon *distance* between the real and synthetic
  value frequencies over the **real** categories (sorted); categories missing from the
  synthetic table contribute 0 and — a reference quirk kept for comparability — are
  appended a second time (`similarity_analysis.py:57-60`); synthetic-only categories are
  ignored;
* numeric column: Wasserstein-1 distance after a min-max scaling fitted on the real
  column (`:62-67`);
* returns ``(mean JSD over categorical columns, mean WD over numeric columns)``.

The reference also label-encodes the synthetic categoricals with encoders fitted on the
real table (`:31-37`), which raises on synthetic-only categories; here that encoding is
not needed for the metrics and is skipped, so the function never crashes on them.
"""
from __future__ import annotations

from typing import Iterable, Sequence, Tuple

import numpy as np
import pandas as pd

from ..fed.stats import jensenshannon, wasserstein_1d


def column_jsd(real: pd.Series, fake: pd.Series) -> float:
    rc = real.value_counts()
    fc = fake.value_counts()
    rp = rc / rc.sum()
    fp = fc / fc.sum() if fc.sum() else fc
    cats = sorted(rp.index.tolist())
    rv = [float(rp[c]) for c in cats]
    fv = [float(fp[c]) if c in fp.index else 0.0 for c in cats]
    missing = set(rc.index) - set(fc.index)
    for z in missing:
        rv.append(float(rp[z]))
        fv.append(0.0)
    if sum(fv) == 0:
        return 1.0
    return jensenshannon(np.asarray(rv), np.asarray(fv), base=2.0)


def column_wd(real: pd.Series, fake: pd.Series) -> float:
    r = pd.to_numeric(real, errors="coerce").to_numpy(dtype=np.float64)
    f = pd.to_numeric(fake, errors="coerce").to_numpy(dtype=np.float64)
    f = f[np.isfinite(f)]
    lo, hi = np.nanmin(r), np.nanmax(r)
    scale = (hi - lo) if hi > lo else 1.0
    return wasserstein_1d((r - lo) / scale, (f - lo) / scale)


def stat_sim(real: pd.DataFrame, fake: pd.DataFrame, cat_cols: Sequence[str]) -> Tuple[float, float]:
    cat_cols = set(cat_cols or [])
    jsd, wd = [], []
    for col in real.columns:
        if col in cat_cols:
            jsd.append(column_jsd(real[col], fake[col]))
        else:
            wd.append(column_wd(real[col], fake[col]))
    return float(np.mean(jsd)) if jsd else float("nan"), float(np.mean(wd)) if wd else float("nan")


def column_similarity(real: pd.DataFrame, fake: pd.DataFrame, cat_cols: Sequence[str]) -> pd.DataFrame:
    """Per-column table behind :func:`stat_sim`: JSD for categorical, normalised W1 for continuous."""
    cat_cols = set(cat_cols or [])
    rows = []
    for col in real.columns:
        if col in cat_cols:
            rows.append([col, "categorical", "JSD", column_jsd(real[col], fake[col])])
        else:
            rows.append([col, "continuous", "WD", column_wd(real[col], fake[col])])
    return pd.DataFrame(rows, columns=["column", "type", "metric", "value"])


def stat_sim_normalize(real_path: str, fake_path: str, cat_cols=None) -> Tuple[float, float]:
    """Path-based entry point with the reference signature."""
    return stat_sim(pd.read_csv(real_path), pd.read_csv(fake_path), cat_cols or [])


def similarity_table(real_path: str, fake_paths: Iterable[str], cat_cols, timestamp_csv: str | None = None):
    real = pd.read_csv(real_path)
    rows = []
    for i, fp in enumerate(fake_paths):
        a, b = stat_sim(real, pd.read_csv(fp), cat_cols)
        rows.append([i, a, b])
    df = pd.DataFrame(rows, columns=["Epoch_No.", "Avg_JSD", "Avg_WD"])
    if timestamp_csv is not None:
        ts = pd.read_csv(timestamp_csv, header=None)
        df["time_stamp"] = ts.iloc[:, 0].cumsum()
    return df
