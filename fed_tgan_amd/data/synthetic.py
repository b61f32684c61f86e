"""Synthetic tabular data with the schemas of the reference's benchmark tables.

There is no network and the reference's Intrusion train split is absent
(`/root/reference/.MISSING_LARGE_BLOBS`), so every benchmark here runs on synthetic rows:

* ``generate_intrusion`` — the 42-column KDD-99 "Intrusion" schema.  Rows are drawn
  class-first from a compact profile built from the shipped ``Intrusion_test.csv``
  (``tools/build_intrusion_profile.py``): class frequency, per-class categorical
  distributions and per-class 65-point quantile tables of every numeric column
  (inverse-CDF sampling, rounded to the column's precision).  Marginals and
  class-conditional marginals therefore match the real test split.
* ``generate_adult`` / ``generate_covertype`` — the UCI Adult (15 cols) and Covertype
  (55 cols) schemas from a latent-class model (no real data available; fidelity is
  schema + plausible ranges only).
* ``generate_wide`` — a wide mixed table (default 512 columns) for stress tests.

``shard`` splits a table over federated clients: ``iid``, ``dirichlet`` (label skew with
concentration ``alpha``) or ``skew`` (each client over-represents one region of a
numeric column).
"""
from __future__ import annotations

import functools
import json
import os
from typing import List, Tuple

import numpy as np
import pandas as pd

_PROFILE_DIR = os.path.join(os.path.dirname(__file__), "profiles")


@functools.lru_cache(maxsize=None)
def _intrusion_profile() -> dict:
    with open(os.path.join(_PROFILE_DIR, "intrusion.json")) as f:
        return json.load(f)


def _sample_quantiles(rng: np.random.Generator, qtab: np.ndarray, n: int) -> np.ndarray:
    u = rng.random(n) * (len(qtab) - 1)
    lo = np.floor(u).astype(np.int64)
    hi = np.minimum(lo + 1, len(qtab) - 1)
    w = u - lo
    return qtab[lo] * (1 - w) + qtab[hi] * w


def generate_intrusion(n_rows: int, seed: int = 0, class_p: np.ndarray | None = None) -> pd.DataFrame:
    prof = _intrusion_profile()
    rng = np.random.default_rng(seed)
    classes = prof["classes"]
    p = np.asarray(prof["class_p"] if class_p is None else class_p, dtype=np.float64)
    p = p / p.sum()
    labels = rng.choice(len(classes), size=n_rows, p=p)
    cols = {c: np.empty(n_rows, dtype=object) for c in prof["columns"]}
    for k, cls in enumerate(classes):
        idx = np.nonzero(labels == k)[0]
        if len(idx) == 0:
            continue
        entry = prof["per_class"][cls]
        cols[prof["target"]][idx] = cls
        for c, d in entry["cat"].items():
            pv = np.asarray(d["p"], dtype=np.float64)
            choice = rng.choice(len(pv), size=len(idx), p=pv / pv.sum())
            vals = np.asarray(d["values"], dtype=object)
            cols[c][idx] = vals[choice]
        for c, q in entry["num"].items():
            v = _sample_quantiles(rng, np.asarray(q, dtype=np.float64), len(idx))
            cols[c][idx] = np.round(v, prof["decimals"][c])
    out = {}
    for c in prof["columns"]:
        kind = prof["kinds"].get(c, "cat_str")
        if kind in ("cat_int", "int"):
            out[c] = cols[c].astype(np.float64).round().astype(np.int64)
        elif kind == "float":
            out[c] = cols[c].astype(np.float64)
        else:
            out[c] = cols[c].astype(str)
    return pd.DataFrame(out, columns=prof["columns"])


# --------------------------------------------------------------------------- Adult
ADULT_COLUMNS = ["age", "workclass", "fnlwgt", "education", "education-num", "marital-status", "occupation",
                 "relationship", "race", "gender", "capital-gain", "capital-loss", "hours-per-week",
                 "native-country", "income"]
ADULT_CATEGORICAL = ["workclass", "education", "marital-status", "occupation", "relationship", "race", "gender",
                     "native-country", "income"]
_ADULT_VOCAB = {
    "workclass": ["Private", "Self-emp-not-inc", "Local-gov", "State-gov", "Self-emp-inc", "Federal-gov", "?",
                  "Without-pay"],
    "education": ["HS-grad", "Some-college", "Bachelors", "Masters", "Assoc-voc", "11th", "Assoc-acdm", "10th",
                  "7th-8th", "Prof-school", "9th", "12th", "Doctorate", "5th-6th", "1st-4th", "Preschool"],
    "marital-status": ["Married-civ-spouse", "Never-married", "Divorced", "Separated", "Widowed",
                       "Married-spouse-absent", "Married-AF-spouse"],
    "occupation": ["Prof-specialty", "Craft-repair", "Exec-managerial", "Adm-clerical", "Sales", "Other-service",
                   "Machine-op-inspct", "?", "Transport-moving", "Handlers-cleaners", "Farming-fishing",
                   "Tech-support", "Protective-serv", "Priv-house-serv", "Armed-Forces"],
    "relationship": ["Husband", "Not-in-family", "Own-child", "Unmarried", "Wife", "Other-relative"],
    "race": ["White", "Black", "Asian-Pac-Islander", "Amer-Indian-Eskimo", "Other"],
    "gender": ["Male", "Female"],
    "native-country": ["United-States", "Mexico", "?", "Philippines", "Germany", "Canada", "Puerto-Rico", "India",
                       "El-Salvador", "Cuba", "England", "China", "Jamaica", "Italy", "South", "Japan"],
    "income": ["<=50K", ">50K"],
}


def _latent_groups(z: np.ndarray):
    """(distinct values of z, row indices of each): shared by every column drawn from the same z."""
    zs, inv = np.unique(z, return_inverse=True)
    return zs, [np.nonzero(inv == g)[0] for g in range(len(zs))]


def _latent_categorical(rng, z: np.ndarray, vocab: List[str], sharp: float, groups=None, as_category: bool = False):
    """Categorical column whose logits depend on a latent class z (Zipf base + shift)."""
    k = len(vocab)
    base = -np.log(np.arange(1, k + 1, dtype=np.float64)) * 1.2
    # the row distribution depends on z alone: one CDF per distinct z value, inverse-CDF by binary search
    # (the same draws and the same codes as thresholding an [n, k] CDF matrix row by row, at a fraction of
    # the cost: generating the 100k x 512 wide table went 26 -> 3.6 s on an 8-CPU host)
    zs, rows = groups if groups is not None else _latent_groups(z)
    shift = np.sin(np.outer(zs + 1, np.arange(k) + 1) * 0.7) * sharp
    logits = base[None, :] + shift
    pr = np.exp(logits - logits.max(1, keepdims=True))
    pr /= pr.sum(1, keepdims=True)
    cdf = pr.cumsum(1)
    u = rng.random(len(z))
    idx = np.empty(len(z), dtype=np.int64)
    for g, sel in enumerate(rows):
        idx[sel] = np.searchsorted(cdf[g], u[sel], side="right")
    idx[idx >= k] = 0          # u above the rounded CDF's last entry: argmax of an all-False row was 0
    if as_category:            # the same values as a pandas categorical: no per-row Python objects
        return pd.Categorical.from_codes(idx, categories=vocab)
    return np.asarray(vocab, dtype=object)[idx]


def generate_adult(n_rows: int, seed: int = 0) -> pd.DataFrame:
    rng = np.random.default_rng(seed)
    z = rng.choice(4, size=n_rows, p=[0.4, 0.3, 0.2, 0.1])
    d = {}
    d["age"] = np.clip(np.round(rng.normal(28 + 8 * z, 9)), 17, 90).astype(np.int64)
    d["workclass"] = _latent_categorical(rng, z, _ADULT_VOCAB["workclass"], 0.8)
    d["fnlwgt"] = np.round(np.exp(rng.normal(12.0, 0.55, n_rows))).astype(np.int64)
    d["education"] = _latent_categorical(rng, z, _ADULT_VOCAB["education"], 1.2)
    d["education-num"] = np.clip(np.round(rng.normal(9 + 1.3 * z, 2.2)), 1, 16).astype(np.int64)
    d["marital-status"] = _latent_categorical(rng, z, _ADULT_VOCAB["marital-status"], 1.0)
    d["occupation"] = _latent_categorical(rng, z, _ADULT_VOCAB["occupation"], 1.0)
    d["relationship"] = _latent_categorical(rng, z, _ADULT_VOCAB["relationship"], 1.0)
    d["race"] = _latent_categorical(rng, z, _ADULT_VOCAB["race"], 0.3)
    d["gender"] = _latent_categorical(rng, z, _ADULT_VOCAB["gender"], 0.6)
    gain = rng.random(n_rows) < 0.05 + 0.04 * z
    d["capital-gain"] = np.where(gain, np.round(np.exp(rng.normal(8.5, 1.0, n_rows))), 0).astype(np.int64)
    loss = rng.random(n_rows) < 0.03 + 0.02 * z
    d["capital-loss"] = np.where(loss, np.round(rng.normal(1900, 300, n_rows)), 0).clip(0).astype(np.int64)
    d["hours-per-week"] = np.clip(np.round(rng.normal(38 + 3 * z, 11)), 1, 99).astype(np.int64)
    d["native-country"] = _latent_categorical(rng, z, _ADULT_VOCAB["native-country"], 0.2)
    pr_hi = 1 / (1 + np.exp(-(z - 1.8) * 1.6))
    d["income"] = np.where(rng.random(n_rows) < pr_hi, ">50K", "<=50K")
    return pd.DataFrame(d, columns=ADULT_COLUMNS)


# --------------------------------------------------------------------------- Covertype
def covertype_columns() -> Tuple[List[str], List[str]]:
    cont = ["Elevation", "Aspect", "Slope", "Horizontal_Distance_To_Hydrology", "Vertical_Distance_To_Hydrology",
            "Horizontal_Distance_To_Roadways", "Hillshade_9am", "Hillshade_Noon", "Hillshade_3pm",
            "Horizontal_Distance_To_Fire_Points"]
    wild = [f"Wilderness_Area{i}" for i in range(1, 5)]
    soil = [f"Soil_Type{i}" for i in range(1, 41)]
    return cont + wild + soil + ["Cover_Type"], wild + soil + ["Cover_Type"]


def generate_covertype(n_rows: int, seed: int = 0) -> pd.DataFrame:
    rng = np.random.default_rng(seed)
    cols, _ = covertype_columns()
    cover = rng.choice(7, size=n_rows, p=[0.365, 0.488, 0.062, 0.005, 0.016, 0.03, 0.034]) + 1
    d = {}
    d["Elevation"] = np.round(rng.normal(2400 + 120 * cover, 180)).astype(np.int64)
    d["Aspect"] = np.round(rng.random(n_rows) * 360).astype(np.int64)
    d["Slope"] = np.clip(np.round(rng.gamma(3, 4.5, n_rows)), 0, 66).astype(np.int64)
    d["Horizontal_Distance_To_Hydrology"] = np.round(rng.gamma(1.5, 180, n_rows)).astype(np.int64)
    d["Vertical_Distance_To_Hydrology"] = np.round(rng.normal(46, 58, n_rows)).astype(np.int64)
    d["Horizontal_Distance_To_Roadways"] = np.round(rng.gamma(2.0, 1200, n_rows)).astype(np.int64)
    d["Hillshade_9am"] = np.clip(np.round(rng.normal(212, 27, n_rows)), 0, 254).astype(np.int64)
    d["Hillshade_Noon"] = np.clip(np.round(rng.normal(223, 20, n_rows)), 0, 254).astype(np.int64)
    d["Hillshade_3pm"] = np.clip(np.round(rng.normal(142, 38, n_rows)), 0, 254).astype(np.int64)
    d["Horizontal_Distance_To_Fire_Points"] = np.round(rng.gamma(2.0, 990, n_rows)).astype(np.int64)
    wild = (cover + rng.integers(0, 2, n_rows)) % 4
    for i in range(4):
        d[f"Wilderness_Area{i + 1}"] = (wild == i).astype(np.int64)
    soil = (cover * 5 + rng.integers(0, 8, n_rows)) % 40
    for i in range(40):
        d[f"Soil_Type{i + 1}"] = (soil == i).astype(np.int64)
    d["Cover_Type"] = cover.astype(np.int64)
    return pd.DataFrame(d, columns=cols)


# --------------------------------------------------------------------------- wide
def wide_columns(n_cols: int = 512, frac_categorical: float = 0.5) -> Tuple[List[str], List[str]]:
    n_cat = max(1, int(round(n_cols * frac_categorical)))
    n_num = n_cols - n_cat
    cols = [f"num_{i}" for i in range(n_num)] + [f"cat_{i}" for i in range(n_cat)]
    return cols, [f"cat_{i}" for i in range(n_cat)]


def generate_wide(n_rows: int, seed: int = 0, n_cols: int = 512, frac_categorical: float = 0.5,
                  as_category: bool = False) -> pd.DataFrame:
    rng = np.random.default_rng(seed)
    cols, cats = wide_columns(n_cols, frac_categorical)
    z = rng.integers(0, 6, n_rows)
    d = {}
    n_num = n_cols - len(cats)
    groups = _latent_groups(z)
    for i in range(n_num):
        n_modes = 1 + i % 4
        mode = (z + i) % n_modes
        d[f"num_{i}"] = rng.normal(mode * 3.0 + (i % 7), 0.5 + 0.25 * (i % 3), n_rows).round(4)
    for i in range(len(cats)):
        k = 2 + (i * 7) % 30
        vocab = [f"v{j}" for j in range(k)]
        d[f"cat_{i}"] = _latent_categorical(rng, z, vocab, 0.9, groups, as_category)
    return pd.DataFrame(d, columns=cols)


def generate(spec, n_rows: int, seed: int = 0, as_category: bool = False) -> pd.DataFrame:
    """``n_rows`` synthetic rows of ``spec``'s schema.  ``as_category``: string columns of the wide table
    as pandas categoricals (same values; what the federated runtime feeds its preprocessor)."""
    gen = (spec.generator or "").lower()
    if gen == "intrusion":
        return generate_intrusion(n_rows, seed)
    if gen == "adult":
        return generate_adult(n_rows, seed)
    if gen == "covertype":
        return generate_covertype(n_rows, seed)
    if gen.startswith("wide"):
        parts = gen.split(":")
        n_cols = int(parts[1]) if len(parts) > 1 else 512
        frac = float(parts[2]) if len(parts) > 2 else 0.5
        return generate_wide(n_rows, seed, n_cols, frac, as_category)
    raise ValueError(f"no synthetic generator for spec {spec.name!r} (generator={spec.generator!r})")


# --------------------------------------------------------------------------- sharding
def shard(df: pd.DataFrame, n_clients: int, mode: str = "iid", seed: int = 0, target: str | None = None,
          alpha: float = 0.5, skew_column: str | None = None) -> List[pd.DataFrame]:
    """Split ``df`` into ``n_clients`` horizontal shards."""
    rng = np.random.default_rng(seed)
    n = len(df)
    if mode == "iid":
        perm = rng.permutation(n)
        parts = np.array_split(perm, n_clients)
    elif mode == "dirichlet":
        if target is None:
            raise ValueError("dirichlet sharding needs a target column")
        labels = df[target].astype(str).to_numpy()
        parts_l: List[List[int]] = [[] for _ in range(n_clients)]
        for lab in np.unique(labels):
            idx = rng.permutation(np.nonzero(labels == lab)[0])
            props = rng.dirichlet(np.full(n_clients, alpha))
            cuts = (np.cumsum(props) * len(idx)).astype(np.int64)[:-1]
            for k, chunk in enumerate(np.split(idx, cuts)):
                parts_l[k].extend(chunk.tolist())
        parts = [np.asarray(sorted(p), dtype=np.int64) for p in parts_l]
    elif mode == "skew":
        col = skew_column or next(c for c in df.columns if df[c].dtype.kind in "if")
        order = np.argsort(df[col].to_numpy(dtype=np.float64) + rng.random(n) * 1e-9, kind="stable")
        blocks = np.array_split(order, n_clients)
        # every client keeps 70% of its block and 30% random rows
        parts = []
        pool = rng.permutation(n)
        for k, b in enumerate(blocks):
            keep = b[: int(len(b) * 0.7)]
            extra = pool[k::n_clients][: len(b) - len(keep)]
            parts.append(np.unique(np.concatenate([keep, extra])))
    else:
        raise ValueError(f"unknown shard mode {mode!r}")
    return [df.iloc[p].reset_index(drop=True) for p in parts]
