"""The reference's other table transformers (not on the Fed-TGAN path, kept for API parity).

Parity: `Server/dtds/features/transformers.py`
* :class:`DiscretizeTransformer`  — uniform KBins on continuous columns (`:82-133`)
* :class:`GeneralTransformer`     — min-max (sigmoid/tanh range) + one-hot (`:136-215`)
* :class:`GMMTransformer`         — plain 5-mode GMM, ``(x - mu) / (2 sigma)``, argmax mode (`:218-305`)
* :class:`BGMTransformer`         — the VGM transformer used by ``CTGANSynthesizer.fit`` (`:467-586`),
                                    identical math to :class:`~fed_tgan_amd.features.transformer.VGMTransformer`
* :class:`TableganTransformer`    — square "image" layout for TableGAN (`:589-626`)
* :func:`decode_train_data`       — decode + integer rounding + optional CSV dump (`:629-699`)
"""
from __future__ import annotations

import datetime
import json
import os
from typing import Sequence

import numpy as np
import pandas as pd

from ..data.constants import CATEGORICAL, CONTINUOUS, EMPTY, ORDINAL
from ..data.date import join_dates
from .transformer import SOFTMAX, VGMTransformer, metadata_from_data


class _Base:
    meta = None

    def _meta(self, data, categorical_columns, ordinal_columns):
        self.meta = metadata_from_data(data, categorical_columns, ordinal_columns)
        return self.meta


class DiscretizeTransformer(_Base):
    def __init__(self, n_bins: int):
        self.n_bins = n_bins
        self.column_index = None
        self.discretizer = None

    def fit(self, data, categorical_columns=(), ordinal_columns=()):
        from sklearn.preprocessing import KBinsDiscretizer
        self._meta(data, categorical_columns, ordinal_columns)
        self.column_index = [i for i, m in enumerate(self.meta) if m["type"] == CONTINUOUS]
        self.discretizer = KBinsDiscretizer(n_bins=self.n_bins, encode="ordinal", strategy="uniform")
        if self.column_index:
            self.discretizer.fit(np.asarray(data[:, self.column_index], dtype=np.float64))
        return self

    def transform(self, data):
        data = np.array(data, dtype=np.float64, copy=True)
        if self.column_index:
            data[:, self.column_index] = self.discretizer.transform(data[:, self.column_index])
        return data.astype("int")

    def inverse_transform(self, data):
        data = np.asarray(data).astype("float32")
        if self.column_index:
            data[:, self.column_index] = self.discretizer.inverse_transform(data[:, self.column_index])
        return data


class GeneralTransformer(_Base):
    def __init__(self, act: str = "sigmoid"):
        self.act = act
        self.output_dim = None
        self.output_info = []

    def fit(self, data, categorical_columns=(), ordinal_columns=()):
        self._meta(data, categorical_columns, ordinal_columns)
        self.output_dim = sum(1 if m["type"] in (CONTINUOUS, ORDINAL) else m["size"] for m in self.meta)
        return self

    def transform(self, data):
        cols, self.output_info = [], []
        for j, m in enumerate(self.meta):
            c = np.asarray(data[:, j])
            if m["type"] == CONTINUOUS:
                v = (c.astype(np.float64) - m["min"]) / (m["max"] - m["min"])
                if self.act == "tanh":
                    v = v * 2 - 1
                cols.append(v.reshape(-1, 1))
                self.output_info.append((1, self.act))
            elif m["type"] == ORDINAL:
                v = c.astype(np.float64) / m["size"]
                if self.act == "tanh":
                    v = v * 2 - 1
                cols.append(v.reshape(-1, 1))
                self.output_info.append((1, self.act))
            else:
                pos = {v: i for i, v in enumerate(m["i2s"])}
                oh = np.zeros((len(c), m["size"]))
                oh[np.arange(len(c)), [pos[v] for v in c]] = 1
                cols.append(oh)
                self.output_info.append((m["size"], SOFTMAX))
        return np.concatenate(cols, axis=1)

    def inverse_transform(self, data):
        out = np.zeros((len(data), len(self.meta)))
        pos = 0
        for j, m in enumerate(self.meta):
            if m["type"] in (CONTINUOUS, ORDINAL):
                v = np.asarray(data[:, pos], dtype=np.float64)
                pos += 1
                if self.act == "tanh":
                    v = (v + 1) / 2
                if m["type"] == CONTINUOUS:
                    out[:, j] = np.clip(v, 0, 1) * (m["max"] - m["min"]) + m["min"]
                else:
                    out[:, j] = np.round(v * m["size"]).clip(0, m["size"] - 1)
            else:
                k = np.asarray(data[:, pos:pos + m["size"]]).argmax(1)
                pos += m["size"]
                out[:, j] = np.asarray(m["i2s"], dtype=np.float64)[k]
        return out


class GMMTransformer(_Base):
    def __init__(self, n_clusters: int = 5):
        self.n_clusters = n_clusters
        self.model = None
        self.output_info = []
        self.output_dim = 0

    def fit(self, data, categorical_columns=(), ordinal_columns=()):
        from sklearn.mixture import GaussianMixture
        self._meta(data, categorical_columns, ordinal_columns)
        self.model, self.output_info, self.output_dim = [], [], 0
        for j, m in enumerate(self.meta):
            if m["type"] == CONTINUOUS:
                gm = GaussianMixture(self.n_clusters)
                gm.fit(np.asarray(data[:, j], dtype=np.float64).reshape(-1, 1))
                self.model.append(gm)
                self.output_info += [(1, "tanh"), (self.n_clusters, SOFTMAX)]
                self.output_dim += 1 + self.n_clusters
            else:
                self.model.append(None)
                self.output_info.append((m["size"], SOFTMAX))
                self.output_dim += m["size"]
        return self

    def transform(self, data):
        vals = []
        for j, m in enumerate(self.meta):
            c = np.asarray(data[:, j])
            if m["type"] == CONTINUOUS:
                x = c.astype(np.float64).reshape(-1, 1)
                gm = self.model[j]
                means = gm.means_.reshape(1, -1)
                stds = np.sqrt(gm.covariances_).reshape(1, -1)
                feats = (x - means) / (2 * stds)
                probs = gm.predict_proba(x)
                k = probs.argmax(1)
                vals += [np.clip(feats[np.arange(len(x)), k], -0.99, 0.99).reshape(-1, 1), probs]
            else:
                pos = {v: i for i, v in enumerate(m["i2s"])}
                oh = np.zeros((len(c), m["size"]))
                oh[np.arange(len(c)), [pos[v] for v in c]] = 1
                vals.append(oh)
        return np.concatenate(vals, axis=1)

    def inverse_transform(self, data, sigmas=None):
        out = np.zeros((len(data), len(self.meta)))
        pos = 0
        for j, m in enumerate(self.meta):
            if m["type"] == CONTINUOUS:
                u = np.asarray(data[:, pos], dtype=np.float64)
                v = np.asarray(data[:, pos + 1:pos + 1 + self.n_clusters])
                if sigmas is not None:
                    u = np.random.normal(u, sigmas[pos])
                u = np.clip(u, -1, 1)
                pos += 1 + self.n_clusters
                gm = self.model[j]
                k = v.argmax(1)
                out[:, j] = u * 2 * np.sqrt(gm.covariances_).reshape(-1)[k] + gm.means_.reshape(-1)[k]
            else:
                k = np.asarray(data[:, pos:pos + m["size"]]).argmax(1)
                pos += m["size"]
                out[:, j] = np.asarray(m["i2s"], dtype=np.float64)[k]
        return out


class BGMTransformer(VGMTransformer):
    """The VGM transformer under the name ``CTGANSynthesizer.fit`` uses (`ctgan.py:337`)."""

    def fit(self, data, categorical_columns=(), ordinal_columns=(), backend: str = "sklearn", seed=None, device=None):
        return super().fit(data, categorical_columns, ordinal_columns, backend=backend, seed=seed, device=device)


class TableganTransformer(_Base):
    def __init__(self, side: int):
        self.height = side

    def fit(self, data, categorical_columns=(), ordinal_columns=()):
        self._meta(data, categorical_columns, ordinal_columns)
        n = len(self.meta)
        self.minn, self.maxx = np.zeros(n), np.zeros(n)
        for i, m in enumerate(self.meta):
            if m["type"] == CONTINUOUS:
                self.minn[i], self.maxx[i] = m["min"] - 1e-3, m["max"] + 1e-3
            else:
                self.minn[i], self.maxx[i] = -1e-3, m["size"] - 1 + 1e-3
        return self

    def transform(self, data):
        d = np.asarray(data, dtype=np.float32).copy()
        d = (d - self.minn) / (self.maxx - self.minn) * 2 - 1
        side2 = self.height * self.height
        if side2 > d.shape[1]:
            d = np.concatenate([d, np.zeros((len(d), side2 - d.shape[1]))], axis=1)
        return d.reshape(-1, 1, self.height, self.height)

    def inverse_transform(self, data):
        d = np.asarray(data).reshape(-1, self.height * self.height)
        out = np.zeros((len(d), len(self.meta)))
        for j, m in enumerate(self.meta):
            out[:, j] = (d[:, j] + 1) / 2 * (self.maxx[j] - self.minn[j]) + self.minn[j]
            if m["type"] in (CATEGORICAL, ORDINAL):
                out[:, j] = np.round(out[:, j])
        return out


def decode_train_data(data, meta_json: str, les: Sequence[dict], model_name: str, pr=None, save: bool = True,
                      output_dir: str = "data/generated/"):
    """Decode a numeric table with the label encoders, undo log1p on non-negative columns (integer
    columns rounded), re-join dates, ``"empty"`` -> ``" "``; optionally dump a timestamped CSV."""
    with open(meta_json) as f:
        meta = json.load(f)
    int_cols = meta["integer_info"]
    nonneg = meta["non_negative_cols"]
    cat_cols = [c["column_name"] for c in meta["columns"] if c["type"] == CATEGORICAL]
    names = [c["column_name"] for c in meta["columns"]]
    df = pd.DataFrame(np.asarray(data), columns=names)
    for entry in les:
        n = entry["column_name"]
        df[n] = entry["label_encoder"].inverse_transform(df[n].astype(int))
    for n in names:
        if n in nonneg:
            v = np.exp(df[n].astype(np.float64).to_numpy()) - 1
            v = np.where(v < 0, np.ceil(v), v)
            if n in int_cols:
                col = np.where(v < 0, np.ceil(v), np.trunc(v)).astype(np.int64).astype(object)
            else:
                col = v.astype(object)
            col[v == -1] = EMPTY
            df[n] = col
    if meta.get("date_info"):
        df = join_dates(df, meta["date_info"])
    df = df.replace(EMPTY, " ")
    for n in int_cols:
        if n in df:
            if n in cat_cols:
                df[n] = df[n].apply(lambda x: int(float(x)) if x != " " else " ")
            else:
                df[n] = df[n].apply(lambda x: int(x) if x != " " else " ")
    if save:
        os.makedirs(output_dir, exist_ok=True)
        ts = str(datetime.datetime.now().timestamp()).replace(".", "")
        df.to_csv(os.path.join(output_dir, f"{model_name.split('-')[0]}_{ts}.csv"), index=False)
    return df.head(pr) if pr is not None else df
