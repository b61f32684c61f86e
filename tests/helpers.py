"""Shared fixtures: a small encoded Intrusion-schema table and an autograd oracle of one step."""
from __future__ import annotations

import functools

import numpy as np
import torch
import torch.nn.functional as F

from fed_tgan_amd.data.schema import intrusion_spec
from fed_tgan_amd.data.synthetic import generate_intrusion
from fed_tgan_amd.data.table import TablePreprocessor
from fed_tgan_amd.features.transformer import VGMTransformer
from fed_tgan_amd.fed.stats import merge_categorical_metas


@functools.lru_cache(maxsize=None)
def small_table(n_rows: int = 1500, seed: int = 0):
    spec = intrusion_spec()
    df = generate_intrusion(n_rows, seed)
    tp = TablePreprocessor(df, "Intrusion_train", spec.problem_type, spec.target_column, spec.categorical_list,
                           spec.nonnegative_list)
    meta, vocabs, _ = merge_categorical_metas([tp.local_meta()])
    enc = tp.encode(vocabs)
    cat = tp.categorical_indices()
    tr = VGMTransformer().fit(enc, cat, (), seed=0, backend="sklearn" if n_rows <= 5000 else "torch")
    tr.refit(enc, meta, vocabs, cat, (), tr.bank, tr.components)
    X = tr.transform(enc, np.random.default_rng(seed))
    return spec, df, tp, meta, vocabs, enc, tr, X


def d_forward_masked(X, Ws, bs, masks, v, e, slope=0.2):
    """Packed D forward with explicit dropout keep-masks (values 0 / 2)."""
    h = X
    for W, b, M in zip(Ws, bs, masks):
        h = F.leaky_relu(h @ W.t() + b, slope) * M
    return h @ v.view(-1, 1) + e


def keep_mask_from_ms(ms, pre, slope=0.2):
    s = torch.where(pre > 0, torch.ones_like(pre), torch.full_like(pre, slope))
    return ms / s
