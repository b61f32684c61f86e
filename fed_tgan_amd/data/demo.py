"""A small encoded Intrusion-schema table: the fixture of ``__graft_entry__.smoke()``, the tests and the
probes (synthetic rows of the Intrusion schema, federated metadata of one client, a fitted VGM
transformer and the encoded training matrix)."""
from __future__ import annotations

import functools

import numpy as np

from .schema import intrusion_spec
from .synthetic import generate_intrusion
from .table import TablePreprocessor


@functools.lru_cache(maxsize=None)
def small_table(n_rows: int = 1500, seed: int = 0):
    """(spec, df, preprocessor, meta, vocabs, label-encoded rows, VGMTransformer, encoded matrix)."""
    from ..features.transformer import VGMTransformer
    from ..fed.stats import merge_categorical_metas
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
