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


@functools.lru_cache(maxsize=None)
def wide_table(n_rows: int = 2000, n_cols: int = 96, seed: int = 0, device: str | None = None):
    """The same tuple for a reduced WIDE table (``generate_wide``): half continuous columns with 1-4
    latent modes, half categoricals of 2-31 values.  Its rows are wider than every threshold of the
    kernels only the 100k x 512 table takes by default (activation row kernels for rows > 512, chunk-split
    gradient-penalty scale for packed rows > 8,192, deep split-K discriminator GEMMs)."""
    from ..features.transformer import VGMTransformer
    from ..fed.stats import merge_categorical_metas
    from .schema import wide_spec
    from .synthetic import generate_wide
    spec = wide_spec(n_cols)
    df = generate_wide(n_rows, seed, n_cols)
    tp = TablePreprocessor(df, "Wide_train", spec.problem_type, spec.target_column, spec.categorical_list,
                           spec.nonnegative_list)
    meta, vocabs, _ = merge_categorical_metas([tp.local_meta()])
    enc = tp.encode(vocabs)
    cat = tp.categorical_indices()
    tr = VGMTransformer().fit(enc, cat, (), seed=0, backend="torch", device=device)   # (device: where the fit runs)
    tr.refit(enc, meta, vocabs, cat, (), tr.bank, tr.components)
    X = tr.transform(enc, np.random.default_rng(seed))
    return spec, df, tp, meta, vocabs, enc, tr, X
