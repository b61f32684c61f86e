"""Decode a numeric synthetic table back to the user's value space.

Behavioural parity with ``Transform.inverse`` (`Server/dtds/data/utils/transform.py:10-69`):

1. categorical columns: integer code -> string through the global vocabulary
   (``LabelEncoder.inverse_transform``, `transform.py:37-40`);
2. non-negative columns: ``v = exp(x) - 1``; when ``v < 0`` it is replaced by
   ``ceil(v)`` (so ``-0.0`` appears); a value of exactly ``-1`` becomes ``"empty"``
   (`transform.py:43-48`);
3. date parts are re-joined (`transform.py:51-52`);
4. ``"empty"`` -> ``" "`` (`transform.py:55`).

Continuous columns keep their float values (the reference does *not* round integer
columns on this path).  ``decode_frame`` is the pandas path; ``csv_columns`` prepares
the column descriptors the native CSV formatter (`csrc/host/csv_writer.cpp`) consumes.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import pandas as pd

from .constants import CATEGORICAL, EMPTY
from .date import join_dates
from .vocab import CategoryVocab


def meta_column_names(meta: dict) -> List[str]:
    return [c["column_name"] for c in meta["columns"]]


def nonneg_inverse(x: np.ndarray) -> np.ndarray:
    v = np.exp(x) - 1.0
    neg = v < 0
    v[neg] = np.ceil(v[neg])
    return v


def decode_frame(values: np.ndarray, meta: dict, vocabs: Sequence[CategoryVocab]) -> pd.DataFrame:
    names = meta_column_names(meta)
    df = pd.DataFrame(values, columns=names)
    cursor = 0
    for c in meta["columns"]:
        if c["type"] == CATEGORICAL:
            n = c["column_name"]
            df[n] = vocabs[cursor].inverse_transform(df[n].astype(int).to_numpy())
            cursor += 1
    for n in names:
        if n in meta["non_negative_cols"]:
            v = nonneg_inverse(df[n].to_numpy(dtype=np.float64).copy())
            if np.any(v == -1.0):
                col = v.astype(object)
                col[v == -1.0] = EMPTY
                df[n] = col
            else:
                df[n] = v
    if meta.get("date_info"):
        df = join_dates(df, meta["date_info"])
    return df.replace(EMPTY, " ")


# column kinds for the native formatter
KIND_FLOAT = 0      # shortest round-trip repr of a float64
KIND_VOCAB = 1      # integer code -> string from a vocabulary
KIND_NONNEG = 2     # exp(x)-1 with ceil for negatives, -1 -> " "


def csv_columns(meta: dict, vocabs: Sequence[CategoryVocab]) -> Tuple[List[str], List[int], List[List[str]]]:
    """(names, kinds, vocab strings per column) for the native formatter.

    Only valid for tables without date columns (date re-joining stays on the pandas path).
    """
    names, kinds, vocab_lists = [], [], []
    cursor = 0
    nonneg = set(meta["non_negative_cols"])
    for c in meta["columns"]:
        names.append(c["column_name"])
        if c["type"] == CATEGORICAL:
            kinds.append(KIND_VOCAB)
            strs = [(" " if s == EMPTY else s) for s in vocabs[cursor].tolist()]
            vocab_lists.append(strs)
            cursor += 1
        elif c["column_name"] in nonneg:
            kinds.append(KIND_NONNEG)
            vocab_lists.append([])
        else:
            kinds.append(KIND_FLOAT)
            vocab_lists.append([])
    return names, kinds, vocab_lists
