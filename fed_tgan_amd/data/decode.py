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
columns on this path).  ``decode_frame`` is the pandas path; ``csv_layout`` prepares
the column descriptors the native CSV formatter (`csrc/host/csv_writer.cpp`) consumes, date columns
included (re-joined from their part codes in C++).
"""
from __future__ import annotations

import dataclasses
from typing import List, Optional, Sequence, Tuple

import numpy as np
import pandas as pd

from .constants import CATEGORICAL, EMPTY
from .date import PART_SUFFIX, join_dates, parse_format
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


# column kinds for the native formatter (csrc/host/csv_writer.h CSV_*)
KIND_FLOAT = 0      # shortest round-trip repr of a float64
KIND_VOCAB = 1      # integer code -> string from a vocabulary
KIND_NONNEG = 2     # exp(x)-1 with ceil for negatives, -1 -> " "
KIND_DATE = 3       # a date re-joined from its categorical part columns

DATE_ELEM = {"YYYY": 0, "MM": 1, "DD": 2, "hh": 3, "mm": 4, "ss": 5}


@dataclasses.dataclass
class CsvLayout:
    """Output columns of the native formatter: names, kinds, vocabularies, the source column of each
    in the decoded value matrix, and the date columns' part descriptors ([mode, n_parts, (src, elem,
    lut_off, lut_len) x n_parts] each, in output order) with their code -> value tables."""
    names: List[str]
    kinds: List[int]
    vocabs: List[List[str]]
    src: List[int]
    date_desc: List[int] = dataclasses.field(default_factory=list)
    date_lut: List[int] = dataclasses.field(default_factory=list)

    @property
    def has_dates(self) -> bool:
        return KIND_DATE in self.kinds


def _part_lut(vocab: CategoryVocab):
    out = []
    for s in vocab.tolist():
        if s == EMPTY:
            out.append(-1)
        elif str(s).isdigit():
            out.append(int(s))
        else:
            return None
    return out


def csv_layout(meta: dict, vocabs: Sequence[CategoryVocab]) -> Optional[CsvLayout]:
    """The native formatter's column layout of ``decode_frame``'s output, or None when a date column's
    format cannot be re-joined natively (its first three parts are not year, month, day in that order --
    the reference repairs the day on exactly those positions -- or a part vocabulary is not numeric)."""
    names, kinds, vocab_lists, src = [], [], [], []
    nonneg = set(meta["non_negative_cols"])
    dates = meta.get("date_info") or {}
    part_cols = {}
    for col, fmt in dates.items():
        _, d_fmt = parse_format(fmt)
        for e in d_fmt.split("-"):
            part_cols[col + PART_SUFFIX[e]] = (col, e)
    cursor = 0
    vocab_of = {}
    for j, c in enumerate(meta["columns"]):
        n = c["column_name"]
        if c["type"] == CATEGORICAL:
            vocab_of[n] = (j, vocabs[cursor])
            cursor += 1
        if n in part_cols:
            continue
        names.append(n)
        src.append(j)
        if c["type"] == CATEGORICAL:
            kinds.append(KIND_VOCAB)
            vocab_lists.append([(" " if s == EMPTY else s) for s in vocabs[cursor - 1].tolist()])
        elif n in nonneg:
            kinds.append(KIND_NONNEG)
            vocab_lists.append([])
        else:
            kinds.append(KIND_FLOAT)
            vocab_lists.append([])
    desc, lut = [], []
    for col, fmt in dates.items():
        o_fmt, d_fmt = parse_format(fmt)
        elems = d_fmt.split("-")
        if len(elems) >= 3 and elems[:3] != ["YYYY", "MM", "DD"]:
            return None
        desc += [1 if o_fmt == "yymmdd" else 0, len(elems)]
        for e in elems:
            pn = col + PART_SUFFIX[e]
            if pn not in vocab_of:
                return None
            j, voc = vocab_of[pn]
            pl = _part_lut(voc)
            if pl is None:
                return None
            desc += [j, DATE_ELEM[e], len(lut), len(pl)]
            lut += pl
        names.append(col)
        kinds.append(KIND_DATE)
        vocab_lists.append([])
        src.append(-1)
    return CsvLayout(names, kinds, vocab_lists, src, desc, lut)


def csv_columns(meta: dict, vocabs: Sequence[CategoryVocab]) -> Tuple[List[str], List[int], List[List[str]]]:
    """(names, kinds, vocab strings per column) for tables without date columns (one output column
    per value column); see :func:`csv_layout` for the general form."""
    if meta.get("date_info"):
        raise ValueError("csv_columns: the table has date columns; use csv_layout")
    lay = csv_layout(meta, vocabs)
    return lay.names, lay.kinds, lay.vocabs
