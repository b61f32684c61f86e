"""Date columns <-> categorical date-part columns.

Behavioural parity with `Server/dtds/data/utils/date.py:6-200`:

* a date column ``c`` with format spec ``"[o_format|]d_format"`` (``d_format`` like
  ``"YYYY-MM-DD"``) is parsed (``o_format == "yymmdd"`` means the raw cells are integers
  such as ``930101``) and replaced by categorical columns ``c-year``, ``c-month``,
  ``c-day``, ``c-hour``, ``c-minute``, ``c-second`` (years as two digits, like the
  reference's ``strftime('%y')``); missing cells stay ``"empty"``;
* the inverse joins the parts with ``-``, repairs impossible days (Feb -> 28/29 with the
  reference's leap rule, other months -> 30) and re-parses.

Deviations (documented): the caller's categorical list is returned, not mutated
(`date.py:28,113` mutate it in place), and the inverse drops the part columns of *every*
date column (`date.py:199` only drops the last one's).
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import pandas as pd

from .constants import EMPTY

PART_SUFFIX = {"YYYY": "-year", "MM": "-month", "DD": "-day", "hh": "-hour", "mm": "-minute", "ss": "-second"}
PART_STRFTIME = {"YYYY": "%y", "MM": "%m", "DD": "%d", "hh": "%H", "mm": "%M", "ss": "%S"}
DAYS_IN_MONTH = {1: 31, 2: 28, 3: 31, 4: 30, 5: 31, 6: 30, 7: 31, 8: 31, 9: 30, 10: 31, 11: 30, 12: 31}


def parse_format(spec: str) -> Tuple[str | None, str]:
    parts = spec.split("|")
    if len(parts) == 2:
        return parts[0], parts[1]
    return None, parts[0]


def split_dates(df: pd.DataFrame, date_columns: Dict[str, str], categorical: List[str]) -> Tuple[pd.DataFrame, List[str]]:
    """Replace every date column by its categorical parts. Returns (frame, categorical list)."""
    categorical = [c for c in categorical if c not in date_columns]
    df = df.copy()
    for col, spec in date_columns.items():
        o_fmt, d_fmt = parse_format(spec)
        raw = df[col]
        present = raw != EMPTY
        if o_fmt == "yymmdd":
            parsed = pd.to_datetime(raw[present].map(lambda v: str(int(float(v)))))
        else:
            parsed = pd.to_datetime(raw[present].astype(str))
        for elem in d_fmt.split("-"):
            name = col + PART_SUFFIX[elem]
            out = pd.Series(EMPTY, index=df.index, dtype=object)
            out[present] = parsed.dt.strftime(PART_STRFTIME[elem])
            df[name] = out
            categorical.append(name)
        df = df.drop(columns=[col])
    return df, categorical


def _repair_day(y: str, m: str, d: str) -> str:
    mi, di = int(m), int(d)
    if di > DAYS_IN_MONTH[mi]:
        if m == "02":
            yi = int(y)
            d = "29" if (yi % 4 == 0 and yi % 100 == 0 and yi % 400 == 0) else "28"
        else:
            d = "30"
    return d


def join_dates(df: pd.DataFrame, date_columns: Dict[str, str]) -> pd.DataFrame:
    """Inverse of :func:`split_dates` on a decoded frame."""
    df = df.copy()
    for col, spec in date_columns.items():
        o_fmt, d_fmt = parse_format(spec)
        elems = d_fmt.split("-")
        names = [col + PART_SUFFIX[e] for e in elems]
        joined = df[names].astype(str).agg("-".join, axis=1)
        fmt = "-".join(PART_STRFTIME[e] for e in elems)

        def rebuild(s: str):
            if EMPTY in s:
                return EMPTY
            p = s.split("-")
            if len(p) >= 3:
                p[2] = _repair_day(p[0], p[1], p[2])
            # explicit format: the reference's bare to_datetime reads "20-01-31" as 2031-01-20
            ts = pd.to_datetime("-".join(p), format=fmt)
            if o_fmt == "yymmdd":
                return int(ts.strftime("%y%m%d"))
            return ts

        df[col] = joined.map(rebuild)
        df = df.drop(columns=names)
    return df
