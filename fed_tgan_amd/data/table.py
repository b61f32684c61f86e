"""Local table preprocessing, meta generation and label encoding.

Behavioural parity with the reference ``FileGenerator`` (`Server/dtds/data/utils/
file_generator.py:59-265`) and ``prepare_data`` / ``encode_data_with_meta_labelencoder``
(`Server/dtds/data/load.py:51-90`):

* integer columns are detected on the raw frame (int dtype, or float whose non-null
  values are whole numbers) (`file_generator.py:104-110`);
* blank cells become NaN then the literal ``"empty"`` (`:115-116`);
* every non-categorical, non-date column listed as non-negative is mapped by
  ``log(x + 1)`` (`:118-126`);
* date columns are split into categorical parts (`:129-133`, see :mod:`.date`);
* ``local_meta()`` returns the reference meta dict, with per-category value counts in
  ``i2s`` (`:191-231`), the ``"continous"`` spelling and ``"column no"``;
* ``encode(vocabs)`` label-encodes categoricals with the *global* vocabularies
  (``astype(str)`` first, `:163-167`) and returns the numeric training matrix.

The reference round-trips the encoded matrix through ``dtds/saved_models/.../*.npz`` on
disk before reading it back (`load.py:38-48, 72-90`); we keep that artefact optional
(``write_artifacts``) and hand the matrix over in memory.
"""
from __future__ import annotations

import datetime
import json
import os
from typing import Dict, List, Optional, Sequence

import numpy as np
import pandas as pd

from .constants import CATEGORICAL, EMPTY, META_CONTINUOUS
from .date import split_dates
from .vocab import CategoryVocab


class NumpyJSONEncoder(json.JSONEncoder):
    """JSON encoder for numpy scalars/arrays (meta files contain numpy ints/floats)."""

    def default(self, o):  # noqa: D401
        if isinstance(o, np.integer):
            return int(o)
        if isinstance(o, np.floating):
            return float(o)
        if isinstance(o, np.bool_):
            return bool(o)
        if isinstance(o, np.ndarray):
            return o.tolist()
        if isinstance(o, complex):
            return {"real": o.real, "imag": o.imag}
        return super().default(o)


def dump_meta_json(meta: dict, path: str) -> None:
    with open(path, "w") as f:
        json.dump(meta, f, sort_keys=True, indent=4, separators=(",", ": "), cls=NumpyJSONEncoder)


def _is_missing(v) -> bool:
    """pd.isna for one object value (None, NaN, NaT, pd.NA), never raising on a non-scalar."""
    try:
        return bool(pd.isna(v))
    except (TypeError, ValueError):
        return False


def _first_appearance(codes: np.ndarray, labels: np.ndarray):
    """(codes, labels) with the labels renumbered in order of first appearance in ``codes`` -- the order
    pd.factorize gives the column itself (its hash pass, which ``value_counts`` ties follow)."""
    u, pos = np.unique(codes, return_index=True)
    order = u[np.argsort(pos, kind="stable")]
    remap = np.empty(len(labels), dtype=np.int64)
    remap[order] = np.arange(len(order))
    return remap[codes], labels[order]


def _categorical_strings(col: pd.Series):
    """(codes, labels) of a pandas categorical column as the object path would see it: blank (" ") and
    missing cells become "empty", labels are the categories' ``str`` forms (equal strings merge), and both
    are in order of first appearance; categories no row holds are dropped (``value_counts`` of the raw
    column does not list them)."""
    cats = np.asarray(col.cat.categories, dtype=object)
    codes = col.cat.codes.to_numpy().astype(np.int64)
    bad = np.asarray([(isinstance(u, str) and u == " ") or _is_missing(u) for u in cats], dtype=bool)
    strs = [str(u) for u in cats[~bad]]
    kmap, labels = pd.factorize(pd.Index(strs, dtype=object)) if strs else (np.zeros(0, np.int64), [])
    labels = list(labels)
    e = labels.index(EMPTY) if EMPTY in labels else len(labels)
    if e == len(labels):
        labels.append(EMPTY)
    m = np.empty(len(cats) + 1, dtype=np.int64)     # m[-1]: the missing code -1
    m[np.nonzero(~bad)[0]] = kmap
    m[np.nonzero(bad)[0]] = e
    m[-1] = e
    return _first_appearance(m[codes], np.asarray(labels, dtype=object))


def timestamp_token() -> str:
    """The reference's folder/file timestamp token (`file_generator.py:97`)."""
    return str(datetime.datetime.now().timestamp()).replace(".", "")


def detect_integer_columns(df: pd.DataFrame) -> List[str]:
    """Integer columns of the raw frame (`file_generator.py:104-110`): an int dtype, or a float dtype whose
    non-null values are all finite whole numbers.  Object columns never qualify (their non-null values
    keep the object dtype), so they are not scanned."""
    out = []
    for c in df.columns:
        col = df[c]
        kind = col.dtype.kind
        if kind in "iu":
            out.append(c)
        elif kind == "f":
            v = col.to_numpy()
            nan = np.isnan(v)
            if nan.any():
                v = v[~nan]
            if np.all(np.isfinite(v)) and np.array_equal(v, np.trunc(v)):
                out.append(c)
    return out


class TablePreprocessor:
    """One client's view of its local CSV (the reference ``FileGenerator``)."""

    def __init__(self, frame: pd.DataFrame, file_name: str, problem_type: str, target_col: str,
                 categorical_list: Sequence[str], non_negative_columns: Sequence[str],
                 date_columns: Optional[Dict[str, str]] = None, synthesizer_used: str = "CTGANSynthesizer"):
        self.file_name = file_name.strip()
        self.problem_type = problem_type.strip()
        self.target_col = target_col.strip()
        self.non_negative_columns = list(non_negative_columns)
        self.date_columns = dict(date_columns or {})
        self.synthesizer_used = synthesizer_used.strip()
        self.output_name = f"{self.file_name}_{self.synthesizer_used}-{timestamp_token()}"

        self.integer_columns = detect_integer_columns(frame)
        self._cat_cache: Dict[str, tuple] = {}
        # blanks -> NaN -> "empty" (`file_generator.py:115-116`), column by column: numeric columns
        # without NaNs are untouched, so only object columns and NaN-holding ones are rewritten.  An
        # object column is factorised once: the blank / missing test runs on its distinct values, and a
        # column of plain strings keeps the factorisation for the categorical pass (_cat_strings)
        df = frame.copy(deep=False)       # columns are replaced, never written in place
        categorical = list(categorical_list) + [d for d in self.date_columns if d not in categorical_list]
        cat_set = set(categorical) - set(self.date_columns)
        for c in df.columns:
            col = df[c]
            if isinstance(col.dtype, pd.CategoricalDtype):
                if c in cat_set:      # codes + categories are already a factorisation: no per-row objects
                    codes, labels = _categorical_strings(col)
                    self._cat_cache[c] = (codes, labels)
                    df[c] = pd.Categorical.from_codes(codes, categories=labels)
                    continue
                col = col.astype(object)
                df[c] = col
            if col.dtype == object:
                codes, uniq = pd.factorize(col, use_na_sentinel=False)
                uniq = np.asarray(uniq, dtype=object)
                bad = np.asarray([(isinstance(u, str) and u == " ") or _is_missing(u) for u in uniq], dtype=bool)
                if bad.any():
                    df[c] = col.where(~bad[codes], EMPTY)
                    if all(isinstance(u, str) for u in uniq[~bad]):
                        # "empty" joins the distinct values (once, even if the literal was already there)
                        labels = list(uniq[~bad])
                        e = labels.index(EMPTY) if EMPTY in labels else len(labels)
                        if e == len(labels):
                            labels.append(EMPTY)
                        remap = np.cumsum(~bad) - 1
                        remap[bad] = e
                        self._cat_cache[c] = _first_appearance(remap[codes], np.asarray(labels, dtype=object))
                elif all(isinstance(u, str) for u in uniq):
                    self._cat_cache[c] = (codes.astype(np.int64, copy=False), uniq)
            elif col.isna().any():
                df[c] = col.astype(object).where(col.notna(), EMPTY)
        untouched = set(categorical) | set(self.date_columns)
        for c in df.columns:
            if c not in untouched and c in self.non_negative_columns:
                df[c] = np.log(df[c].astype(np.float64) + 1.0)
        if self.date_columns:
            df, categorical = split_dates(df, self.date_columns, categorical)
        self.categorical_list = categorical
        # (a date column is replaced by its parts: its factorisation is stale)
        self._cat_cache = {k: v for k, v in self._cat_cache.items() if k in set(categorical) and
                           k not in self.date_columns}
        self.df = df

    def _cat_strings(self, c: str):
        """Column ``c`` as ``(codes, labels)`` with ``labels[codes]`` == ``df[c].astype(str)``.

        Factorises the raw column once and stringifies only its distinct values (a few dozen) instead
        of every row; ``labels`` are in first-appearance order, like the hash pass of ``value_counts``.
        Cached: ``local_meta`` and ``encode`` both need it."""
        hit = self._cat_cache.get(c)
        if hit is None:
            col = self.df[c]
            if col.dtype == object and pd.api.types.infer_dtype(col, skipna=False) != "string":
                # factorize merges objects that hash and compare equal (1, 1.0, True) although they print
                # differently ('1', '1.0', 'True'): key a mixed object column by (type, value)
                keys = pd.Series([(type(v).__name__, None if _is_missing(v) else v) for v in col.tolist()],
                                 dtype=object)
                codes, _ = pd.factorize(keys, use_na_sentinel=False)
                first = pd.Series(np.arange(len(codes))).groupby(codes).first().to_numpy()
                uniq = col.to_numpy()[first]
            else:
                codes, uniq = pd.factorize(col, use_na_sentinel=False)
            strs = pd.Index(uniq).astype(str)
            remap, labels = pd.factorize(strs)          # distinct raw values that print the same merge
            hit = (remap[codes], np.asarray(labels, dtype=object))
            self._cat_cache[c] = hit
        return hit

    # ------------------------------------------------------------------ meta
    def local_meta(self) -> dict:
        cols = []
        for pos, c in enumerate(self.df.columns):
            entry: dict = {"column_name": c}
            if c in self.categorical_list:
                codes, labels = self._cat_strings(c)
                n = np.bincount(codes, minlength=len(labels))
                counts = pd.Series(n, index=pd.Index(labels, dtype=object)).sort_values(ascending=False)
                entry["type"] = CATEGORICAL
                entry["size"] = int(len(counts))
                entry["i2s"] = {str(k): int(v) for k, v in counts.items()}
            else:
                entry["type"] = META_CONTINUOUS
                entry["min"] = self.df[c].min()
                entry["max"] = self.df[c].max()
            entry["column no"] = pos
            cols.append(entry)
        meta = {
            "columns": cols,
            "problem_type": self.problem_type,
            "name": self.output_name,
            "date_info": self.date_columns,
            "integer_info": self.integer_columns,
            "non_negative_cols": self.non_negative_columns,
        }
        if self.target_col:
            meta["target"] = self.target_col
        return meta

    # ------------------------------------------------------------------ encode
    def encode(self, vocabs: Sequence[CategoryVocab]) -> np.ndarray:
        """Label-encode with the global vocabularies; returns float64 [rows, cols] in column-major
        (Fortran) order: every column is written and later read (VGM fits, device upload) contiguously."""
        out = np.empty((self.df.shape[1], len(self.df)), dtype=np.float64).T
        cursor = 0
        for j, c in enumerate(self.df.columns):
            if c in self.categorical_list:
                codes, labels = self._cat_strings(c)
                out[:, j] = vocabs[cursor].transform(labels)[codes]
                cursor += 1
            else:
                out[:, j] = pd.to_numeric(self.df[c]).to_numpy(dtype=np.float64)
        return out

    def categorical_indices(self) -> List[int]:
        return [j for j, c in enumerate(self.df.columns) if c in self.categorical_list]

    def write_artifacts(self, meta: dict, encoded: np.ndarray, timestamp: str,
                        root: str = "dtds/saved_models") -> str:
        """Reference-compatible on-disk dump (`file_generator.py:156-188`)."""
        name = f"{self.file_name}_{self.synthesizer_used}-{timestamp}"
        path = os.path.join(root, name)
        os.makedirs(path, mode=0o760, exist_ok=True)
        dump_meta_json(meta, os.path.join(path, name + ".json"))
        np.savez(os.path.join(path, name + ".npz"), train=encoded, test=encoded[:0])
        frame = pd.DataFrame(encoded, columns=self.df.columns)
        frame.to_csv(os.path.join(path, name + ".csv"), index=False)
        return path


def categorical_columns_of(meta: dict) -> List[int]:
    """Indices of categorical columns in a meta dict (`load.py:26-35`)."""
    return [i for i, c in enumerate(meta["columns"]) if c["type"] == CATEGORICAL]


# pandas.read_csv's default missing-value strings (the arrow reader is told the same)
_PANDAS_NA = ["", "#N/A", "#N/A N/A", "#NA", "-1.#IND", "-1.#QNAN", "-NaN", "-nan", "1.#IND", "1.#QNAN", "<NA>", "N/A",
              "NA", "NULL", "NaN", "None", "n/a", "nan", "null"]
ARROW_MIN_BYTES = 32 << 20


def read_csv_table(path: str, reader: str = "auto") -> pd.DataFrame:
    """A client's CSV (the reference's ``pd.read_csv``, `Server/dtds/data/load.py:51-70`).

    reader "pandas": ``pd.read_csv``.  "arrow": pyarrow's multi-threaded parser with pandas' missing-value and
    boolean spellings; string columns arrive dictionary-encoded, as pandas categoricals, so the preprocessor's
    categorical path never builds per-row Python strings (the wide 100k x 512 table: ~8 s -> ~3.5 s on an
    8-CPU host).  Files with date / time columns or duplicate names (which pandas parses or renames its own
    way) fall back to pandas.  "auto" is pandas: arrow's float parser rounds correctly and pandas' default one
    does not, so the two disagree in the last ulp of ~15-45 % of random doubles (measured on a 400k-row table;
    tests/test_data.py::test_auto_reader_is_pandas_bitwise) and the VGM fits / encodings would differ from the
    reference's load path.
    Arrow stays an explicit opt-in (``-table_reader arrow``) for tables where that does not matter."""
    if reader == "auto":
        reader = "pandas"
    if reader == "pandas":
        return pd.read_csv(path)
    if reader != "arrow":
        raise ValueError(f"table reader must be auto, pandas or arrow, got {reader!r}")
    import pyarrow as pa
    import pyarrow.csv as pc
    opts = pc.ConvertOptions(null_values=_PANDAS_NA, strings_can_be_null=True, true_values=["True", "TRUE", "true"],
                             false_values=["False", "FALSE", "false"], auto_dict_encode=True,
                             auto_dict_max_cardinality=1 << 30, timestamp_parsers=[])
    tb = pc.read_csv(path, convert_options=opts)
    names = tb.schema.names
    if len(set(names)) != len(names) or any(pa.types.is_temporal(f.type) for f in tb.schema):
        return pd.read_csv(path)
    return tb.to_pandas()


def load_table(path: str, spec, reader: str = "auto") -> TablePreprocessor:
    frame = read_csv_table(path, reader)
    stem = os.path.splitext(os.path.basename(path))[0]
    return TablePreprocessor(frame[spec.selected_variables], stem, spec.problem_type,
                             "" if spec.target_column == "none" else spec.target_column,
                             spec.categorical_list, spec.nonnegative_list, spec.date_dic)
