"""Synthetic-table CSV writer.

The reference writes every epoch's 40,000-row table with ``DataFrame.to_csv`` after a
pandas ``Transform.inverse`` pass (`Server/dtds/distributed.py:584-590`), ~1.1 s per epoch on
the survey box.  The native path formats the numeric decode output directly in C++
(``csrc/host/csv_writer.cpp``: Python-``repr``-compatible shortest round-trip floats, vocab
lookups for categoricals, the non-negative ``exp(x)-1`` / ceil rule, multi-threaded over
row blocks, date columns re-joined from their part codes) and writes the file in one call.
Byte-for-byte the output equals the pandas path (tested, date schemas included).
"""
from __future__ import annotations

from typing import Sequence

import numpy as np

from ..data.decode import KIND_FLOAT, KIND_NONNEG, KIND_VOCAB, CsvLayout


def _native():
    from ..ops import native
    return native.lib() if native.available() else None


def available() -> bool:
    try:
        return _native() is not None
    except Exception:
        return False


def _py_float(x: float) -> str:
    return repr(float(x))


def format_table_py(values: np.ndarray, names: Sequence[str], kinds: Sequence[int],
                    vocabs: Sequence[Sequence[str]], empty_minus_one=None) -> bytes:
    out = [",".join(_quote(n) for n in names)]
    cols = []
    for j, k in enumerate(kinds):
        v = values[:, j]
        if k == KIND_FLOAT and empty_minus_one is not None and empty_minus_one[j]:
            cols.append([" " if x == -1.0 else _py_float(x) for x in v])
        elif k == KIND_FLOAT:
            cols.append([_py_float(x) for x in v])
        elif k == KIND_VOCAB:
            voc = vocabs[j]
            cols.append([voc[int(x)] for x in v])
        else:
            w = np.exp(v) - 1.0
            neg = w < 0
            w[neg] = np.ceil(w[neg])
            cols.append([" " if x == -1.0 else _py_float(x) for x in w])
    for row in zip(*cols):
        out.append(",".join(_quote(s) for s in row))
    return ("\n".join(out) + "\n").encode()


def _quote(s: str) -> str:
    if any(ch in s for ch in ',"\n\r'):
        return '"' + s.replace('"', '""') + '"'
    return s


def write_table(path: str, values: np.ndarray, names: Sequence[str], kinds: Sequence[int],
                vocabs: Sequence[Sequence[str]], threads: int = 0) -> None:
    """One output column per value column (kinds 0..2)."""
    write_layout(path, values, CsvLayout(list(names), list(kinds), [list(v) for v in vocabs], list(range(len(kinds)))),
                 threads)


def _nonneg(v: np.ndarray) -> np.ndarray:
    """exp(x)-1 with ceil for negatives, with numpy's exp (bit-identical to the pandas path)."""
    w = np.exp(v) - 1.0
    neg = w < 0
    w[neg] = np.ceil(w[neg])
    return w


def write_layout(path: str, values: np.ndarray, layout: CsvLayout, threads: int = 0) -> None:
    """Write the decoded value matrix as ``layout`` (``data.decode.csv_layout``) describes it.

    The matrix is read in place: only the non-negative columns are mapped (into a small side matrix
    the formatter reads them from).  A full host copy of a 40k-row table costs ~2 ms of GIL-holding
    memcpy per epoch -- in the background writer that stalls the main thread's graph launches."""
    values = np.ascontiguousarray(values, dtype=np.float64)
    nn = [j for j, k in enumerate(layout.kinds) if k == KIND_NONNEG]
    lib = _native()
    if lib is not None:
        from ..ops import native
        src = list(layout.src)
        aux = None
        if nn:
            aux = np.empty((values.shape[0], len(nn)), dtype=np.float64)
            for i, j in enumerate(nn):
                aux[:, i] = _nonneg(values[:, layout.src[j]])
                src[j] = values.shape[1] + i
        native.write_csv(path, values, layout.names, layout.kinds, layout.vocabs, threads, src,
                         layout.date_desc, layout.date_lut, aux=aux)
        return
    if layout.has_dates:
        raise RuntimeError("the Python CSV formatter has no date columns (native library not loaded)")
    vals = values[:, layout.src]          # (a copy: fancy indexing)
    for j in nn:
        vals[:, j] = _nonneg(vals[:, j])
    kinds_py = [KIND_FLOAT if k == KIND_NONNEG else k for k in layout.kinds]
    with open(path, "wb") as f:
        f.write(format_table_py(vals, layout.names, kinds_py, layout.vocabs,
                                empty_minus_one=[k == KIND_NONNEG for k in layout.kinds]))


class AsyncTableWriter:
    """Writes epoch tables on one background thread so formatting + file IO of round ``r``
    overlaps the GPU training of round ``r + 1`` (the native formatter releases the GIL).
    Writes complete in submission order; :meth:`flush` waits for all of them and re-raises
    the first failure."""

    def __init__(self):
        from concurrent.futures import ThreadPoolExecutor
        self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="csv-writer")
        self._pending = []

    def submit(self, fn, *args, **kwargs):
        self._pending.append(self._pool.submit(fn, *args, **kwargs))
        self._pending = [f for f in self._pending if not f.done() or f.exception() is not None]

    def flush(self):
        pending, self._pending = self._pending, []
        for f in pending:
            f.result()

    def close(self):
        self.flush()
        self._pool.shutdown(wait=True)
