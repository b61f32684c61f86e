"""Loader for the in-tree native library ``fed_tgan_amd/_C.so`` (HIP kernels + host C++).

Built by ``csrc/build.py`` (hipcc, ``--offload-arch=gfx950``) and registered as the
``torch.ops.fedtgan`` namespace.  On a GPU box the HIP backend refuses to fall back to
eager PyTorch: :func:`require` raises if the library is missing or fails to load.
"""
from __future__ import annotations

import os
import threading
from typing import Sequence

import numpy as np
import torch

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# FEDTGAN_CHECKED=1: the device bounds-checked build (csrc/build.py --checked)
CHECKED = os.environ.get("FEDTGAN_CHECKED", "0") not in ("", "0")
LIB_PATH = os.path.join(PKG_DIR, "_C_checked.so" if CHECKED else "_C.so")
# FEDTGAN_LIB=<path>: load another build of the same ops (A/B of kernel revisions on one box)
LIB_PATH = os.environ.get("FEDTGAN_LIB") or LIB_PATH

CHECK_NAMES = {0: "sampler CSR pick outside the row lists", 1: "sampler data row outside the training matrix",
               2: "sampler condition outside the span tables", 3: "decode code index outside the code table",
               4: "decode mode index >= K", 5: "one-hot gather index outside the conditional block",
               6: "encode label outside the lookup table"}

_lock = threading.Lock()
_loaded = None
_error = None


def _load():
    global _loaded, _error
    with _lock:
        if _loaded is not None or _error is not None:
            return
        if not os.path.exists(LIB_PATH):
            _error = f"native library not built: {LIB_PATH} (run `python csrc/build.py`)"
            return
        try:
            torch.ops.load_library(LIB_PATH)
            _loaded = torch.ops.fedtgan
        except Exception as e:  # pragma: no cover - surfaced by require()
            _error = f"failed to load {LIB_PATH}: {e}"


def available() -> bool:
    _load()
    return _loaded is not None


def lib():
    _load()
    return _loaded


def require():
    _load()
    if _loaded is None:
        raise RuntimeError(_error or "native library unavailable")
    return _loaded


def check() -> None:
    """Checked build: raise if any kernel since the last call flagged an out-of-range index (the
    access itself was clamped).  A no-op with the release library."""
    L = require()
    if not CHECKED:
        return
    bits = int(L.check_status())
    if bits:
        raise RuntimeError("device bounds check failed: " +
                           "; ".join(n for b, n in CHECK_NAMES.items() if bits >> b & 1))


def write_csv(path: str, values: np.ndarray, names: Sequence[str], kinds: Sequence[int],
              vocabs: Sequence[Sequence[str]], threads: int = 0, src: Sequence[int] = (),
              date_desc: Sequence[int] = (), date_lut: Sequence[int] = (), aux: np.ndarray | None = None) -> None:
    """Native CSV formatter (csrc/host/csv_writer.cpp).  Output column j has kinds[j], names[j], vocabs[j]
    and reads value column src[j] (default j; src >= values' width reads column src - width of ``aux``);
    date columns: see ``data.decode.CsvLayout``."""
    L = require()
    flat, offs = [], [0]
    for v in vocabs:
        flat.extend(v)
        offs.append(len(flat))
    t = torch.from_numpy(np.ascontiguousarray(values, dtype=np.float64))
    L.write_csv(path, t, list(names), [int(k) for k in kinds], flat, offs, int(threads), [int(x) for x in src],
                [int(x) for x in date_desc], [int(x) for x in date_lut],
                None if aux is None else torch.from_numpy(np.ascontiguousarray(aux, dtype=np.float64)))
