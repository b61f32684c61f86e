"""Device-side VGM encode and real-row index (K1 + K5 tables of the survey).

:func:`encode_on_device` runs the HIP ``vgm_encode`` kernel (csrc/kernels/vgm.hip) over the
label-encoded table and returns a :class:`DeviceEncoded`. It holds:
- the encoded training matrix, resident on the GPU;
- the option index of every (row, conditional span);
- the CSR real-row lists per (span, option), built from one stable device sort per span (the
  reference builds them with a Python loop, `Server/dtds/synthesizers/ctgan.py:205-217`);
- the one-hot column sums that drive the conditional sampler.

Nothing of size ``rows x data_dim`` crosses PCIe. On the wide 100k x 512 table the encoded
matrix is 2.8 GB.

The host path (:meth:`VGMTransformer.transform`, numpy) remains the CPU implementation and
the test oracle. The two draw different uniforms, so they agree in distribution; they agree
bit for bit on the categorical one-hots and on alpha given the drawn mode.
"""
from __future__ import annotations

import dataclasses
from typing import Dict

import numpy as np
import torch

from .transformer import CONTINUOUS, VGMTransformer


@dataclasses.dataclass
class DeviceEncoded:
    data: torch.Tensor          # [N, data_dim] float32
    opt: torch.Tensor           # [N, n_col] int32
    counts: np.ndarray          # [n_col, max_width] float64 one-hot column sums
    rows: Dict[str, torch.Tensor]   # row_offset / row_count [n_col, max_width] int64, rows [n_col * N] int64

    def __len__(self) -> int:
        return int(self.data.shape[0])


def _tables(tr: VGMTransformer, device) -> Dict[str, torch.Tensor]:
    cache = getattr(tr, "_device_tables", None)
    if cache is not None and cache.get("device") == str(device):
        return cache
    lay = tr.layout
    bank = tr.bank
    K = tr.n_clusters
    if K != 10:
        raise ValueError("the device encoder is built for 10-component VGMs")
    kind, pos, aux, span, lut_n = [], [], [], [], []
    lut = []
    p = 0
    c = 0
    s = 0   # conditional span counter (every softmax span in order)
    for m in tr.meta:
        if m["type"] == CONTINUOUS:
            kind.append(0)
            pos.append(p)
            aux.append(c)
            span.append(s)
            lut_n.append(0)
            if not tr.components[c].any():
                raise ValueError("a continuous column without a valid VGM mode")
            p += 1 + int(tr.components[c].sum())
            c += 1
        else:
            kind.append(1)
            pos.append(p)
            aux.append(len(lut))
            span.append(s)
            codes = [int(v) for v in m["i2s"]]
            if any(v < 0 or float(v) != float(w) for v, w in zip(codes, m["i2s"])):
                raise ValueError("device encode needs label codes 0..V-1 in categorical columns")
            table = np.zeros(max(codes) + 1 if codes else 1, dtype=np.int32)
            for i, v in enumerate(codes):
                table[v] = i
            lut.extend(table.tolist())
            lut_n.append(len(table))
            p += int(m["size"])
        s += 1
    assert s == lay.n_col and p == lay.data_dim
    n_cont = bank.n
    if n_cont:
        consts = bank.log_prob_consts()
        vrank = np.where(tr.components, np.cumsum(tr.components, axis=1) - 1, -1)
        means, prec, stds = bank.means, bank.prec_chol, bank.stds
    else:
        consts = means = prec = stds = np.zeros((1, K))
        vrank = -np.ones((1, K), dtype=np.int64)
    i32 = lambda v: torch.as_tensor(np.asarray(v, dtype=np.int32), device=device)    # noqa: E731
    f32 = lambda v: torch.as_tensor(np.asarray(v, dtype=np.float32), device=device)  # noqa: E731
    cache = {"device": str(device), "kind": i32(kind), "pos": i32(pos), "aux": i32(aux), "span": i32(span),
             "lut_n": i32(lut_n), "cat_cols": [j for j, k in enumerate(kind) if k == 1],
             "cat_n": [n for n, k in zip(lut_n, kind) if k == 1],
             "consts": f32(consts), "means": f32(means), "prec": f32(prec), "stds": f32(stds), "vrank": i32(vrank),
             "lut": i32(lut if lut else [0])}
    tr._device_tables = cache
    return cache


def row_index_on_device(opt: torch.Tensor, layout) -> tuple:
    """CSR row lists per (span, option) + one-hot counts from the option matrix [N, n_col]: this library's
    counting sort (csrc/kernels/init_ops.hip csr_rows; rows ascending in every list, deterministic) on a GPU,
    the torch formulation below elsewhere (and as its test oracle)."""
    n, n_col = opt.shape
    maxw = int(layout.cond_width.max()) if layout.n_col else 0
    if opt.is_cuda and n and n_col and maxw:
        from ..ops import native
        dev = opt.device
        chunk = 4096
        chunks = -(-n // chunk)
        part = torch.empty(n_col * chunks * maxw, dtype=torch.int32, device=dev)
        count = torch.empty(n_col, maxw, dtype=torch.int64, device=dev)
        offset = torch.empty(n_col, maxw, dtype=torch.int64, device=dev)
        rows = torch.empty(n_col * n, dtype=torch.int64, device=dev)
        width = torch.as_tensor(np.asarray(layout.cond_width, dtype=np.int32), device=dev)
        native.require().csr_rows(opt.contiguous(), width, maxw, part, count, offset, rows, chunk)
        return ({"row_offset": offset, "row_count": count, "rows": rows},
                count.cpu().numpy().astype(np.float64))
    return row_index_torch(opt, layout)


def row_index_torch(opt: torch.Tensor, layout) -> tuple:
    """row_index_on_device as torch ops (argsort per span)."""
    n, n_col = opt.shape
    maxw = int(layout.cond_width.max()) if layout.n_col else 0
    o = opt.long()
    order = torch.argsort(o, dim=0, stable=True)                       # per span: rows by option
    counts = torch.zeros(n_col, maxw, dtype=torch.int64, device=opt.device)
    counts.scatter_add_(1, o.t(), torch.ones_like(o.t()))
    starts = torch.cumsum(counts, dim=1) - counts
    base = (torch.arange(n_col, device=opt.device, dtype=torch.int64) * n)[:, None]
    width = torch.as_tensor(np.asarray(layout.cond_width, dtype=np.int64), device=opt.device)
    live = torch.arange(maxw, device=opt.device)[None, :] < width[:, None]     # padding slots stay 0
    rows = {"row_offset": torch.where(live, starts + base, torch.zeros_like(starts)).contiguous(), "row_count": counts,
            "rows": order.t().contiguous().reshape(-1)}
    return rows, counts.double().cpu().numpy()


def encode_on_device(tr: VGMTransformer, data: np.ndarray, device, seed: int = 0) -> DeviceEncoded:
    from ..ops import native
    L = native.require()
    t = _tables(tr, device)
    data = np.asarray(data, dtype=np.float64)
    if data.ndim != 2 or data.shape[1] != len(tr.meta):
        raise ValueError(f"expected a [rows, {len(tr.meta)}] table")
    # a column-major table (TablePreprocessor.encode) is uploaded as its [cols, rows] transpose and
    # turned row-major on the device: no host-side transposing copy of the (wide: 400 MB) matrix
    if t["cat_cols"]:
        # every code must index its LUT row (checked on the host, column by column: no ATen kernel)
        for j, nc in zip(t["cat_cols"], t["cat_n"]):
            v = data[:, j]
            bad = ~np.isfinite(v) | (v < 0) | (v >= nc) | (v != np.floor(v))
            if len(v) and bad.any():
                raise ValueError(f"column {j}: category codes outside 0..{int(nc) - 1}")
    if data.flags.f_contiguous and not data.flags.c_contiguous:
        x = torch.as_tensor(data.T, device=device).t()     # read column-major by the kernel (ldc = rows)
    else:
        x = torch.as_tensor(np.ascontiguousarray(data), device=device)
    n = x.shape[0]
    lay = tr.layout
    out = torch.zeros(n, lay.data_dim, dtype=torch.float32, device=device)
    opt = torch.zeros(n, lay.n_col, dtype=torch.int32, device=device)
    L.vgm_encode(x, out, opt, t["kind"], t["pos"], t["aux"], t["span"], t["lut_n"], t["consts"], t["means"], t["prec"],
                 t["stds"], t["vrank"], t["lut"], int(seed) & ((1 << 62) - 1), 41)
    rows, counts = row_index_on_device(opt, lay)
    return DeviceEncoded(out, opt, counts, rows)
