"""Device memory for the batched multi-client engine: K identical client slabs in one allocation.

The HIP kernels run K federated clients' training steps in ONE launch each (``csrc/kernels/launch.h``
``ClientBatch``): client c = blockIdx.z reads and writes the buffers ``c * stride`` bytes after client
0's.  That only works if every buffer a step touches lives in one arena with an identical layout per
client, which is what this module provides:

* ``TorchAlloc`` -- plain torch allocations (the single-client engine, and every engine once a batch
  is frozen, for anything outside a batched launch -- generation buffers, decode tables);
* ``Arena`` -- one ``uint8`` device tensor of ``K * stride`` bytes; ``Arena.slab(c)`` is client c's
  bump allocator.  Engines built from slab allocators in the same order with the same shapes end up
  with byte-identical layouts (``Arena.freeze`` verifies the allocation logs);
* ``Arena.group`` -- the allocator of the lazily created operands of a batched launch (split-K
  workspaces, span tables...): one offset reserved in every slab at once.

The native launchers refuse any pointer of a batched launch that is not inside client 0's slab, so a
buffer that escaped the arena fails loudly instead of silently aliasing client 0's memory.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np
import torch

ALIGN = 256


def _nbytes(shape, dtype) -> int:
    return int(np.prod(shape, dtype=np.int64)) * torch.empty((), dtype=dtype).element_size()


class TorchAlloc:
    """The allocator interface on plain torch allocations."""

    def __init__(self, device):
        self.device = torch.device(device)

    def zeros(self, *shape, dtype=torch.float32) -> torch.Tensor:
        if len(shape) == 1 and isinstance(shape[0], (tuple, list)):
            shape = tuple(shape[0])
        return torch.zeros(*shape, dtype=dtype, device=self.device)

    def tensor(self, data, dtype=None) -> torch.Tensor:
        """A device copy of ``data`` (array-like or tensor)."""
        t = torch.as_tensor(data, dtype=dtype)
        return t.to(self.device, copy=True).contiguous() if t.device != self.device else t.clone().contiguous()


class _Slab(TorchAlloc):
    def __init__(self, arena: "Arena", c: int):
        super().__init__(arena.device)
        self.arena, self.c = arena, c
        self.log: List[Tuple[int, int]] = []

    def zeros(self, *shape, dtype=torch.float32) -> torch.Tensor:
        if len(shape) == 1 and isinstance(shape[0], (tuple, list)):
            shape = tuple(shape[0])
        a = self.arena
        if a.batch_active:            # an operand created while a batched step is issued: every slab
            return a.group.zeros(*shape, dtype=dtype)
        if a.frozen:                  # outside a batched launch after the freeze: plain memory
            return super().zeros(*shape, dtype=dtype)
        n = _nbytes(shape, dtype)
        off = a.cursor[self.c]
        a.cursor[self.c] = off + (n + ALIGN - 1) // ALIGN * ALIGN
        if a.cursor[self.c] > a.stride:
            raise MemoryError(f"client slab overflow: {a.cursor[self.c]} > {a.stride} bytes (raise the arena size)")
        self.log.append((off, n))
        return a.view(self.c, off, shape, dtype)

    def tensor(self, data, dtype=None) -> torch.Tensor:
        if self.arena.batch_active:   # a table created while a batched step is issued: shared by every client
            return self.arena.group.tensor(data, dtype)
        t = torch.as_tensor(data, dtype=dtype)
        out = self.zeros(*t.shape, dtype=t.dtype)
        out.copy_(t)
        return out


class _Group(TorchAlloc):
    """One allocation at the same offset of every slab; returns client 0's view."""

    def __init__(self, arena: "Arena"):
        super().__init__(arena.device)
        self.arena = arena

    def zeros(self, *shape, dtype=torch.float32) -> torch.Tensor:
        if len(shape) == 1 and isinstance(shape[0], (tuple, list)):
            shape = tuple(shape[0])
        a = self.arena
        n = _nbytes(shape, dtype)
        off = max(a.cursor)
        end = off + (n + ALIGN - 1) // ALIGN * ALIGN
        if end > a.stride:
            raise MemoryError(f"client slab overflow in a batched launch: {end} > {a.stride} bytes")
        a.cursor = [end] * a.k
        for c in range(a.k):
            a.view(c, off, shape, dtype).zero_()
        return a.view(0, off, shape, dtype)

    def tensor(self, data, dtype=None) -> torch.Tensor:
        """The same data in every slab (a table shared by every client)."""
        t = torch.as_tensor(data, dtype=dtype)
        out = self.zeros(*t.shape, dtype=t.dtype)
        a = self.arena
        off = out.data_ptr() - a.base
        for c in range(a.k):
            a.view(c, off, tuple(t.shape), t.dtype).copy_(t)
        return out


class Arena:
    def __init__(self, k: int, slab_bytes: int, device):
        self.k = int(k)
        self.stride = (int(slab_bytes) + ALIGN - 1) // ALIGN * ALIGN
        self.device = torch.device(device)
        self.buf = torch.zeros(self.k * self.stride, dtype=torch.uint8, device=self.device)
        self.base = self.buf.data_ptr()
        self.cursor = [0] * self.k
        self.frozen = False
        self.batch_active = False
        self.slabs = [_Slab(self, c) for c in range(self.k)]
        self.group = _Group(self)

    def slab(self, c: int) -> _Slab:
        return self.slabs[c]

    def view(self, c: int, off: int, shape, dtype) -> torch.Tensor:
        n = _nbytes(shape, dtype)
        start = c * self.stride + off
        return self.buf[start:start + n].view(dtype).view(*shape) if n else \
            torch.zeros(shape, dtype=dtype, device=self.device)

    def client_view(self, t: torch.Tensor, c: int) -> torch.Tensor:
        """Client c's copy of a tensor that lives in client 0's slab (same shape, strides, offset)."""
        off = t.data_ptr() - self.base
        if not 0 <= off < self.stride:
            raise ValueError("client_view: the tensor is not in client 0's slab")
        flat = self.buf[c * self.stride:(c + 1) * self.stride].view(t.dtype) if off % t.element_size() == 0 else None
        if flat is None:
            raise ValueError("client_view: misaligned tensor")
        return flat.as_strided(t.shape, t.stride(), off // t.element_size())

    def freeze(self) -> None:
        """Every client slab was filled by the same allocation sequence (identical layouts); from here
        on allocations outside a batched launch are plain torch memory."""
        logs = [s.log for s in self.slabs]
        for c, lg in enumerate(logs[1:], 1):
            if lg != logs[0]:
                first = next((i for i, (x, y) in enumerate(zip(lg, logs[0])) if x != y), min(len(lg), len(logs[0])))
                raise RuntimeError(f"client {c}'s buffers do not mirror client 0's (first difference at allocation "
                                   f"{first} of {len(logs[0])} / {len(lg)}): the batched engine needs identical "
                                   "shapes on every client (same row counts, same layout)")
        self.frozen = True

    @staticmethod
    def estimate_slab_bytes(layout, cfg, n_rows: int, extra: int = 64 << 20) -> int:
        """Upper bound of one client's arena bytes: the flat parameter / gradient / Adam buffers, the
        step's activations, the training tables, and ``extra`` for the lazily sized operands (split-K
        workspaces, BN partials, span tables)."""
        E, C, Dd = cfg.embedding_dim, layout.n_opt, layout.data_dim
        din = Dd + C
        k1 = cfg.pack * din
        g, d = list(cfg.gen_dims), list(cfg.dis_dims)
        params = 0
        dim = E + C
        for h in g:
            params += (h + 4) * (dim + 4) + 4 * h
            dim += h
        params += (Dd + 4) * (dim + 4) + Dd
        dim = k1
        for h in d:
            params += h * (dim + 4) + h
            dim = h
        params += dim + 8 + 4 * sum(g)
        B = cfg.batch_size
        hw = E + C + sum(g)
        acts = 2 * B * (hw + 4) + 6 * 2 * B * max(g + [1]) + 4 * B * (Dd + 4) + B * (hw + 4) + 4 * B * din \
            + 12 * (3 * B // cfg.pack) * max(d + [1]) + (B // cfg.pack) * k1 + 8 * B
        data = n_rows * Dd + 2 * n_rows * layout.n_col + 4 * layout.n_col * max(1, int(np.max(layout.cond_width)))
        return int(4 * (4 * params + acts) + 4 * data + extra)
