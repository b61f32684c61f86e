"""K federated clients' training steps as ONE batched launch sequence on one GPU.

The reference trains its clients in parallel processes (`Server/dtds/distributed.py:794-825`: an
``rpc_async(train_model)`` per client, then the weighted merge).  On a single MI355X, K clients used
to be K threads, each with its own engine, HIP stream and step graph (``fed/local.py``): 25 small
launches per step per client, spread over the 4 hardware queues.  Here the K engines share one device
arena (``models/arena.py``) with identical per-client layouts, and client 0's engine issues every launch
of a step ONCE for all of them: the kernels take the client index from ``blockIdx.z`` and offset every
pointer by ``client * slab_stride`` (``csrc/kernels/launch.h`` ``ClientBatch``).  A K-client step is the
same 25 launches with K times the workgroups; the weighted FedAvg of the K flat buffers is one reduction
over the arena instead of K device-synchronised accumulations on the host's thread.

Every client keeps its own model, Adam moments, Philox streams (seed ``seed_0 + c``), BN statistics and
training tables, so each client's trajectory is bit-identical to a single-client engine with the same
seed, weights and data (tests/test_batched.py).  Requirements: the HIP backend, the same layout and
row count on every client (identical buffer shapes), consecutive engine seeds.
"""
from __future__ import annotations

import weakref
from typing import List, Sequence

import numpy as np
import torch

from .arena import Arena
from .engine import CTGANEngine, EngineConfig


class BatchedClients:
    def __init__(self, layout, cfg: EngineConfig, device, seeds: Sequence[int], n_rows: int, backend: str = "hip",
                 slab_bytes: int | None = None):
        seeds = [int(s) for s in seeds]
        if any(s != seeds[0] + c for c, s in enumerate(seeds)):
            raise ValueError(f"batched clients need consecutive engine seeds (client c: seed_0 + c), got {seeds}")
        self.k = len(seeds)
        self.device = torch.device(device)
        self.arena = Arena(self.k, slab_bytes or Arena.estimate_slab_bytes(layout, cfg, n_rows), self.device)
        self.engines: List[CTGANEngine] = [
            CTGANEngine(layout, cfg, self.device, backend=backend, seed=seeds[c], mem=self.arena.slab(c))
            for c in range(self.k)]
        e0 = self.engines[0]
        if e0.ops.name != "hip":
            raise ValueError("batched clients need the HIP backend")
        # (a weak back-reference: a strong one would make a cycle whose collection -- at an arbitrary moment,
        # e.g. while another engine captures a graph -- destroys this group's step graphs mid-capture)
        e0.batch = weakref.proxy(self)
        self._frozen = False

    @classmethod
    def empty(cls, k: int, device, stride: int):
        """An arena without engines yet: engines are built one by one by the client threads
        (``engine_for``), each from its own slab."""
        self = cls.__new__(cls)
        self.k = int(k)
        self.device = torch.device(device)
        self.arena = Arena(self.k, stride, self.device)
        self.engines = [None] * self.k
        self._frozen = False
        return self

    def engine_for(self, c: int, layout, cfg: EngineConfig, seed: int, backend: str = "hip") -> CTGANEngine:
        e = CTGANEngine(layout, cfg, self.device, backend=backend, seed=seed, mem=self.arena.slab(c))
        self.engines[c] = e
        if c == 0:
            e.batch = weakref.proxy(self)
        return e

    # ------------------------------------------------------------------ state
    def freeze(self) -> None:
        """All clients' engines are built and hold their training tables: verify identical layouts
        and consecutive seeds; from here on client 0 issues the batched steps."""
        if self._frozen:
            return
        if any(e is None for e in self.engines):
            raise RuntimeError("batched clients: not every client built its engine")
        s0 = self.engines[0].ops.seed
        for c, e in enumerate(self.engines):
            if e.ops.seed != s0 + c:
                raise RuntimeError(f"batched clients: client {c}'s seed {e.ops.seed} is not seed_0 + {c}")
            if not e.tables:
                raise RuntimeError(f"batched clients: client {c} has no training data")
            if e.steps_per_epoch != self.engines[0].steps_per_epoch:
                raise RuntimeError("batched clients: every client needs the same steps per epoch")
        self.arena.freeze()
        self._frozen = True

    def state_tensors(self) -> List[torch.Tensor]:
        """Every client's persistent training state (the capture warm-up snapshot)."""
        out = []
        for e in self.engines:
            out += [e.flat, e.mG, e.vG, e.mD, e.vD, e.stepG, e.stepD]
        return out

    # ------------------------------------------------------------------ training
    def _batched(self):
        e0 = self.engines[0]
        a = self.arena
        return _BatchContext(e0.ops, self.k, a.stride, a.base, a)

    def train_steps(self, n: int, use_graph: bool | None = None) -> None:
        """n steps of every client, each launch of a step issued once for all K clients."""
        self.freeze()
        e0 = self.engines[0]
        with self._batched():
            e0.train_steps(n, use_graph)
        for e in self.engines[1:]:
            e.bn_batches = e0.bn_batches

    def train_epoch(self, use_graph: bool | None = None) -> None:
        self.train_steps(self.engines[0].steps_per_epoch, use_graph)

    # ------------------------------------------------------------------ aggregation
    def owns(self, flat: torch.Tensor) -> bool:
        """Is ``flat`` one of the clients' flat buffers?"""
        return any(e is not None and e.flat.data_ptr() == flat.data_ptr() for e in self.engines)

    def flats(self) -> torch.Tensor:
        """[K, n] view of every client's flat buffer (parameters + BN statistics)."""
        f0 = self.engines[0].flat
        off = f0.data_ptr() - self.arena.base
        n = f0.numel()
        return self.arena.buf.view(self.k, self.arena.stride)[:, off:off + 4 * n].view(torch.float32)

    def weighted_average(self, weights: Sequence[float]) -> None:
        """FedAvg of every client's parameters and BN statistics (`Server/dtds/distributed.py:86-106`):
        every client ends holding sum_c w_c theta_c.  Runs on the current stream, no host sync."""
        w = torch.as_tensor(np.asarray(weights, dtype=np.float32), device=self.device)
        F = self.flats()
        agg = torch.mv(F.t(), w) if self.k > 1 else F[0] * w[0]
        F.copy_(agg.unsqueeze(0).expand_as(F))


class _BatchContext:
    def __init__(self, ops, k, stride, base, arena):
        self.ops, self.k, self.stride, self.base, self.arena = ops, k, stride, base, arena

    def __enter__(self):
        self.arena.batch_active = True
        self.prev = self.ops.set_client_batch(self.k, self.stride, 1, self.base)
        return self

    def __exit__(self, *exc):
        self.ops.set_client_batch(1)
        self.arena.batch_active = False
        return False
