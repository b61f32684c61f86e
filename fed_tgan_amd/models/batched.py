"""K federated clients' training steps as ONE batched launch sequence on one GPU.

The reference trains its clients in parallel processes (`Server/dtds/distributed.py:794-825`: an
``rpc_async(train_model)`` per client, then the weighted merge).  On a single MI355X, K clients used
to be K threads, each with its own engine, HIP stream and step graph (``fed/local.py``): 25 small
launches per step per client, spread over the 4 hardware queues.  Here the K engines share one device
arena (``models/arena.py``) with identical per-client layouts, and client 0's engine issues every launch
of a step ONCE for all of them: the kernels take the client index from ``blockIdx.z`` and offset every
pointer by ``client * slab_stride`` (``csrc/kernels/launch.h`` ``ClientBatch``).  A K-client step is the
same 25 launches with K times the workgroups; the weighted FedAvg of the K flat buffers is one reduction
over the arena instead of K accumulations on the host's thread.

Every client keeps its own model, Adam moments, Philox streams (seed ``seed_0 + c``), BN statistics and
training tables, so each client's trajectory is bit-identical to a single-client engine with the same
seed, weights and data (tests/test_batched.py).

Clients with different row counts (non-IID shards): in the reference every client trains
``len(train) // batch_size`` steps per round (`Client/.../dtds/distributed.py:155, 186`) and the server
waits for all of them (`Server/dtds/distributed.py:800-806`).  Here every slab reserves the largest
client's row tables (``CTGANEngine.pad_rows``), and the slabs hold the clients in non-increasing order of
steps per epoch, so at any step of an epoch the clients still training are a PREFIX of the slabs: an epoch
is a few segments, each a launch sequence over the first k clients (grid.z = k; k = 1 is the plain
single-client launch).  A client whose epoch is over takes no part in the launches that remain, so its
Adam step counters, Philox stream and BN statistics stop exactly where a single engine's would.
Requirements: the HIP backend, the same layout on every client, consecutive engine seeds in slab order.
"""
from __future__ import annotations

import weakref
from typing import List, Sequence

import numpy as np
import torch

from .arena import Arena
from .engine import CTGANEngine, EngineConfig


def slab_order(steps: Sequence[int]) -> List[int]:
    """Clients in slab order: non-increasing steps per epoch, ties by client index (so equal clients keep
    their own index as slab).  ``slab_order(steps)[s]`` is the client held by slab s."""
    return sorted(range(len(steps)), key=lambda c: (-int(steps[c]), c))


class BatchedClients:
    def __init__(self, layout, cfg: EngineConfig, device, seeds: Sequence[int], n_rows: int, backend: str = "hip",
                 slab_bytes: int | None = None):
        """n_rows: the largest client's row count (every slab's row tables are sized for it)."""
        seeds = [int(s) for s in seeds]
        if any(s != seeds[0] + c for c, s in enumerate(seeds)):
            raise ValueError(f"batched clients need consecutive engine seeds (client c: seed_0 + c), got {seeds}")
        self.k = len(seeds)
        self.device = torch.device(device)
        self.n_rows = int(n_rows)
        self.arena = Arena(self.k, slab_bytes or Arena.estimate_slab_bytes(layout, cfg, n_rows), self.device)
        self.engines: List[CTGANEngine] = []
        for c in range(self.k):
            e = CTGANEngine(layout, cfg, self.device, backend=backend, seed=seeds[c], mem=self.arena.slab(c))
            e.pad_rows = self.n_rows
            self.engines.append(e)
        e0 = self.engines[0]
        if e0.ops.name != "hip":
            raise ValueError("batched clients need the HIP backend")
        # (a weak back-reference: a strong one would make a cycle whose collection -- at an arbitrary moment,
        # e.g. while another engine captures a graph -- destroys this group's step graphs mid-capture)
        e0.batch = weakref.proxy(self)
        self.client_of_slab = list(range(self.k))
        self._frozen = False

    @classmethod
    def empty(cls, k: int, device, stride: int, n_rows: int = 0):
        """An arena without engines yet: engines are built one by one by the client threads
        (``engine_for``), each from its own slab.  Every slab is zero-filled and the fill is complete on
        the device when this returns (the threads write their slabs from their own streams)."""
        self = cls.__new__(cls)
        self.k = int(k)
        self.device = torch.device(device)
        self.n_rows = int(n_rows)
        self.arena = Arena(self.k, stride, self.device)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        self.engines = [None] * self.k
        self.client_of_slab = list(range(self.k))
        self._frozen = False
        return self

    def engine_for(self, slab: int, layout, cfg: EngineConfig, seed: int, backend: str = "hip") -> CTGANEngine:
        e = CTGANEngine(layout, cfg, self.device, backend=backend, seed=seed, mem=self.arena.slab(slab))
        e.pad_rows = self.n_rows or None
        self.engines[slab] = e
        if slab == 0:
            e.batch = weakref.proxy(self)
        return e

    # ------------------------------------------------------------------ state
    def freeze(self) -> None:
        """All clients' engines are built and hold their training tables: verify identical layouts,
        consecutive seeds and the slab order (non-increasing steps per epoch); from here on client 0's
        engine issues the batched steps.  The first call synchronises the device once: every client's
        initial state was written on its own thread's stream, the batched launches run on one stream."""
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
        steps = self.steps()
        if any(a < b for a, b in zip(steps, steps[1:])):
            raise RuntimeError(f"batched clients: the slabs must hold the clients in non-increasing order of steps "
                               f"per epoch (models/batched.py slab_order), got {steps}")
        self.arena.freeze()
        if self.device.type == "cuda":
            from ..utils.devsync import device_sync
            device_sync(self.device)
        self._frozen = True

    def steps(self) -> List[int]:
        """Steps per epoch of every slab's client."""
        return [int(e.steps_per_epoch) for e in self.engines]

    def state_tensors(self) -> List[torch.Tensor]:
        """Every client's persistent training state (the capture warm-up snapshot)."""
        out = []
        for e in self.engines:
            out += [e.flat, e.mG, e.vG, e.mD, e.vD, e.stepG, e.stepD, e.ops.ctr]
        return out

    # ------------------------------------------------------------------ training
    def _batched(self, k: int | None = None):
        e0 = self.engines[0]
        a = self.arena
        return _BatchContext(e0.ops, self.k if k is None else int(k), a.stride, a.base, a)

    def train_steps(self, n: int, use_graph: bool | None = None, clients: int | None = None) -> None:
        """n steps of the first ``clients`` slabs' clients (default: all), each launch of a step issued
        once for all of them."""
        self.freeze()
        k = self.k if clients is None else int(clients)
        e0 = self.engines[0]
        b0 = e0.bn_batches
        with self._batched(k):
            e0.train_steps(n, use_graph)
        for e in self.engines[1:k]:
            e.bn_batches += e0.bn_batches - b0

    def _segments(self):
        """(clients, steps) of an epoch's launch segments (see train_epoch)."""
        steps, done, out = self.steps(), 0, []
        for k in range(self.k, 0, -1):
            n = steps[k - 1] - done
            if n > 0:
                out.append((k, n))
                done += n
        return out

    def prepare(self, use_graph: bool | None = None) -> None:
        """Freeze the arena and capture every step graph an epoch replays (the capture's warm-up step also
        sizes the lazily allocated operands, so an arena that is too small fails here, not mid-round)."""
        self.freeze()
        e0 = self.engines[0]
        if use_graph is None:
            use_graph = self.device.type == "cuda"
        if not use_graph:
            return
        U = max(1, int(e0.cfg.graph_unroll))
        for k, n in self._segments():
            with self._batched(k):
                if n >= U and e0._graph_key(U) not in e0.graphs:
                    e0._capture(U)
                if n % U and e0._graph_key(1) not in e0.graphs:
                    e0._capture(1)

    def train_epoch(self, use_graph: bool | None = None) -> None:
        """One local epoch of every client: ``steps_per_epoch`` of its own (the reference's
        ``len(train) // batch_size``).  Segment j runs the steps that the first k_j slabs' clients still
        have, k_j falling as clients finish; graphs are captured per (steps, k)."""
        self.freeze()
        for k, n in self._segments():
            self.train_steps(n, use_graph, clients=k)

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

    def slab_weights(self, client_weights: Sequence[float]) -> List[float]:
        """Per-client weights (client order) -> per-slab weights (slab order)."""
        return [float(client_weights[c]) for c in self.client_of_slab]

    def weighted_sum(self, weights: Sequence[float]) -> torch.Tensor:
        """sum_s w_s theta_s over the slabs (weights in slab order), on the current stream."""
        w = torch.as_tensor(np.asarray(weights, dtype=np.float32), device=self.device)
        F = self.flats()
        return torch.mv(F.t(), w) if self.k > 1 else F[0] * w[0]

    def set_all(self, agg: torch.Tensor) -> None:
        """Every client's flat buffer <- agg (on the current stream)."""
        F = self.flats()
        F.copy_(agg.unsqueeze(0).expand_as(F))

    def weighted_average(self, weights: Sequence[float]) -> None:
        """FedAvg of every client's parameters and BN statistics (`Server/dtds/distributed.py:86-106`):
        every client ends holding sum_c w_c theta_c (weights in slab order).  Runs on the current stream,
        no host sync."""
        self.set_all(self.weighted_sum(weights))


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
