"""Several clients per process (``-local_clients K``).

RCCL allows one rank per device, so more clients than GPUs run as threads: K clients are K
threads of one process sharing its GPU, each with its own HIP stream and its own captured step
graph (thread-local capture mode).

* ``ThreadComm`` -- one process, K clients: the :class:`~fed_tgan_amd.parallel.comm.Comm`
  collectives over a thread barrier and shared slots; the aggregation sums the clients'
  pre-scaled device buffers on the GPU.
* ``HierComm`` -- N processes (one per GPU, ``-world_size N -local_clients K``), K clients each:
  N*K clients in all, client ``r*K + t`` being thread ``t`` of rank ``r``.  Every collective is
  two-level: the threads of a process combine on their shared GPU, thread 0 runs the process-level
  collective (RCCL all-reduce / gather over xGMI, gloo for the control plane) on the combined
  value, and the threads pick the result up.  One RCCL all-reduce per process per round instead of
  one per client.
"""
from __future__ import annotations

import contextlib
import threading
import traceback
from typing import Any, List, Optional

import torch

from ..parallel.comm import Comm


class LocalGroup:
    def __init__(self, k: int):
        self.k = k
        self.barrier = threading.Barrier(k)
        self.slots: List[Any] = [None] * k
        self.result: Any = None
        self.failed = threading.Event()
        # the batched multi-client engine of this process' clients (models/batched.py), if they use one:
        # thread 0 then issues every client's training steps, the FedAvg and the generation
        self.batch = None
        self.lock = threading.Lock()
        self._acc = None

    def reduce_buffer(self, like: torch.Tensor) -> torch.Tensor:
        """The accumulator of ``stream_reduce`` (kept across rounds: the other threads' streams read it
        after the host has moved on, so it must never return to the caching allocator mid-round)."""
        if self._acc is None or self._acc.shape != like.shape or self._acc.device != like.device:
            self._acc = torch.empty_like(like)
        return self._acc

    def local_all(self, t: int, ok: bool) -> bool:
        """Host-side AND of a flag over the group's threads (collective)."""
        self.slots[t] = bool(ok)
        self.wait()
        out = all(self.slots)
        self.wait()
        return out

    def wait(self):
        if self.failed.is_set():
            raise RuntimeError("another emulated client failed")
        try:
            self.barrier.wait(timeout=3600)
        except threading.BrokenBarrierError:
            raise RuntimeError("emulated federation aborted")


def _stream_event(t: torch.Tensor):
    """An event recorded on the current stream of ``t``'s device (None for a host tensor)."""
    if not t.is_cuda:
        return None
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(t.device))
    return ev


def stream_reduce(g: LocalGroup, t: int, flat: torch.Tensor, weight: float, outer=None) -> torch.Tensor:
    """sum_i w_i * flat_i over the threads of ``g``; every thread ends holding the sum in ``flat``.

    The threads' HIP streams are ordered by events, exchanged at host barriers: thread i records an
    event once its ``flat`` is final; thread 0's stream waits for every one of them, accumulates into a
    buffer kept by the group, runs ``outer(acc)`` (HierComm: the process-level all-reduce), and records
    a done event; every thread's stream waits for that event and copies the sum.  The host never waits
    for the device, and the clients' kernels keep running while the host exchanges events (the thread
    path used to synchronise the whole device three times per round)."""
    g.slots[t] = (flat, float(weight), _stream_event(flat))
    g.wait()
    if t == 0:
        parts = list(g.slots)
        if flat.is_cuda:
            cur = torch.cuda.current_stream(flat.device)
            for _, _, ev in parts:
                if ev is not None:
                    cur.wait_event(ev)
        acc = g.reduce_buffer(flat)
        acc.zero_()
        for buf, w, _ in parts:
            if w != 0.0:
                acc.add_(buf, alpha=w)
        if outer is not None:
            outer(acc)
        g.result = (acc, _stream_event(acc))
    g.wait()
    acc, done = g.result
    if t != 0 and done is not None:
        torch.cuda.current_stream(flat.device).wait_event(done)
    flat.copy_(acc)
    g.wait()        # g.result stays valid until every thread has read it
    return flat


class ThreadComm(Comm):
    def __init__(self, group: LocalGroup, rank: int, device: torch.device):
        super().__init__(rank, group.k, list(range(group.k)), "local", device=device, init=False)
        self.g = group

    def all_gather_object(self, obj):
        self.g.slots[self.rank] = obj
        self.g.wait()
        out = list(self.g.slots)
        self.g.wait()
        return out

    def broadcast_object(self, obj, src: int = 0):
        if self.rank == src:
            self.g.result = obj
        self.g.wait()
        out = self.g.result
        self.g.wait()
        return out

    def barrier(self):
        self.g.wait()

    def broadcast_tensor(self, t, src: int = 0):
        # the source's copy is made on its stream: the readers' streams wait for it (event), not the host
        if self.rank == src:
            c = t.detach().clone()
            self.g.result = (c, _stream_event(c))
        self.g.wait()
        if self.rank != src:
            c, ev = self.g.result
            if ev is not None:
                torch.cuda.current_stream(t.device).wait_event(ev)
            t.copy_(c)
            done = _stream_event(t)
        else:
            done = None
        self.g.slots[self.rank] = done
        self.g.wait()
        if self.rank == src and t.is_cuda:   # the copy stays alive until every reader's stream has read it
            cur = torch.cuda.current_stream(t.device)
            for ev in self.g.slots:
                if ev is not None:
                    cur.wait_event(ev)
        self.g.wait()
        return t

    def all_reduce_cpu(self, t, op=None):
        self.g.slots[self.rank] = t.detach().clone()
        self.g.wait()
        total = self.g.slots[0].clone()
        for x in self.g.slots[1:]:
            total += x
        self.g.wait()
        t.copy_(total)
        return t

    def max_float(self, x: float) -> float:
        return max(self.all_gather_object(float(x)))

    def heartbeat(self, timeout_s: float):
        self.g.wait()

    def gather_rows(self, t, counts, ranks, dst: int = 0, to_host: bool = True):
        """The threads' row blocks concatenated on ``dst``'s stream: ``dst`` waits for each thread's rows
        through an event (no host synchronisation), marks them in use by its stream (they are freed by
        their own threads later), and copies the result to the host once if ``to_host``."""
        self.g.slots[self.rank] = (t, _stream_event(t))
        self.g.wait()
        out = None
        if self.rank == dst:
            parts = list(self.g.slots)
            if t.is_cuda:
                cur = torch.cuda.current_stream(t.device)
                for p, ev in parts:
                    if ev is not None:
                        cur.wait_event(ev)
                    p.record_stream(cur)
            out = torch.cat([parts[r][0][:n] for r, n in zip(ranks, counts)])
            if to_host:
                out = out.cpu()
        self.g.wait()           # every thread keeps its rows referenced until dst has enqueued its reads
        return out

    def gather_bytes(self, payload, dst: int = 0):
        out = self.all_gather_object(payload)
        return out if self.rank == dst else None

    def destroy(self):
        pass

    def weighted_all_reduce(self, flat, weight: float):
        """sum_i w_i * flat_i: every rank posts (buffer, weight); rank 0 accumulates on the device.
        Batched clients (the buffers live in one arena): thread 0 reduces over the arena on its stream,
        the stream every client's training ran on -- no copies.  Otherwise the clients' streams are
        ordered by events (``stream_reduce``).  No host synchronisation with the device either way."""
        b = self.g.batch
        if b is not None and flat.is_cuda and b.owns(flat):
            self.g.slots[self.rank] = float(weight)
            self.g.wait()
            if self.rank == 0:
                b.weighted_average(b.slab_weights(list(self.g.slots)))
            self.g.wait()
            return flat
        return stream_reduce(self.g, self.rank, flat, weight)


class HierComm(Comm):
    """Client ``outer.rank * K + t`` of ``outer.world_size * K``: thread ``t`` of this process.

    Needs a co-located federation (every process runs clients; the federator is client 0, thread 0
    of rank 0).  Only thread 0 touches the process-level ``outer`` communicator."""

    def __init__(self, group: LocalGroup, thread: int, device: torch.device, outer: Comm):
        k = group.k
        n = outer.world_size
        if outer.client_ranks != list(range(n)):
            raise ValueError("several clients per process need every process to run clients (-colocated)")
        super().__init__(outer.rank * k + thread, n * k, list(range(n * k)), outer.data_backend, device=device,
                         init=False)
        self.g, self.t, self.k, self.outer = group, thread, k, outer
        self.dist_active = outer.dist_active

    def data_world_size(self) -> int:
        return self.outer.data_world_size() * self.k

    # ---- thread-level building blocks
    def _tgather(self, obj) -> list:
        self.g.slots[self.t] = obj
        self.g.wait()
        out = list(self.g.slots)
        self.g.wait()
        return out

    def _lead(self, fn):
        """Thread 0 computes fn() (a process-level collective); every thread returns its result."""
        if self.t == 0:
            self.g.result = fn()
        self.g.wait()
        out = self.g.result
        self.g.wait()
        return out

    # ---- control plane
    def all_gather_object(self, obj):
        local = self._tgather(obj)
        return self._lead(lambda: [x for part in self.outer.all_gather_object(local) for x in part])

    def broadcast_object(self, obj, src: int = 0):
        if self.t == src % self.k:
            self.g.result = obj
        self.g.wait()
        return self._lead(lambda: self.outer.broadcast_object(self.g.result, src=src // self.k))

    def barrier(self):
        self.g.wait()
        self._lead(lambda: self.outer.barrier())

    def heartbeat(self, timeout_s: float):
        self.g.wait()
        self._lead(lambda: self.outer.heartbeat(timeout_s))

    def broadcast_tensor(self, t, src: int = 0):
        """The source thread's copy is ordered to thread 0 and from thread 0 to every thread by stream
        events; the process-level broadcast stages the tensor through host memory (gloo), which waits for
        thread 0's stream only -- no device-wide synchronisation."""
        if self.t == src % self.k:
            c = t.detach().clone()
            self.g.result = (c, _stream_event(c))
        self.g.wait()
        shared = self.g.result
        self.g.wait()

        def bcast():
            c, ev = shared
            if ev is not None and self.t != src % self.k:
                torch.cuda.current_stream(t.device).wait_event(ev)
                c.record_stream(torch.cuda.current_stream(t.device))
            v = self.outer.broadcast_tensor(c, src=src // self.k)
            return v, _stream_event(v)
        v, ev = self._lead(bcast)
        if ev is not None and self.t != 0:
            torch.cuda.current_stream(t.device).wait_event(ev)
            v.record_stream(torch.cuda.current_stream(t.device))   # (allocated on the source thread's stream)
        t.copy_(v)
        done = self._tgather(_stream_event(t))
        if self.t == 0 and t.is_cuda:       # v stays alive until every thread's stream has read it
            cur = torch.cuda.current_stream(t.device)
            for e in done:
                if e is not None:
                    cur.wait_event(e)
        self.g.wait()
        return t

    def all_reduce_cpu(self, t, op=None):
        parts = self._tgather(t.detach().clone())

        def reduce():
            total = parts[0].clone()
            for x in parts[1:]:
                total += x
            return self.outer.all_reduce_cpu(total)
        t.copy_(self._lead(reduce))
        return t

    def max_float(self, x: float) -> float:
        m = max(self._tgather(float(x)))
        return self._lead(lambda: self.outer.max_float(m))

    def gather_bytes(self, payload, dst: int = 0):
        out = self.all_gather_object(payload)
        return out if self.rank == dst else None

    # ---- data plane
    def weighted_all_reduce(self, flat, weight: float):
        """sum_i w_i * flat_i: the process' clients are summed on its GPU by thread 0, which then
        runs ONE process-level all-reduce (weight 1: the terms are already scaled).  Batched clients:
        the local sum is one reduction over the arena (models/batched.py), the aggregate is copied into
        every slab; otherwise the threads' streams are ordered by events (``stream_reduce``)."""
        b = self.g.batch
        if b is not None and flat.is_cuda and b.owns(flat):
            self.g.slots[self.t] = float(weight)
            self.g.wait()
            if self.t == 0:
                agg = b.weighted_sum(b.slab_weights(list(self.g.slots)))
                self.outer.weighted_all_reduce(agg, 1.0)
                b.set_all(agg)
            self.g.wait()
            return flat
        return stream_reduce(self.g, self.t, flat, weight, outer=lambda acc: self.outer.weighted_all_reduce(acc, 1.0))

    def share_with_federator(self, flat, federator: int = 0, extra=None):
        return False        # co-located: the federator is a client and already holds the aggregate

    def gather_rows(self, t, counts, ranks, dst: int = 0, to_host: bool = True):
        """The process' client shares are concatenated on its GPU, then one process-level gather."""
        if list(ranks) != self.client_ranks:
            raise ValueError("HierComm.gather_rows gathers from every client, in client order")
        parts = self._tgather((t, _stream_event(t)))
        k, n = self.k, self.outer.world_size

        def gather():
            me = self.outer.rank
            if t.is_cuda:      # thread 0's stream waits for every thread's rows (events, no host sync)
                cur = torch.cuda.current_stream(t.device)
                for p, ev in parts:
                    if ev is not None:
                        cur.wait_event(ev)
                    p.record_stream(cur)     # freed by its thread later: not reused before this stream reads it
            local = torch.cat([p[:counts[me * k + i]] for i, (p, _) in enumerate(parts)])
            per = [sum(counts[q * k:(q + 1) * k]) for q in range(n)]
            return self.outer.gather_rows(local, per, list(range(n)), dst=dst // k, to_host=to_host)
        out = self._lead(gather)
        return out if self.rank == dst else None

    def init_p2p(self):
        raise NotImplementedError("MD-GAN split mode runs one client per process")

    def warmup(self, width: int = 4, dst: int = 0, gather: bool = True):
        self.g.wait()
        self._lead(lambda: self.outer.warmup(width, dst=dst // self.k, gather=gather))

    def destroy(self):
        pass        # the process-level communicator belongs to the caller


def run_local_emulation(cfg, k: int, backend: str = "auto", device: Optional[torch.device] = None,
                        outer: Optional[Comm] = None):
    """Run K clients as threads of this process; returns the runtime of the process' first client
    (the federator on rank 0).  With ``outer`` (a process-level Comm over N ranks) the threads are
    clients ``outer.rank*K .. outer.rank*K + K-1`` of an N*K-client federation (``HierComm``)."""
    from .runtime import FedRuntime
    if device is None:
        device = torch.device("cuda", 0) if (torch.cuda.is_available() and backend != "torch") else torch.device("cpu")
    cfg.backend = backend
    group = LocalGroup(k)
    runtimes: List[Optional[FedRuntime]] = [None] * k
    errors: List[BaseException] = []

    # one HIP stream per emulated client: the clients' small step kernels (a few dozen workgroups each) run
    # concurrently on the 256 CUs instead of queueing on one stream.  HIP maps streams onto its few hardware queues
    # (GPU_MAX_HW_QUEUES, 4) round-robin in creation order, and a hardware queue runs its streams' kernels in
    # order: the K client streams are created here, back to back, so they spread evenly (8 clients: 2 per queue).
    # Created inside the threads they interleaved with each engine's capture / lane streams -- measured, 3 clients
    # on one queue and 1 on another, 72 ms rounds for 8 clients (profiles/multiclient_r5.txt).
    client_streams = None
    if device.type == "cuda" and getattr(cfg, "client_streams", True):
        torch.cuda.set_device(device)
        client_streams = [torch.cuda.Stream(device) for _ in range(k)]

    def worker(rank: int):
        try:
            stream_ctx = contextlib.nullcontext()
            if device.type == "cuda":
                torch.cuda.set_device(device)
                if client_streams is not None:
                    stream_ctx = torch.cuda.stream(client_streams[rank])
            with stream_ctx:
                comm = ThreadComm(group, rank, device) if outer is None else HierComm(group, rank, device, outer)
                rt = FedRuntime(cfg, comm, device, federator=0)
                rt.thread_local_capture = True
                runtimes[rank] = rt
                rt.initialize()
                rt.fit()
        except BaseException as e:  # pragma: no cover - surfaced below
            errors.append(e)
            traceback.print_exc()
            group.failed.set()
            group.barrier.abort()

    # CPU clients: K threads each running intra-op parallel torch ops would oversubscribe the cores
    # (measured: a 2-rank x 2-client CPU round 38 s with 4 intra-op threads per client, 1.3 s with 2)
    n_threads = torch.get_num_threads()
    if device.type == "cpu" and outer is None:
        torch.set_num_threads(max(1, n_threads // k))
    threads = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(k)]
    try:
        for t in threads:
            t.start()
        for t in threads:
            t.join()
    finally:
        torch.set_num_threads(n_threads)
    if errors:
        raise RuntimeError(f"local emulation failed: {errors[0]!r}")
    return runtimes[0]
