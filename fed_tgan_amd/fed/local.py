"""Single-process multi-client emulation (``-local_clients K``).

A ``gpurun`` box exposes one MI355X and RCCL forbids two ranks on one device, so the
federation logic (init protocol, weighted aggregation, fault injection, sampling) is also run
with K clients as K threads of one process sharing one GPU.  ``ThreadComm`` implements the
:class:`~fed_tgan_amd.parallel.comm.Comm` collectives with a barrier and shared slots; the
aggregation sums the clients' pre-scaled device buffers on the GPU.  Graph capture uses the
thread-local capture mode so every client captures and replays its own step graph.
"""
from __future__ import annotations

import contextlib
import threading
import traceback
from typing import Any, List, Optional

import torch

from ..parallel.comm import Comm
from ..utils.devsync import device_sync


class LocalGroup:
    def __init__(self, k: int):
        self.k = k
        self.barrier = threading.Barrier(k)
        self.slots: List[Any] = [None] * k
        self.result: Any = None
        self.failed = threading.Event()

    def wait(self):
        if self.failed.is_set():
            raise RuntimeError("another emulated client failed")
        try:
            self.barrier.wait(timeout=3600)
        except threading.BrokenBarrierError:
            raise RuntimeError("emulated federation aborted")


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
        if self.rank == src:
            self.g.result = t.detach().clone()
        self.g.wait()
        if self.rank != src:
            t.copy_(self.g.result)
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
        # (threads share host memory: the rows always come back as host tensors)
        parts = self.all_gather_object(t.cpu())
        if self.rank != dst:
            return None
        return torch.cat([parts[r][:n] for r, n in zip(ranks, counts)])

    def gather_bytes(self, payload, dst: int = 0):
        out = self.all_gather_object(payload)
        return out if self.rank == dst else None

    def destroy(self):
        pass

    def weighted_all_reduce(self, flat, weight: float):
        """sum_i w_i * flat_i: every rank posts (buffer, weight); rank 0 accumulates on the device."""
        if flat.is_cuda:
            device_sync(flat.device)
        self.g.slots[self.rank] = (flat, float(weight))
        self.g.wait()
        if self.rank == 0:
            acc = torch.zeros_like(flat)
            for buf, w in self.g.slots:
                if w != 0.0:
                    acc.add_(buf, alpha=w)
            if flat.is_cuda:
                device_sync(flat.device)
            self.g.result = acc
        self.g.wait()
        flat.copy_(self.g.result)
        if flat.is_cuda:
            device_sync(flat.device)
        self.g.wait()
        return flat


def run_local_emulation(cfg, k: int, backend: str = "auto", device: Optional[torch.device] = None):
    """Run a K-client federation in one process; returns the federator's runtime (rank 0)."""
    from .runtime import FedRuntime
    if device is None:
        device = torch.device("cuda", 0) if (torch.cuda.is_available() and backend != "torch") else torch.device("cpu")
    cfg.backend = backend
    group = LocalGroup(k)
    runtimes: List[Optional[FedRuntime]] = [None] * k
    errors: List[BaseException] = []

    def worker(rank: int):
        try:
            stream_ctx = contextlib.nullcontext()
            if device.type == "cuda":
                torch.cuda.set_device(device)
                # one HIP stream per emulated client: the clients' small step kernels (a few dozen
                # workgroups each) run concurrently on the 256 CUs instead of queueing on one stream
                if getattr(cfg, "client_streams", True):
                    stream_ctx = torch.cuda.stream(torch.cuda.Stream(device))
            with stream_ctx:
                comm = ThreadComm(group, rank, device)
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

    threads = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(k)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise RuntimeError(f"local emulation failed: {errors[0]!r}")
    return runtimes[0]
