"""Native RCCL data plane (``csrc/comm/rccl_comm.cpp``): the round's weight all-reduce issued from C++ on the
caller's HIP stream, outside torch.distributed's ProcessGroup.

The reference aggregates by pulling every client's state dict over RPC and pushing the weighted average back
(`Server/dtds/distributed.py:794-823`).  Here the client ranks form one RCCL communicator and the aggregate is one
in-place all-reduce of the flat parameter buffer with the client weight folded in (pre-multiplied sum).  Through
this plane the collective is a plain stream operation: it can be captured into a hipGraph with the device work
around it, and it carries no ProcessGroup work object, watchdog or stream hand-off.  It uses the RCCL library torch
already loaded (one RCCL instance per process).

``Comm(native_rccl=True)`` (or ``FEDTGAN_NATIVE_RCCL=1``) routes ``weighted_all_reduce`` through it; the gathers and
the control plane stay on torch.distributed.
"""
from __future__ import annotations

import os
from typing import Callable, Optional

import torch


def _lib():
    from ..ops import native
    return native.require()


def rccl_library_path() -> str:
    return os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")


class NativeRccl:
    """One RCCL communicator over ``nranks`` ranks of this process group.

    share_id: called on every rank (with None) and returns rank 0's unique id, which the caller generated and
    distributed over the control plane (the ids must reach every member before any member initialises)."""

    def __init__(self, rank: int, nranks: int, device: torch.device,
                 share_id: Optional[Callable[[Optional[torch.Tensor]], torch.Tensor]] = None):
        L = _lib()
        L.rccl_load(rccl_library_path())
        # (each ncclGetUniqueId starts a bootstrap root -- a listening socket and a thread -- so an id is only
        # generated here when no caller shares one: a one-rank communicator without a control plane)
        if share_id is not None:
            uid = share_id(None)
        elif nranks != 1:
            raise ValueError("NativeRccl over several ranks needs share_id (the control plane's broadcast)")
        else:
            uid = L.rccl_unique_id()
        torch.cuda.set_device(device)
        self.rank, self.nranks, self.device = rank, nranks, device
        self.handle = int(L.rccl_init(uid.contiguous(), int(rank), int(nranks)))

    def all_reduce(self, t: torch.Tensor, weight: float = 1.0) -> torch.Tensor:
        """t <- sum over ranks of weight_rank * t_rank, in place, on the current stream."""
        _lib().rccl_all_reduce(self.handle, t, float(weight))
        return t

    def destroy(self):
        if self.handle is not None:
            _lib().rccl_destroy(self.handle)
            self.handle = None
