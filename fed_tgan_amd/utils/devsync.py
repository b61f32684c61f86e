"""Device-wide synchronisation that is safe next to hipGraph captures in other threads.

The in-process multi-client emulation (fed/local.py) runs one engine per thread, and each
captures its step graph in ``thread_local`` mode.  HIP refuses a device-wide synchronize
while ANY stream of the device is capturing, so captures and device syncs are made mutually
exclusive with one process-wide lock (captures are one-off; syncs are per phase).
"""
from __future__ import annotations

import threading

import torch

CAPTURE_LOCK = threading.RLock()


def device_sync(device) -> None:
    if device is None or getattr(device, "type", "") != "cuda":
        return
    with CAPTURE_LOCK:
        torch.cuda.synchronize(device)


def stream_sync(device) -> None:
    """Wait for the current stream of ``device`` only: side streams (the asynchronous device-to-host
    copy of a generated table) keep running.  Allowed while another thread captures."""
    if device is None or getattr(device, "type", "") != "cuda":
        return
    torch.cuda.current_stream(device).synchronize()


class PendingHost:
    """A device tensor being copied to pinned host memory on a side stream; ``get()`` waits for the
    copy (from any thread) and returns the NumPy view."""

    def __init__(self, t: torch.Tensor, copy_stream: "torch.cuda.Stream"):
        cur = torch.cuda.current_stream(t.device)
        copy_stream.wait_stream(cur)
        self.host = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        with torch.cuda.stream(copy_stream):
            self.host.copy_(t, non_blocking=True)
            self.event = torch.cuda.Event()
            self.event.record(copy_stream)
        t.record_stream(copy_stream)     # the allocator must not hand t's memory out before the copy ends

    def get(self):
        self.event.synchronize()
        return self.host.numpy()

    @property
    def shape(self):
        return tuple(self.host.shape)
