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
