"""Per-phase timers and a JSONL metrics log.

The reference keeps ad-hoc wall timers per round (`Server/dtds/distributed.py:790-829`) and
only writes the accumulated round time.  ``PhaseTimer`` records train / aggregate /
sample+dump phases (HIP events on a GPU: no host synchronisation) and ``MetricsLog`` appends one
JSON object per round (losses, weights, phase times) for observability.
"""
from __future__ import annotations

import contextlib
import json
import time
from typing import Dict, List

from .devsync import stream_sync


class PhaseTimer:
    """Accumulated time per named phase.

    events=True (GPU): each phase is bracketed by two HIP events on the current stream -- nothing
    waits for the device; the elapsed times are collected once the end events have completed
    (``resolve``, non-blocking unless asked).  sync=True: wall time with the current stream
    synchronised at both boundaries (the round-2 behaviour).  Otherwise plain host wall time."""

    def __init__(self, sync: bool = False, events: bool = False):
        self.sync = sync
        self.events = events
        self._totals: Dict[str, float] = {}
        self._last: Dict[str, float] = {}
        self._pending: List[tuple] = []

    @contextlib.contextmanager
    def phase(self, name: str, device=None):
        cuda = device is not None and getattr(device, "type", "") == "cuda"
        if self.events and cuda:
            import torch
            if len(self._pending) > 64:
                self.resolve()
            start = torch.cuda.Event(enable_timing=True)
            start.record()
            try:
                yield
            finally:
                end = torch.cuda.Event(enable_timing=True)
                end.record()
                self._pending.append((name, start, end))
            return
        if self.sync and cuda:
            stream_sync(device)
        t = time.perf_counter()
        try:
            yield
        finally:
            if self.sync and cuda:
                stream_sync(device)
            dt = time.perf_counter() - t
            self._add(name, dt)

    def _add(self, name: str, dt: float):
        self._totals[name] = self._totals.get(name, 0.0) + dt
        self._last[name] = dt

    def resolve(self, block: bool = False) -> None:
        """Fold completed event pairs into the totals (block: wait for the outstanding ones)."""
        keep = []
        for name, s, e in self._pending:
            if block:
                e.synchronize()
            elif not e.query():
                keep.append((name, s, e))
                continue
            self._add(name, s.elapsed_time(e) / 1e3)
        self._pending = keep

    @property
    def totals(self) -> Dict[str, float]:
        self.resolve(block=False)
        return self._totals

    def reset(self) -> None:
        """Forget every phase so far (pending event pairs included)."""
        self._pending = []
        self._totals = {}
        self._last = {}

    def last(self) -> Dict[str, float]:
        self.resolve(block=False)
        return {f"t_{k}": v for k, v in self._last.items()}


class MetricsLog:
    def __init__(self, path: str):
        self.path = path
        open(path, "w").close()

    def write(self, record: dict):
        with open(self.path, "a") as f:
            f.write(json.dumps(record) + "\n")
