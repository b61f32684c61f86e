"""Per-phase timers and a JSONL metrics log.

The reference keeps ad-hoc wall timers per round (`Server/dtds/distributed.py:790-829`) and
only writes the accumulated round time.  ``PhaseTimer`` records train / aggregate /
sample+dump phases (synchronised with the compute stream when a GPU is used) and ``MetricsLog`` appends one
JSON object per round (losses, weights, phase times) for observability.
"""
from __future__ import annotations

import contextlib
import json
import time
from typing import Dict

from .devsync import stream_sync


class PhaseTimer:
    def __init__(self, sync: bool = False):
        self.sync = sync
        self.totals: Dict[str, float] = {}
        self._last: Dict[str, float] = {}

    @contextlib.contextmanager
    def phase(self, name: str, device=None):
        if self.sync and device is not None and getattr(device, "type", "") == "cuda":
            stream_sync(device)
        t = time.perf_counter()
        try:
            yield
        finally:
            if self.sync and device is not None and getattr(device, "type", "") == "cuda":
                stream_sync(device)
            dt = time.perf_counter() - t
            self.totals[name] = self.totals.get(name, 0.0) + dt
            self._last[name] = dt

    def last(self) -> Dict[str, float]:
        return {f"t_{k}": v for k, v in self._last.items()}


class MetricsLog:
    def __init__(self, path: str):
        self.path = path
        open(path, "w").close()

    def write(self, record: dict):
        with open(self.path, "a") as f:
            f.write(json.dumps(record) + "\n")
