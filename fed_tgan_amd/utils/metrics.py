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


_CPU_STAT = None


def cgroup_cpu_stat() -> Dict[str, int]:
    """The process cgroup's CPU accounting: usage and CFS-bandwidth throttling counters (cgroup v2
    ``cpu.stat``: usage_usec, nr_periods, nr_throttled, throttled_usec; v1 ``cpu.stat`` +
    ``cpuacct.usage``).  Empty where the file is absent.  A round whose host issue time jumps while
    ``throttled_usec`` grows was descheduled by the CPU quota, not slowed by the GPU."""
    global _CPU_STAT
    if _CPU_STAT is None:
        _CPU_STAT = ""
        for p in ("/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu,cpuacct/cpu.stat", "/sys/fs/cgroup/cpu/cpu.stat"):
            try:
                with open(p):
                    _CPU_STAT = p
                    break
            except OSError:
                continue
    if not _CPU_STAT:
        return {}
    out: Dict[str, int] = {}
    try:
        with open(_CPU_STAT) as f:
            for line in f:
                k, _, v = line.partition(" ")
                if v.strip().isdigit():
                    out[k] = int(v)
    except OSError:
        return {}
    if "throttled_time" in out and "throttled_usec" not in out:       # cgroup v1 (nanoseconds)
        out["throttled_usec"] = out["throttled_time"] // 1000
    return out


def cpu_quota() -> Dict[str, float]:
    """CPU quota of the process cgroup (cgroup v2 ``cpu.max`` / v1 cfs files) and the affinity size."""
    import os
    info: Dict[str, float] = {"affinity": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else 0,
                              "cpu_count": os.cpu_count() or 0}
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                info["quota_cpus"] = int(q) / int(per)
                info["period_us"] = int(per)
    except (OSError, ValueError):
        pass
    return info


class MetricsLog:
    def __init__(self, path: str):
        self.path = path
        open(path, "w").close()

    def write(self, record: dict):
        with open(self.path, "a") as f:
            f.write(json.dumps(record) + "\n")
