"""Per-phase timing with HIP events (in-process timer per phase)."""
from __future__ import annotations

import json
import time
from collections import defaultdict
from contextlib import contextmanager

import torch


class GpuTimer:
    """Accumulates device time of named regions using HIP events (no host sync inside regions)."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self.pending = []
        self.totals = defaultdict(float)
        self.counts = defaultdict(int)

    @contextmanager
    def region(self, name: str):
        if not self.enabled:
            yield
            return
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        yield
        e.record()
        self.pending.append((name, s, e))

    def collect(self) -> dict:
        if self.pending:
            torch.cuda.synchronize()
        for name, s, e in self.pending:
            self.totals[name] += s.elapsed_time(e)
            self.counts[name] += 1
        self.pending.clear()
        return {k: {"ms_total": v, "count": self.counts[k], "ms_mean": v / max(1, self.counts[k])}
                for k, v in self.totals.items()}

    def dump(self, path: str) -> None:
        with open(path, "w") as fh:
            json.dump(self.collect(), fh, indent=1)


class PhaseTimer:
    """Host wall-clock phases."""

    def __init__(self):
        self.totals = defaultdict(float)

    @contextmanager
    def region(self, name: str):
        t = time.perf_counter()
        yield
        self.totals[name] += time.perf_counter() - t
