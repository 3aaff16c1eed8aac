"""Per-stage timers and roctx ranges.

* :class:`StageTimer` -- host wall-clock accumulation per named stage.
* :class:`EventTimer` -- HIP-event timing of device work per stage on the current
  stream; events are resolved lazily (``summary()`` synchronises once), so timing
  adds no host stalls inside the encode loop.
* ``range_push/range_pop/nvtx_range`` -- roctx ranges (``torch.cuda.nvtx`` maps to
  roctx on ROCm builds) that show up in ``rocprofv3 --marker-trace`` timelines; no-ops
  without a GPU.
"""
from __future__ import annotations

import contextlib
import time
from collections import defaultdict


class StageTimer:
    def __init__(self):
        self.total = defaultdict(float)
        self.count = defaultdict(int)

    @contextlib.contextmanager
    def __call__(self, stage: str):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.total[stage] += time.perf_counter() - t0
            self.count[stage] += 1

    def add(self, stage: str, seconds: float):
        self.total[stage] += seconds
        self.count[stage] += 1

    def summary(self) -> dict:
        return {k: {"s": round(v, 6), "n": self.count[k]} for k, v in self.total.items()}


class EventTimer:
    def __init__(self, enabled: bool = True):
        self.enabled = enabled
        self.pending: list[tuple[str, object, object]] = []
        self.total = defaultdict(float)
        self.count = defaultdict(int)

    @contextlib.contextmanager
    def __call__(self, stage: str):
        if not self.enabled:
            yield
            return
        import torch
        if not torch.cuda.is_available():
            yield
            return
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        torch.cuda.nvtx.range_push(stage)  # roctx range for rocprofv3 --marker-trace
        try:
            yield
        finally:
            torch.cuda.nvtx.range_pop()
            b.record()
            self.pending.append((stage, a, b))

    def resolve(self):
        if not self.pending:
            return
        import torch
        torch.cuda.synchronize()
        for stage, a, b in self.pending:
            self.total[stage] += a.elapsed_time(b) / 1000.0
            self.count[stage] += 1
        self.pending.clear()

    def summary(self) -> dict:
        self.resolve()
        return {k: {"s": round(v, 6), "n": self.count[k]} for k, v in self.total.items()}

    def reset(self) -> None:
        self.resolve()
        self.total.clear()
        self.count.clear()


def _nvtx():
    try:
        import torch
        if torch.cuda.is_available():
            return torch.cuda.nvtx
    except Exception:  # noqa: BLE001
        pass
    return None


def range_push(name: str) -> None:
    n = _nvtx()
    if n is not None:
        n.range_push(name)


def range_pop() -> None:
    n = _nvtx()
    if n is not None:
        n.range_pop()


@contextlib.contextmanager
def nvtx_range(name: str):
    range_push(name)
    try:
        yield
    finally:
        range_pop()
