"""Preallocated device/host memory for the encode loop.

* :class:`EncoderPool` keeps batched encoders resident keyed by their geometry and
  batch width: an encoder owns all of its HBM state (source planes, ping-pong
  reconstructions, decision records, CAVLC buffers), so reusing it means the steady
  state allocates nothing.  LRU eviction bounds the resident set.
* :class:`PinnedPool` hands out page-locked host buffers by size class for H2D uploads
  of decoded/raw frames (``non_blocking`` copies need pinned memory).
"""
from __future__ import annotations

import collections
import threading


class EncoderPool:
    def __init__(self, factory, max_resident: int = 2):
        self.factory = factory
        self.max_resident = max_resident
        self._lru: collections.OrderedDict = collections.OrderedDict()
        self._lock = threading.Lock()

    def get(self, key, *args, **kw):
        with self._lock:
            enc = self._lru.pop(key, None)
            if enc is None:
                while len(self._lru) >= self.max_resident:
                    _, old = self._lru.popitem(last=False)
                    close = getattr(old, "close", None)
                    if close:
                        close()
                enc = self.factory(*args, **kw)
            self._lru[key] = enc
            return enc

    def __len__(self):
        return len(self._lru)

    def close(self):
        with self._lock:
            for enc in self._lru.values():
                close = getattr(enc, "close", None)
                if close:
                    close()
            self._lru.clear()


class PinnedPool:
    """Pinned uint8 host buffers rounded up to powers of two; ``get(n)`` -> 1-D tensor view of n bytes."""

    def __init__(self, max_cached: int = 8):
        self.max_cached = max_cached
        self._free: dict[int, list] = collections.defaultdict(list)
        self._lock = threading.Lock()

    @staticmethod
    def _cls(n: int) -> int:
        c = 1 << 20
        while c < n:
            c <<= 1
        return c

    def get(self, n: int):
        import torch
        c = self._cls(n)
        with self._lock:
            lst = self._free.get(c)
            buf = lst.pop() if lst else None
        if buf is None:
            buf = torch.empty(c, dtype=torch.uint8)
            if torch.cuda.is_available():
                buf = buf.pin_memory()
        return buf[:n]

    def put(self, t) -> None:
        base = t._base if t._base is not None else t
        c = base.numel()
        with self._lock:
            if sum(len(v) for v in self._free.values()) < self.max_cached:
                self._free[c].append(base)
