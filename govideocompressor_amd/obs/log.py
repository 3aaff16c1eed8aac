"""JSON-lines structured logger: one object per event with rank, stage and timings.

Human-readable parity lines (the reference's console strings)
stay on stdout through the coordinator's ``log`` callable; this logger is the
machine-readable channel next to them (``MIVC_LOG_JSON=path`` or ``-`` for stderr).
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time


class JsonLogger:
    def __init__(self, path: str | None = None, rank: int | None = None, component: str = ""):
        self.path = path
        self.rank = int(os.environ.get("RANK", "0")) if rank is None else rank
        self.component = component
        self._lock = threading.Lock()
        self._fh = None
        if path and path != "-":
            os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
            self._fh = open(path, "a", buffering=1)

    @property
    def enabled(self) -> bool:
        return self.path is not None

    def event(self, event: str, **fields) -> dict:
        rec = {"ts": round(time.time(), 6), "rank": self.rank, "component": self.component, "event": event}
        rec.update(fields)
        if self.path is None:
            return rec
        line = json.dumps(rec, default=_default)
        with self._lock:
            if self._fh is not None:
                self._fh.write(line + "\n")
            else:
                sys.stderr.write(line + "\n")
        return rec

    def close(self):
        if self._fh is not None:
            self._fh.close()
            self._fh = None


def _default(o):
    try:
        import numpy as np
        if isinstance(o, np.generic):
            return o.item()
        if isinstance(o, np.ndarray):
            return o.tolist()
    except ImportError:  # pragma: no cover
        pass
    return str(o)


_loggers: dict[str, JsonLogger] = {}


def get_logger(component: str = "") -> JsonLogger:
    """Process-wide logger configured by ``MIVC_LOG_JSON`` (unset: events are built, not written)."""
    lg = _loggers.get(component)
    if lg is None:
        lg = JsonLogger(os.environ.get("MIVC_LOG_JSON"), component=component)
        _loggers[component] = lg
    return lg
