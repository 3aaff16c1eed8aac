"""Observability: structured JSON-lines logging, per-stage
timers (host wall clock and HIP events), roctx ranges, and per-segment metrics.

The reference has none of this: ``fmt.Printf`` progress lines on the server
(server.go:183,286,298), a silenced worker (``printLog=false``, client.go:16) and an
uploaded ffmpeg stderr dump as the only per-job artefact (client.go:116-161).
"""
from .log import JsonLogger, get_logger
from .timers import EventTimer, StageTimer, range_push, range_pop, nvtx_range

__all__ = ["JsonLogger", "get_logger", "EventTimer", "StageTimer", "range_push", "range_pop", "nvtx_range"]
