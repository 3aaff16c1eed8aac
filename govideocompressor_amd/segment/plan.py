"""Segment planning: how a clip is cut into independent closed-GOP pieces.

Two planners:

* :func:`reference_segment_seconds` -- the reference's size -> time heuristic
  (server.go:54-58) with its exact integer arithmetic::

      fileMiB     = size_bytes / 1024 / 1024          (integer)
      secondTime  = GetSumTime(file)                  (whole seconds + 1)
      segmentTime = sizeMB * secondTime / fileMiB     (integer)

  The reference divides by zero for files under 1 MiB (defect D1); here the
  divisor is clamped to 1 and the result to >= 1 second.

* :func:`balanced_plan` -- the MI355X plan for raw input, where a size target
  is meaningless (10 MB is ~3 frames of 1080p): equal GOP-aligned frame ranges,
  ``n_seg`` a multiple of ``world * slots`` so every GPU holds the same number of
  batch slots, optionally weighted by lowres complexity (est_cost) so that
  dynamic tickets hand out the expensive segments first.

A plan is an int64 array ``[n_seg, 3] = (start_frame, n_frames, est_cost)``
(SURVEY.md K-B), which is what rank 0 broadcasts (CC-4).
"""
from __future__ import annotations

import math
import re

import numpy as np


def reference_segment_seconds(size_mb: int, duration_plus1_s: int, file_bytes: int) -> int:
    file_mib = max(1, file_bytes // 1024 // 1024)   # D1 fixed: no division by zero
    return max(1, (size_mb * duration_plus1_s) // file_mib)


def frames_for_seconds(seconds: float, fps: float) -> int:
    return max(1, int(round(seconds * fps)))


def fixed_plan(n_frames: int, seg_frames: int) -> np.ndarray:
    """Cut every ``seg_frames`` frames (the last piece may be shorter)."""
    if n_frames <= 0:
        return np.zeros((0, 3), dtype=np.int64)
    seg_frames = max(1, int(seg_frames))
    starts = np.arange(0, n_frames, seg_frames, dtype=np.int64)
    counts = np.minimum(seg_frames, n_frames - starts)
    return np.stack([starts, counts, counts], axis=1)


def balanced_plan(n_frames: int, world: int = 1, per_rank: int = 4, min_frames: int = 8,
                  max_frames: int | None = None, gop: int | None = None) -> np.ndarray:
    """``n_seg ~= per_rank * world`` near-equal segments (lengths differ by <= 1 GOP unit).

    ``gop``: segment boundaries are multiples of it (keyframe grid).  ``max_frames`` caps a
    segment's length (more segments then)."""
    if n_frames <= 0:
        return np.zeros((0, 3), dtype=np.int64)
    unit = max(1, int(gop or 1))
    units = math.ceil(n_frames / unit)
    n_seg = max(1, world * per_rank)
    n_seg = min(n_seg, max(1, n_frames // max(1, min_frames)), units)
    if max_frames:
        n_seg = max(n_seg, math.ceil(n_frames / max_frames))
    n_seg = max(1, min(n_seg, units))
    base, extra = divmod(units, n_seg)
    out = []
    f = 0
    for i in range(n_seg):
        c = min((base + (1 if i < extra else 0)) * unit, n_frames - f)
        if c <= 0:
            break
        out.append((f, c, c))
        f += c
    return np.array(out, dtype=np.int64)


def weight_plan(plan: np.ndarray, frame_costs: np.ndarray) -> np.ndarray:
    """Replace est_cost with the summed lowres cost of each segment (scaled to int64)."""
    p = plan.copy()
    cs = np.concatenate([[0.0], np.cumsum(np.asarray(frame_costs, dtype=np.float64))])
    for i, (s, c, _) in enumerate(plan):
        p[i, 2] = int(round(cs[s + c] - cs[s]))
    return p


def shard(plan: np.ndarray, rank: int, world: int, by_cost: bool = False) -> list[int]:
    """Static assignment of segment indices to a rank.

    Round-robin by default; ``by_cost`` runs longest-processing-time-first greedy so each
    rank's summed est_cost is balanced."""
    n = len(plan)
    if not by_cost:
        return list(range(rank, n, world))
    order = np.argsort(-plan[:, 2], kind="stable")
    load = [0] * world
    owner = [0] * n
    for i in order:
        r = int(np.argmin(load))
        owner[int(i)] = r
        load[r] += int(plan[int(i), 2])
    return [i for i in range(n) if owner[i] == rank]


def parse_pieces(spec: str) -> list[str]:
    """``-p "3;7"`` -> ["3", "7"] (server.go:73-86).

    Every token must parse as an integer (the reference's ``strconv.Atoi``; otherwise
    "输入参数错误" / bad input argument, server.go:77-79) but is kept verbatim, so
    ``-p 03`` addresses piece ``03``.  Order is preserved (the dispatcher hands out
    the LAST token first, as JobAlloc walks initMap downwards); duplicates collapse,
    as they do in the reference's remainMap."""
    out: list[str] = []
    seen: set[int] = set()
    for t in spec.split(";"):
        if not re.fullmatch(r"[+-]?[0-9]+", t):
            raise ValueError(f"bad input argument [{spec}]")
        v = int(t)
        if v not in seen:
            seen.add(v)
            out.append(t)
    return out
