"""Bitrate targeting for the job API: ``-b:v`` (ABR), ``-pass 1/2`` and VBV.

The reference forwards raw ffmpeg arguments to every worker (``-f`` flag,
server.go:23-31; split on spaces at client.go:105), so ``-b:v 2M``, ``-pass 2`` and
``-maxrate/-bufsize`` reach libx264/libx265 there.  A batched GPU encoder re-encodes
a whole batch in milliseconds per frame, so instead of x264's one-pass predictor this
module drives the lookahead-CRF encoder with a *global QP offset* per rate group (one
piece, or -- in ``mivc encode`` -- the whole file, all-reduced over ranks, CC-1) and
solves ``bits(offset) = target`` by the secant method on log2(bits):

* pass A encodes at the rate factor of CRF 23 (or reads the ``-pass 1`` stats file);
* the model ``bits(d) = bits_A * 2^(-e d / 6)`` (e = 1, refined from two passes and
  clamped to [0.4, 2.5]) proposes the next offset; fractional offsets reach the frame
  QPs through ordered dithering (:func:`apply_delta`), so bits move smoothly with d;
* at most ``max_passes`` encodes; the pass closest to the target is kept.

VBV (``-maxrate``/``-bufsize``, x264 ``--vbv-init 0.9``): the final pass is simulated
as a leaky bucket in coding order; frames that would underflow get a QP increase sized
by the same bits model (:func:`vbv_deltas`) and the batch is encoded once more.

The ``-pass 1`` stats file (JSON) holds, per rate group, the pass-A bits and the offset
it was encoded at; ``-pass 2`` starts its search from it and skips pass A.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass, field

import numpy as np

GOLDEN = 0.6180339887498949


def apply_delta(qps: np.ndarray, delta) -> np.ndarray:
    """Integer QPs + float offsets [B, F] (or [B] / scalar), ordered dithering along F."""
    q = np.asarray(qps, dtype=np.float64)
    B, F = q.shape
    d = np.asarray(delta, dtype=np.float64)
    d = np.broadcast_to(d[:, None] if d.ndim == 1 else d, (B, F))
    r = (np.arange(F) * GOLDEN) % 1.0
    return np.clip(np.floor(q + d + r[None, :]), 0, 51).astype(np.int32)


@dataclass
class OffsetSearch:
    """Per-group secant search for the QP offset that makes bits == target."""
    targets: np.ndarray                 # [G] bits
    tol: float = 0.02
    max_passes: int = 4
    exponent: float = 1.0
    hist: list = field(default_factory=list)   # [(offsets [G], bits [G])]

    def __post_init__(self):
        self.targets = np.asarray(self.targets, dtype=np.float64)

    def observe(self, offsets, bits):
        self.hist.append((np.asarray(offsets, dtype=np.float64).copy(), np.asarray(bits, dtype=np.float64).copy()))

    def error(self, k: int = -1) -> np.ndarray:
        _, b = self.hist[k]
        return b / np.maximum(self.targets, 1.0) - 1.0

    def done(self) -> bool:
        if not self.hist:
            return False
        return len(self.hist) >= self.max_passes or bool(np.all(np.abs(self.error()) <= self.tol))

    def propose(self) -> np.ndarray:
        d1, b1 = self.hist[-1]
        e = np.full_like(d1, self.exponent)
        if len(self.hist) >= 2:
            d0, b0 = self.hist[-2]
            ok = (np.abs(d1 - d0) > 0.2) & (b0 > 0) & (b1 > 0)
            est = np.where(ok, -6.0 * np.log2(np.maximum(b1, 1) / np.maximum(b0, 1)) / np.where(ok, d1 - d0, 1.0), e)
            e = np.clip(est, 0.4, 2.5)
        step = -6.0 / e * np.log2(np.maximum(self.targets, 1.0) / np.maximum(b1, 1.0))
        return np.clip(d1 + step, -30.0, 30.0)

    def best(self) -> int:
        errs = [np.mean(np.abs(b / np.maximum(self.targets, 1.0) - 1.0)) for _, b in self.hist]
        return int(np.argmin(errs))

    def best_per_group(self) -> np.ndarray:
        """[G] index of the pass closest to each group's target."""
        e = np.stack([np.abs(b / np.maximum(self.targets, 1.0) - 1.0) for _, b in self.hist])
        return np.argmin(e, axis=0)


# ---------------------------------------------------------------------- VBV
def vbv_fill(frame_bits, maxrate: float, bufsize: float, fps: float, init: float = 0.9) -> np.ndarray:
    """Leaky-bucket decoder buffer (bits) after removing each frame, coding order; a
    negative value is an underflow (the frame arrives late)."""
    fill = init * bufsize
    per = maxrate / fps
    out = np.empty(len(frame_bits))
    for i, b in enumerate(frame_bits):
        fill -= float(b)
        out[i] = fill
        fill = min(fill + per, bufsize)
    return out


def vbv_deltas(frame_bits, maxrate: float, bufsize: float, fps: float, init: float = 0.9, exponent: float = 1.0,
               margin: float = 0.1) -> np.ndarray:
    """QP increases (coding order) that keep the predicted buffer non-negative: each frame
    that would underflow is cut to the bits available (less ``margin``); when one frame
    cannot absorb it (>= 12 QP) the preceding frames share the rest."""
    bits = np.asarray(frame_bits, dtype=np.float64).copy()
    dq = np.zeros(len(bits))
    per = maxrate / fps
    for _ in range(4):
        fill = init * bufsize
        changed = False
        for i in range(len(bits)):
            if bits[i] > fill:
                want = max(fill * (1.0 - margin), 1.0)
                need = 6.0 / exponent * math.log2(bits[i] / want)
                add = min(need, 12.0 - dq[i])
                if add > 0:
                    dq[i] += add
                    bits[i] *= 2.0 ** (-exponent * add / 6.0)
                    changed = True
                rest = need - add
                j = i - 1
                while rest > 0 and j >= 0 and j > i - 8:  # spread over up to 7 earlier frames
                    a = min(rest, 6.0 - min(dq[j], 6.0))
                    if a > 0:
                        dq[j] += a
                        bits[j] *= 2.0 ** (-exponent * a / 6.0)
                        changed = True
                    rest -= max(a, 0.0)
                    j -= 1
            fill = min(fill - bits[i] + per, bufsize)
        if not changed:
            break
    return np.ceil(dq * 4.0) / 4.0


# ---------------------------------------------------------------------- stats file
def stats_path_for(out_path: str, passlogfile: str | None = None) -> str:
    """``-passlogfile PREFIX`` -> PREFIX-<piece>.mivc2pass.json; default: beside the piece output."""
    base = os.path.splitext(os.path.basename(out_path))[0]
    if passlogfile:
        return f"{passlogfile}-{base}.mivc2pass.json"
    return os.path.splitext(out_path)[0] + ".mivc2pass.json"


def save_stats(path: str, groups: dict[str, dict]) -> None:
    tmp = path + ".part"
    with open(tmp, "w") as f:
        json.dump({"version": 1, "groups": groups}, f)
    os.replace(tmp, path)


def load_stats(path: str) -> dict[str, dict]:
    with open(path) as f:
        d = json.load(f)
    if d.get("version") != 1:
        raise ValueError(f"{path}: unknown two-pass stats version")
    return d["groups"]
