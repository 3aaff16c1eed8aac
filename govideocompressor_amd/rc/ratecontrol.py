"""Rate control: CRF and two-pass average bitrate over closed-GOP segments.

Reference: the rate is whatever ``-crf`` / ``-b:v`` ffmpeg receives in the worker's
argument string (``-threads 4 -vcodec libx265 -crf 26`` / libx264's default CRF 23,
server.go:67-71); every segment is rate-controlled independently, so quality and
rate jump at segment boundaries.

Here:

* **CRF** (x264-style, without MB-tree): a frame's quantiser scale follows the
  blurred lowres complexity ``C`` of its frame type,
  ``qscale = C^(1-qcomp) / rate_factor``, ``rate_factor = base^(1-qcomp) / qp2qscale(crf)``,
  with ``qcomp = 0.6`` and the I/P offset of ``ipratio = 1.4`` (3 QP).
* **Two-pass ABR**: pass 1 measures per-frame bits at a fixed QP (or uses lowres
  complexity when no pass-1 encode is available).  The per-frame statistics of
  *all* segments of *all* ranks are summed into one global tensor with a single
  all-reduce (CC-1, RCCL over xGMI on a GPU node), so every rank solves the same
  global rate factor: the bitrate budget is shared across segment boundaries
  instead of being met segment by segment.

The model of bits versus quantiser is the standard ``bits ~ qscale^-1`` around the
pass-1 point; pass 2 re-solves it during the encode with the exponent measured on the
frames already coded (:class:`TwoPassFeedback`).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

QCOMP = 0.6
IP_OFFSET = 3          # I-frame QP = P QP - 3 (ipratio 1.4)
# x264 / x265 --pbratio 1.3 and --ipratio 1.4 as QP offsets (6 log2 ratio)
PB_OFFSET = 6.0 * math.log2(1.3)
IP_OFFSET_F = 6.0 * math.log2(1.4)


def crf_base_complexity(mb_count: int, bframes: int) -> float:
    """x264 / x265 CRF reference complexity: ``mb_count * (bframes ? 120 : 80)``.  With B
    pictures the anchors sit farther apart and cost more, so the constant grows with them;
    using 80 with B pictures on would code every frame ~1.4 QP coarser than the same CRF."""
    return float(mb_count) * (120.0 if int(bframes) > 0 else 80.0)
# x264 ratecontrol.c: with MB-tree the CRF constant is taken (1 - qcomp) * 13.5 QP higher;
# the (mostly negative) MB-tree offsets bring propagated blocks back down
MBTREE_CRF_OFFSET = (1.0 - QCOMP) * 13.5
MBTREE_STRENGTH = 5.0 * (1.0 - QCOMP)
QP_MIN, QP_MAX = 0, 51


def qp2qscale(qp: float) -> float:
    return 0.85 * 2.0 ** ((qp - 12.0) / 6.0)


def qscale2qp(q: float) -> float:
    return 12.0 + 6.0 * math.log2(max(q, 1e-9) / 0.85)


def clamp_qp(qp: float) -> int:
    return int(max(QP_MIN, min(QP_MAX, round(qp))))


@dataclass
class FrameStats:
    """Per-frame statistics of one segment: [n_frames, 4] = (cost_intra, cost_inter, bits, qp)."""
    data: np.ndarray

    @staticmethod
    def from_costs(intra, inter, bits=None, qp=None) -> "FrameStats":
        n = len(intra)
        d = np.zeros((n, 4), dtype=np.float64)
        d[:, 0] = intra
        d[:, 1] = inter
        if bits is not None:
            d[:, 2] = bits
        if qp is not None:
            d[:, 3] = qp
        return FrameStats(d)


def frame_complexity(intra: np.ndarray, inter: np.ndarray, keyint: int | None = None) -> np.ndarray:
    """Complexity used for frame f: intra cost for key frames, inter cost otherwise."""
    n = len(intra)
    c = np.array(inter, dtype=np.float64, copy=True)
    g = keyint if keyint and keyint > 0 else n
    c[::g] = np.asarray(intra, dtype=np.float64)[::g]
    return np.maximum(c, 1.0)


def crf_qps(intra: np.ndarray, inter: np.ndarray, crf: float, mb_count: int, keyint: int | None = None,
            blur: float = 0.5, bframes: int = 0) -> np.ndarray:
    """Per-frame QPs of a CRF encode of one segment (x264 rc_crf without MB-tree).

    ``mb_count`` = 16x16 macroblocks per frame; complexities are per frame lowres SATD
    sums (half-resolution 8x8 blocks: one per MB)."""
    cplx = frame_complexity(intra, inter, keyint)
    # temporal blur of the complexity (x264 keeps a decaying sum)
    blurred = np.empty_like(cplx)
    acc, w = 0.0, 0.0
    for i, c in enumerate(cplx):
        acc = acc * blur + c
        w = w * blur + 1.0
        blurred[i] = acc / w
    base = crf_base_complexity(mb_count, bframes)  # x264: complexity of a "typical" frame
    rate_factor = base ** (1.0 - QCOMP) / qp2qscale(crf)
    qs = blurred ** (1.0 - QCOMP) / rate_factor
    qp = np.array([qscale2qp(q) for q in qs])
    g = keyint if keyint and keyint > 0 else len(qp)
    qp[::g] -= IP_OFFSET
    return np.array([clamp_qp(q) for q in qp], dtype=np.int32)


def scenecut_flags(costs: np.ndarray, scenecut: float = 40.0, keyint: int | None = None,
                   keyint_max: int = 250, keyint_min: int | None = None) -> np.ndarray:
    """[B, F] scene-cut decisions from lowres frame costs (x264 ``--scenecut``, default 40).

    x264 (slicetype.c ``scenecut_internal``) flags frame t when its P cost from t - 1 is
    ``pcost >= (1 - bias) * icost`` (``cost_best = sum of per-block min(intra, inter)``,
    ``icost`` the intra sum), with a bias that grows with the distance from the last key
    frame: ``thresh_max = scenecut / 100``, ``thresh_min = thresh_max / 4``; up to
    keyint_min / 4 frames after a key frame ``bias = thresh_min / 4``, up to keyint_min
    ``thresh_min * gop / keyint_min``, then linear up to thresh_max at keyint_max.  So a cut
    right after a key frame needs the inter prediction to save almost nothing (x264's
    defaults: keyint 250, keyint_min = min(250 / 10, fps) = 25).  Key frames (frame 0, every
    ``keyint``-th) are not flagged; a flagged frame restarts the distance.  ``scenecut <= 0``
    disables detection."""
    c = np.asarray(costs, dtype=np.float64)
    B, F = c.shape[0], c.shape[1]
    flags = np.zeros((B, F), dtype=bool)
    if scenecut <= 0 or F < 2:
        return flags
    intra, best = c[:, :, 0], c[:, :, 1]
    tmax = scenecut / 100.0
    tmin = tmax * 0.25
    kmax = int(keyint) if keyint and keyint > 0 else int(keyint_max)
    kmin = int(keyint_min) if keyint_min else max(1, min(kmax // 10, 25))
    g = keyint if keyint and keyint > 0 else F
    last = np.zeros(B, dtype=np.int64)
    for t in range(1, F):
        if t % g == 0:
            last[:] = t
            continue
        gop = t - last
        bias = np.where(gop <= kmin / 4, tmin / 4,
                        np.where(gop <= kmin, tmin * gop / kmin,
                                 tmin + (tmax - tmin) * (gop - kmin) / max(1, kmax - kmin)))
        cut = best[:, t] >= (1.0 - bias) * np.maximum(intra[:, t], 1.0)
        flags[:, t] = cut
        last[cut] = t
    return flags


def crf_qps_batch(costs: np.ndarray, crf: float, mb_count: int, keyint: int | None = None, blur: float = 0.5,
                  qp_min: int = QP_MIN, qp_max: int = QP_MAX, scenecuts: np.ndarray | None = None,
                  mbtree: bool = False, bframes: int = 0) -> np.ndarray:
    """:func:`crf_qps` for B closed-GOP segments at once.

    ``costs``: [B, F, 2] lowres frame costs (intra, min(intra, inter)) as produced by
    :class:`~govideocompressor_amd.rc.lookahead.GpuLookahead`; frame 0 of each segment
    is the IDR (intra complexity, QP - IP_OFFSET), and so is every ``keyint``-th frame and
    every frame flagged in ``scenecuts`` ([B, F] bool, see :func:`scenecut_flags`).
    Returns [B, F] int32 QPs."""
    c = np.asarray(costs, dtype=np.float64)
    B, F = c.shape[0], c.shape[1]
    g = keyint if keyint and keyint > 0 else F
    key = np.zeros((B, F), dtype=bool)
    key[:, ::g] = True
    if scenecuts is not None:
        key |= np.asarray(scenecuts, dtype=bool)
    cplx = np.maximum(np.where(key, c[:, :, 0], c[:, :, 1]), 1.0)
    blurred = np.empty_like(cplx)
    acc = np.zeros(B)
    wsum = 0.0
    for t in range(F):
        acc = acc * blur + cplx[:, t]
        wsum = wsum * blur + 1.0
        blurred[:, t] = acc / wsum
    base = crf_base_complexity(mb_count, bframes)
    rate_factor = base ** (1.0 - QCOMP) / qp2qscale(crf + (MBTREE_CRF_OFFSET if mbtree else 0.0))
    qs = np.maximum(blurred ** (1.0 - QCOMP) / rate_factor, 1e-9)
    qp = 12.0 + 6.0 * np.log2(qs / 0.85)
    qp[key] -= IP_OFFSET
    return np.clip(np.round(qp), max(QP_MIN, qp_min), min(QP_MAX, qp_max)).astype(np.int32)


def crf_qps_anchors(cplx: np.ndarray, intra: np.ndarray, crf: float, mb_count: int, keys: np.ndarray,
                    blur: float = 0.5, qp_min: int = QP_MIN, qp_max: int = QP_MAX, mbtree: bool = False,
                    bframes: int = 0) -> np.ndarray:
    """CRF QPs of the anchor pictures of B segments with per-slot GOP structures.

    ``cplx``: [B, F] complexity of every anchor at its real reference distance (NaN for B
    pictures: x264 keeps their complexity out of the rate-control state and gives them their
    references' QP, :func:`b_qps_from_refs`); ``intra``: [B, F] intra costs; ``keys``: [B, F]
    pictures coded intra (the IDR, scene cuts: intra complexity, QP - ipratio).  Returns
    [B, F] int32 with the B pictures' entries left at the anchors' curve value of their
    neighbourhood (callers overwrite them)."""
    c = np.asarray(cplx, dtype=np.float64)
    B, F = c.shape
    keys = np.asarray(keys, dtype=bool)
    anchor = ~np.isnan(c)
    cx = np.where(keys, np.asarray(intra, dtype=np.float64), np.nan_to_num(c, nan=1.0))
    cx = np.maximum(cx, 1.0)
    blurred = np.empty_like(cx)
    acc = np.zeros(B)
    wsum = np.zeros(B)
    for t in range(F):
        a = anchor[:, t] | keys[:, t]
        acc = np.where(a, acc * blur + cx[:, t], acc)
        wsum = np.where(a, wsum * blur + 1.0, wsum)
        blurred[:, t] = acc / np.maximum(wsum, 1e-9)
    base = crf_base_complexity(mb_count, bframes)
    rate_factor = base ** (1.0 - QCOMP) / qp2qscale(crf + (MBTREE_CRF_OFFSET if mbtree else 0.0))
    qs = np.maximum(blurred ** (1.0 - QCOMP) / rate_factor, 1e-9)
    qp = 12.0 + 6.0 * np.log2(qs / 0.85)
    qp[keys] -= IP_OFFSET
    return np.clip(np.round(qp), max(QP_MIN, qp_min), min(QP_MAX, qp_max)).astype(np.int32)


def b_qps_from_refs(qps: np.ndarray, plans, pb_offset: float = PB_OFFSET, ip_offset: float = IP_OFFSET_F,
                    qp_max: int = QP_MAX) -> np.ndarray:
    """B-picture QPs from their references, the x264 / x265 CRF rule: a B picture has no rate
    control of its own, it takes the POC-distance weighted mean QP of its nearest list-0 and
    list-1 references (an I reference is replaced by the other side, or both I: their mean +
    ipratio) plus ``pb_offset`` (--pbratio 1.3), half of it for a reference B (b-pyramid),
    whose own QP is taken ``pb_offset / 2`` lower when it serves as a reference.

    ``qps``: [B, F] display-order QPs (anchors already set); ``plans``: one coding-order plan
    shared by all slots or a list of per-slot plans; a picture needs ``d``, ``kind``, ``l0``,
    ``l1`` (display indices of the nearest references) and optionally ``ref``.  Coding order
    guarantees a B picture's references got their QPs first.  Returns a new int32 array."""
    q = np.asarray(qps, dtype=np.float64).copy()
    B = q.shape[0]
    per_slot = len(plans) == B and len(plans) > 0 and isinstance(plans[0], (list, tuple))
    for b in range(B):
        plan = plans[b] if per_slot else plans
        kind = {pic.d: pic.kind for pic in plan}
        bref = {pic.d for pic in plan if pic.kind == "B" and getattr(pic, "ref", False)}
        for pic in plan:
            if pic.kind != "B":
                continue
            d0, d1 = pic.l0, pic.l1
            q0, q1 = q[b, d0], q[b, d1]
            if d0 in bref:
                q0 -= pb_offset / 2
            if d1 in bref:
                q1 -= pb_offset / 2
            i0, i1 = kind.get(d0) == "I", kind.get(d1) == "I"
            if i0 and i1:
                v = (q0 + q1) / 2 + ip_offset
            elif i0:
                v = q1
            elif i1:
                v = q0
            else:
                t0, t1 = abs(pic.d - d0), abs(d1 - pic.d)
                v = (q0 * t1 + q1 * t0) / max(1, t0 + t1)
            q[b, pic.d] = v + (pb_offset / 2 if pic.d in bref else pb_offset)
    return np.clip(np.round(q), QP_MIN, qp_max).astype(np.int32)


def abr_solve(stats: np.ndarray, target_bits: float, exponent: float = 1.0) -> float:
    """Global QP offset so that the predicted total bits hit ``target_bits``.

    ``stats``: [n_frames_total, 4] pass-1 statistics (bits measured at qp).  Predicted
    bits of frame f at QP qp_f + d: bits_f * (qscale(qp_f) / qscale(qp_f + d))^exponent
    = bits_f * 2^(-exponent * d / 6).  Solved in closed form."""
    b1 = float(np.sum(stats[:, 2]))
    if b1 <= 0 or target_bits <= 0:
        return 0.0
    return -6.0 / exponent * math.log2(target_bits / b1)


def abr_qps(stats: np.ndarray, target_bits: float, exponent: float = 1.0) -> np.ndarray:
    d = abr_solve(stats, target_bits, exponent)
    return np.array([clamp_qp(q + d) for q in stats[:, 3]], dtype=np.int32)


def estimate_exponent(bits_a: float, qp_a: float, bits_b: float, qp_b: float) -> float:
    """bits ~ qscale^-e: e from two encodes of the same content."""
    if bits_a <= 0 or bits_b <= 0 or qp_a == qp_b:
        return 1.0
    return -math.log2(bits_b / bits_a) * 6.0 / (qp_b - qp_a)


class TwoPassFeedback:
    """Pass-2 rate feedback: the closed-form solve of :func:`abr_solve` assumes
    ``bits ~ qscale^-1``; real encodes deviate (the exponent depends on content, frame type
    and QP range -- config 5 landed at 66 % of its target with it).  This controller
    re-solves the offset of the frames not yet encoded from what pass 2 has spent so far,
    x264-style (its 2-pass ``overflow`` compensation), with the exponent measured on the
    frames already coded:

    * ``r = spent / pass1_bits(done)`` at the mean QP offset ``d_done`` of those frames gives
      ``e = -6 log2(r) / d_done`` (the prior when ``|d_done|`` is small), clamped and damped;
    * the remaining budget ``target - spent`` over ``pass1_bits(rest)`` gives the offset of
      the rest, ``d = -6 / e * log2(budget / rest1)``, dithered over the slots so that the
      fractional part is realised on average.

    One instance per rank: the global solve (CC-1) splits the file's budget into per-rank
    shares, each rank steers its own share, so the file total follows without further
    collectives.  Inputs are [B, F] arrays in coding order."""

    def __init__(self, pass1_bits: np.ndarray, pass1_qps: np.ndarray, target_bits: float, exponent: float = 1.0,
                 qp_min: int = QP_MIN, qp_max: int = QP_MAX):
        self.b1 = np.asarray(pass1_bits, dtype=np.float64)
        self.q1 = np.asarray(pass1_qps, dtype=np.float64)
        self.target = float(target_bits)
        self.e = float(exponent)
        self.qmin, self.qmax = qp_min, qp_max
        d0 = abr_solve(np.stack([np.zeros(self.b1.size), np.zeros(self.b1.size), self.b1.reshape(-1),
                                 self.q1.reshape(-1)], axis=1), self.target, self.e)
        self.qps = self._dither(np.full(self.b1.shape, d0), 0)
        self.history: list[tuple[int, float, float]] = []  # (frames known, exponent, offset of the rest)

    def _dither(self, d: np.ndarray, t0: int) -> np.ndarray:
        """q1 + d rounded so that every frame step's mean offset over the slots equals d."""
        q = self.q1 + d
        B = q.shape[0]
        out = np.rint(q)
        for t in range(t0, q.shape[1]):
            frac = q[:, t] - np.floor(q[:, t])
            base = np.floor(q[:, t])
            k = int(round(float(np.sum(frac))))
            order = np.argsort(-frac, kind="stable")
            up = np.zeros(B, dtype=bool)
            up[order[:k]] = True
            out[:, t] = base + up
        return np.clip(out, self.qmin, self.qmax).astype(np.int32)

    def update(self, known: int, spent_bits: np.ndarray, t_next: int) -> np.ndarray:
        """``spent_bits``: [B, known] pass-2 bits of frames < known (all slots);
        returns the [B, F] QPs with frames >= t_next re-solved."""
        F = self.b1.shape[1]
        if known <= 0 or t_next >= F:
            return self.qps
        spent = float(np.sum(spent_bits[:, :known]))
        b1_done = float(np.sum(self.b1[:, :known]))
        rest1 = float(np.sum(self.b1[:, t_next:]))
        # mean QP offset actually used on the known frames (bits-weighted)
        w = np.maximum(self.b1[:, :known], 1.0)
        d_done = float(np.sum((self.qps[:, :known] - self.q1[:, :known]) * w) / np.sum(w))
        if b1_done > 0 and spent > 0 and abs(d_done) >= 0.75:
            e_meas = -6.0 * math.log2(spent / b1_done) / d_done
            e_meas = min(2.5, max(0.35, e_meas))
            # damped: trust the measurement more as more frames are known
            a = min(0.8, known / max(1.0, F / 3.0))
            self.e = (1.0 - a) * self.e + a * e_meas
        # frames between `known` and `t_next` are in flight at their current QPs: predict them
        inflight = 0.0
        if t_next > known:
            dq = self.qps[:, known:t_next] - self.q1[:, known:t_next]
            inflight = float(np.sum(self.b1[:, known:t_next] * 2.0 ** (-self.e * dq / 6.0)))
        budget = self.target - spent - inflight
        if rest1 <= 0:
            return self.qps
        budget = max(budget, 0.05 * rest1)  # overshoot: coarsest allowed, never a negative budget
        d = -6.0 / self.e * math.log2(budget / rest1)
        d = min(24.0, max(-24.0, d))
        new = self._dither(np.full(self.b1.shape, d), t_next)
        self.qps = np.concatenate([self.qps[:, :t_next], new[:, t_next:]], axis=1)
        self.history.append((known, self.e, d))
        return self.qps


class GlobalStats:
    """CC-1: every rank writes the rows of its own segments into a zero-initialised
    [n_frames_total, 4] tensor; one SUM all-reduce gives every rank the global table."""

    def __init__(self, n_frames_total: int, env=None):
        import torch
        self.env = env
        from ..parallel.dist import coll_device
        dev = coll_device(env) if env is not None else torch.device("cpu")
        self.t = torch.zeros((n_frames_total, 4), dtype=torch.float64, device=dev)

    def put(self, frame0: int, stats: np.ndarray):
        import torch
        self.t[frame0:frame0 + len(stats)] = torch.from_numpy(np.asarray(stats, dtype=np.float64)).to(self.t.device)

    def reduce(self) -> np.ndarray:
        from ..parallel import dist as D
        if self.env is not None:
            D.allreduce_stats(self.env, self.t)
        return self.t.cpu().numpy()
