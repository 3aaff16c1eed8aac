"""GOP structure shared by the H.264 and HEVC encoders: closed GOPs in coding order.

An I picture, then P anchors every ``bframes + 1`` display pictures (and at the last
picture and at forced anchors such as scene cuts), each followed in coding order by the
non-reference B pictures before it -- x264 / x265 ``--b-adapt 0`` without a pyramid.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class PicPlan:
    """One picture of a closed GOP in coding order."""
    d: int          # display index
    kind: str       # "I", "P" or "B"
    frame_num: int
    poc: int        # PicOrderCnt (2 * display index)
    anchor: int     # I / P: anchor ordinal (its recon / half-sample buffer is anchor & 1); B: -1
    l0: int = -1    # display index of RefPicList0[0] (P, B)
    l1: int = -1    # display index of RefPicList1[0] (B)
    l1_anchor: int = -1  # B: anchor ordinal of RefPicList1[0]

    @property
    def slice_type(self) -> int:  # SliceType (csrc/common/h264_mb.h)
        return {"P": 0, "B": 1, "I": 2}[self.kind]

    @property
    def nal_ref_idc(self) -> int:
        return {"I": 3, "P": 2, "B": 0}[self.kind]


def gop_plan(frames: int, bframes: int, anchors_at=()) -> list[PicPlan]:
    """Coding order of a closed GOP of ``frames`` pictures: I0, then every anchor (P at
    display indices 0, bframes + 1, ... and the last picture) followed by the B pictures
    before it (x264's fixed --b-adapt 0 pattern, no pyramid).  frame_num counts reference
    pictures (clause 7.4.3); B pictures are non-reference.

    anchors_at: extra display indices that must be anchors.  A picture d that is an anchor
    ends a coding-order prefix holding exactly pictures 0..d, so a segment shorter than the
    batch (padded to F frames) is cut there (SegmentResult.display_prefix)."""
    if frames < 1:
        return []
    step = max(0, int(bframes)) + 1
    anchors = set(range(0, frames, step)) | {frames - 1} | {int(d) for d in anchors_at if 0 <= int(d) < frames}
    if step > 1:  # keep every B run <= bframes after inserting the extra anchors
        out_a, prev = [0], 0
        for a in sorted(anchors - {0}):
            while a - prev > step:
                prev += step
                out_a.append(prev)
            out_a.append(a)
            prev = a
        anchors = out_a
    else:
        anchors = sorted(anchors)
    out = [PicPlan(0, "I", 0, 0, 0)]
    fn = 1
    for i in range(1, len(anchors)):
        a0, a1 = anchors[i - 1], anchors[i]
        out.append(PicPlan(a1, "P", fn & 0xFFFF, 2 * a1, i, l0=a0))
        fn += 1
        for d in range(a0 + 1, a1):
            out.append(PicPlan(d, "B", fn & 0xFFFF, 2 * d, -1, l0=a0, l1=a1, l1_anchor=i))
    return out


@dataclass(frozen=True)
class GopPic:
    """One picture of an HEVC closed GOP in coding order (models/hevc_gpu.py).

    ``rps``: the reference picture set of the picture, ``(display index, used by the
    current picture)`` for every picture the DPB must still hold; ``slot``: the
    reconstruction buffer (0 .. ref_slots - 1 for reference pictures, ``ref_slots`` for
    non-reference B pictures); ``l0`` / ``l1``: display indices of RefPicList0[0] /
    RefPicList1[0] and ``s0`` / ``s1`` their buffers."""
    d: int
    kind: str                # "I", "P", "B"
    ref: bool                # referenced by later pictures (I, P, the pyramid's middle B)
    slot: int
    rps: tuple = ()
    l0: int = -1
    l1: int = -1
    s0: int = -1
    s1: int = -1


def hevc_gop_plan(frames: int, bframes: int, pyramid: bool = True, anchors_at=(), ref_slots: int = 3) -> list[GopPic]:
    """x265-style closed GOP: I0, P anchors every ``bframes + 1`` pictures (plus the last
    picture and ``anchors_at``), each followed by the B pictures before it.  With
    ``pyramid`` and two or more B pictures in a run, the middle one is a reference B
    (list 0 = the previous anchor, list 1 = the new one) coded first, and the others are
    non-reference b pictures predicting from their nearest references on both sides
    (x265 --b-pyramid).  The DPB is simulated to give every picture its RPS and buffer."""
    if frames < 1:
        return []
    step = max(0, int(bframes)) + 1
    anchors = sorted(set(range(0, frames, step)) | {frames - 1} | {int(d) for d in anchors_at if 0 <= int(d) < frames})
    if step > 1:  # keep every B run <= bframes after inserting the extra anchors
        out_a, prev = [0], 0
        for a in anchors[1:]:
            while a - prev > step:
                prev += step
                out_a.append(prev)
            out_a.append(a)
            prev = a
        anchors = out_a
    # (display index, kind, ref, l0, l1) in coding order
    seq = [(0, "I", True, -1, -1)]
    for a0, a1 in zip(anchors, anchors[1:]):
        seq.append((a1, "P", True, a0, -1))
        run = list(range(a0 + 1, a1))
        if pyramid and len(run) >= 2:
            mid = (a0 + a1) // 2
            seq.append((mid, "B", True, a0, a1))
            seq += [(d, "B", False, a0, mid) for d in run if d < mid]
            seq += [(d, "B", False, mid, a1) for d in run if d > mid]
        else:
            seq += [(d, "B", False, a0, a1) for d in run]
    # a reference picture stays in the DPB until the last picture that uses it
    last_use: dict = {}
    for i, (d, kind, ref, l0, l1) in enumerate(seq):
        for r in (l0, l1):
            if r >= 0:
                last_use[r] = i
    dpb: dict = {}  # display index -> slot
    out = []
    for i, (d, kind, ref, l0, l1) in enumerate(seq):
        if kind == "I":
            dpb = {}
        keep = {r: s for r, s in dpb.items() if last_use.get(r, -1) >= i}
        dpb = keep
        rps = tuple(sorted((r, r in (l0, l1)) for r in keep))
        if ref:
            free = [s for s in range(ref_slots) if s not in dpb.values()]
            if not free:
                raise ValueError("hevc_gop_plan: more reference pictures than buffers")
            slot = free[0]
        else:
            slot = ref_slots
        out.append(GopPic(d, kind, ref, slot, rps, l0, l1, dpb.get(l0, -1), dpb.get(l1, -1)))
        if ref:
            dpb[d] = slot
    return out
