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
