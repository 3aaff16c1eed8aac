"""GOP structure shared by the H.264 and HEVC encoders: closed GOPs in coding order.

An I picture, then P anchors (every ``bframes + 1`` display pictures for x264's fixed
``--b-adapt 0`` pattern, wherever the lookahead put them for ``--b-adapt 1``, and at the
last picture and at forced anchors such as scene cuts), each followed in coding order by
the B pictures before it; with ``--b-pyramid`` the middle B of a run is a reference
picture coded first.  H.264 plans are per slot (models/h264_gpu.py routes every slot of a
batch through its own plan).
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class PicPlan:
    """One picture of an H.264 closed GOP in coding order (one slot's plan, models/h264_gpu.py).

    ``refs0`` / ``refs1``: display indices of the active RefPicList0 / RefPicList1 entries
    (nearest first); ``buf``: the reconstruction pool buffer of the picture (reference
    pictures own theirs while they are in the DPB; every non-reference B uses the scratch
    buffer), ``bufs0`` / ``buf1`` those of its references; ``mod_l0``: the
    ref_pic_list_modification commands that turn the default (PicNum) list-0 order into the
    POC-distance order, empty when they agree."""
    d: int          # display index
    kind: str       # "I", "P" or "B"
    frame_num: int
    poc: int        # PicOrderCnt (2 * display index)
    anchor: int     # I / P: anchor ordinal; B: -1
    l0: int = -1    # display index of RefPicList0[0] (P, B)
    l1: int = -1    # display index of RefPicList1[0] (B)
    l1_anchor: int = -1  # B: anchor ordinal of RefPicList1[0] (-1 when it is a reference B)
    ref: bool = False    # referenced by later pictures (I, P, a pyramid's reference B)
    refs0: tuple = ()
    refs1: tuple = ()
    buf: int = -1
    bufs0: tuple = ()
    buf1: int = -1
    mod_l0: tuple = ()

    @property
    def slice_type(self) -> int:  # SliceType (csrc/common/h264_mb.h)
        return {"P": 0, "B": 1, "I": 2}[self.kind]

    @property
    def nal_ref_idc(self) -> int:  # x264: I 3, P 2, reference B 1, B 0
        return {"I": 3, "P": 2, "B": 1 if self.ref else 0}[self.kind]


def fixed_types(frames: int, bframes: int, anchors_at=()) -> str:
    """Display-order picture types of x264's fixed --b-adapt 0 pattern: I0, P every
    ``bframes + 1`` pictures and at the last picture and at ``anchors_at``, B between them
    (runs never longer than ``bframes``)."""
    if frames < 1:
        return ""
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
        anchors = set(out_a)
    return "".join("I" if d == 0 else ("P" if d in anchors else "B") for d in range(frames))


def dpb_frames(refs: int, pyramid: bool, bframes: int) -> int:
    """max_num_ref_frames of the stream (the SPS value, csrc/host/cpu_encoder.cc): the active
    references plus one when B pictures are on (a reference B or the next anchor's slot).  A
    pyramid (runs of two or more B) needs at least 4 even with ``refs`` 1: the window (no MMCO,
    oldest frame_num out) holds the run's anchors a0 / a1 and its reference B, plus the previous
    run's reference B, which sits between a0 and a1 in frame_num order -- with fewer, storing
    the new reference B evicts a0 and the B pictures after it lose their list-0 anchor."""
    n = max(1, int(refs)) + (1 if int(bframes) > 0 else 0)
    if pyramid and int(bframes) >= 2:
        n = max(n, 4)
    return n


def h264_plan(types: str, refs: int = 1, pyramid: bool = False, nref_frames: int | None = None) -> list[PicPlan]:
    """Coding-order plan of one closed GOP from its display-order picture types (``"IBBBP..."``,
    an I at 0, P anchors, B pictures between them).

    * Coding order: every anchor, then the B pictures before it -- with ``pyramid`` (x264
      --b-pyramid normal) and a run of two or more, its middle picture first, as a reference B
      (list 0 = the earlier anchor, list 1 = the new one), the others between it and the anchors.
    * frame_num counts reference pictures (7.4.3); the DPB is a sliding window of
      ``nref_frames`` frames (8.2.5.3), simulated to give every picture its buffer.
    * P lists: the DPB's pictures nearest first in POC (x264's distance order), the first
      ``refs``; a ref_pic_list_modification is emitted where the default PicNum order differs
      (a P after a reference B).  B lists: the default order (POC below the picture, nearest
      first, at most ``refs``; list 1 = the nearest picture above), no modification."""
    n = len(types)
    if n == 0:
        return []
    if types[0] != "I" or any(t not in "PB" for t in types[1:]) or types[-1] == "B":
        raise ValueError(f"h264_plan: types must be I, then P / B, ending on an anchor: {types!r}")
    refs = max(1, int(refs))
    nb = max((len(r) for r in types[1:].split("P") + types[1:].split("I")), default=0)
    if nref_frames is None:
        nref_frames = dpb_frames(refs, pyramid, nb)
    nbuf_ref = nref_frames + 1
    anchors = [d for d, t in enumerate(types) if t != "B"]
    # (display, kind, ref) in coding order
    seq = [(0, "I", True)]
    for a0, a1 in zip(anchors, anchors[1:]):
        seq.append((a1, types[a1], True))
        run = list(range(a0 + 1, a1))
        if pyramid and len(run) >= 2:
            mid = (a0 + a1) // 2
            seq.append((mid, "B", True))
            seq += [(d, "B", False) for d in run if d != mid]
        else:
            seq += [(d, "B", False) for d in run]
    out: list[PicPlan] = []
    dpb: list[tuple[int, int, int]] = []  # (display, frame_num, buffer) of the reference pictures
    prev_ref_fn = -1
    anchor_ord = {}
    for d, kind, ref in seq:
        if kind == "I":
            dpb, fn = [], 0
        else:
            fn = (prev_ref_fn + 1) & 0xFFFF
        if kind != "B":
            anchor_ord[d] = len(anchor_ord)
        used = {b for _, _, b in dpb}
        buf = next(b for b in range(nbuf_ref) if b not in used) if ref else nbuf_ref
        refs0: tuple = ()
        refs1: tuple = ()
        mods: tuple = ()
        if kind == "P":
            order = sorted(dpb, key=lambda e: -e[0])[:refs]
            refs0 = tuple(e[0] for e in order)
            default = sorted(dpb, key=lambda e: -e[1])[:len(order)]
            if [e[0] for e in default] != list(refs0):
                cmds, pred = [], fn
                for _, pn, _ in order:
                    cmds.append((0, pred - pn - 1) if pn < pred else (1, pn - pred - 1))
                    pred = pn
                mods = tuple(cmds)
        elif kind == "B":
            below = sorted((e for e in dpb if e[0] < d), key=lambda e: -e[0])[:refs]
            above = sorted((e for e in dpb if e[0] > d), key=lambda e: e[0])[:1]
            refs0 = tuple(e[0] for e in below)
            refs1 = tuple(e[0] for e in above)
        bof = {e[0]: e[2] for e in dpb}
        l1 = refs1[0] if refs1 else -1
        out.append(PicPlan(d, kind, fn, 2 * d, anchor_ord.get(d, -1) if kind != "B" else -1,
                           l0=refs0[0] if refs0 else -1, l1=l1,
                           l1_anchor=anchor_ord.get(l1, -1) if kind == "B" else -1, ref=ref, refs0=refs0,
                           refs1=refs1, buf=buf, bufs0=tuple(bof[r] for r in refs0), buf1=bof.get(l1, -1),
                           mod_l0=mods))
        if ref:
            prev_ref_fn = fn
            dpb.append((d, fn, buf))
            if len(dpb) > nref_frames:  # sliding window: drop the smallest FrameNumWrap
                dpb.remove(min(dpb, key=lambda e: e[1]))
    return out


def gop_plan(frames: int, bframes: int, anchors_at=(), refs: int = 1, pyramid: bool = False) -> list[PicPlan]:
    """Coding order of a closed GOP of ``frames`` pictures with x264's fixed --b-adapt 0
    pattern (:func:`fixed_types`, :func:`h264_plan`).

    anchors_at: extra display indices that must be anchors.  A picture d that is an anchor
    ends a coding-order prefix holding exactly pictures 0..d, so a segment shorter than the
    batch (padded to F frames) is cut there (SegmentResult.display_prefix)."""
    return h264_plan(fixed_types(frames, bframes, anchors_at), refs, pyramid)


@dataclass(frozen=True)
class GopPic:
    """One picture of an HEVC closed GOP in coding order (models/hevc_gpu.py).

    ``rps``: the reference picture set of the picture, ``(display index, used by the
    current picture)`` for every picture the DPB must still hold; ``slot``: the
    reconstruction buffer (0 .. ref_slots - 1 for reference pictures, ``ref_slots`` for
    non-reference B pictures); ``l0`` / ``l1``: display indices of RefPicList0[0] /
    RefPicList1[0] and ``s0`` / ``s1`` their buffers; ``refs0`` / ``srefs0``: every active
    RefPicList0 entry (nearest first; P pictures with x265 --ref > 1) and its buffer."""
    d: int
    kind: str                # "I", "P", "B"
    ref: bool                # referenced by later pictures (I, P, the pyramid's middle B)
    slot: int
    rps: tuple = ()
    l0: int = -1
    l1: int = -1
    s0: int = -1
    s1: int = -1
    refs0: tuple = ()
    srefs0: tuple = ()


def hevc_ref_slots(bframes: int, pyramid: bool, refs: int = 1) -> int:
    """Reconstruction buffers of reference pictures :func:`hevc_gop_plan` needs: the list-0
    pictures a P anchor keeps for itself and the next anchors plus the one being coded, one more
    for a pyramid's reference B (at least 2 for P-only GOPs and 3 with B pictures, the round-4
    layout)."""
    nb = max(0, int(bframes))
    need = max(1, int(refs)) + 1 + (1 if pyramid and nb >= 2 else 0)
    return max(need, 3 if nb else 2)


def hevc_gop_plan(frames: int, bframes: int, pyramid: bool = True, anchors_at=(), ref_slots: int = 3,
                  refs: int = 1, types: str | None = None) -> list[GopPic]:
    """x265-style closed GOP: I0, P anchors every ``bframes + 1`` pictures (plus the last
    picture and ``anchors_at``), each followed by the B pictures before it.  With
    ``pyramid`` and two or more B pictures in a run, the middle one is a reference B
    (list 0 = the previous anchor, list 1 = the new one) coded first, and the others are
    non-reference b pictures predicting from their nearest references on both sides
    (x265 --b-pyramid).  ``refs`` (x265 --ref): a P anchor's list 0 holds up to that many
    reference pictures, nearest first.  ``types``: display-order picture types of an adaptive
    placement (x265 --b-adapt, ``"IPBBP..."``: every non-B picture is an anchor, runs of at most
    ``bframes`` B pictures) instead of the fixed pattern.  The DPB is simulated to give every
    picture its RPS and buffer."""
    if frames < 1:
        return []
    step = max(0, int(bframes)) + 1
    nref = max(1, int(refs))
    if types is not None:
        if len(types) != frames or types[0] != "I" or types[-1] == "B":
            raise ValueError(f"hevc_gop_plan: types must cover the frames, start with I and end on an anchor: {types!r}")
        anchors = [d for d, t in enumerate(types) if t != "B"]
        if any(b - a - 1 > max(0, int(bframes)) for a, b in zip(anchors, anchors[1:])):
            raise ValueError("hevc_gop_plan: a B run longer than bframes")
        step = 1  # the runs are as given
    else:
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
    # list 0 of every P anchor: the nearest reference pictures coded before it (in its closed GOP)
    lists0 = []
    coded_refs: list = []
    for d, kind, ref, l0, l1 in seq:
        if kind == "I":
            coded_refs = []
        if kind == "P":
            near = sorted((r for r in coded_refs if r < d), key=lambda r: -r)[:nref]
            assert near and near[0] == l0, (d, near, l0)
            lists0.append(tuple(near))
        else:
            lists0.append((l0,) if l0 >= 0 else ())
        if ref:
            coded_refs.append(d)
    # a reference picture stays in the DPB until the last picture that uses it
    last_use: dict = {}
    for i, ((d, kind, ref, l0, l1), r0) in enumerate(zip(seq, lists0)):
        for r in (*r0, l0, l1):
            if r >= 0:
                last_use[r] = i
    dpb: dict = {}  # display index -> slot
    out = []
    for i, ((d, kind, ref, l0, l1), r0) in enumerate(zip(seq, lists0)):
        if kind == "I":
            dpb = {}
        keep = {r: s for r, s in dpb.items() if last_use.get(r, -1) >= i}
        dpb = keep
        used = set(r0) | {l0, l1}
        rps = tuple(sorted((r, r in used) for r in keep))
        if ref:
            free = [s for s in range(ref_slots) if s not in dpb.values()]
            if not free:
                raise ValueError("hevc_gop_plan: more reference pictures than buffers")
            slot = free[0]
        else:
            slot = ref_slots
        out.append(GopPic(d, kind, ref, slot, rps, l0, l1, dpb.get(l0, -1), dpb.get(l1, -1), r0,
                          tuple(dpb.get(r, -1) for r in r0)))
        if ref:
            dpb[d] = slot
    return out
