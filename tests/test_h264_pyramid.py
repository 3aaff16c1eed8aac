"""Per-slot GOP plans (models/gop.py h264_plan): b-pyramid, list modification, DPB.

x264's ``--b-pyramid normal`` (a default of the reference's bare ``-vcodec libx264``,
server.go:69-70) keeps the middle B picture of a run as a reference and orders every P
picture's list 0 by POC distance, which differs from the default PicNum order once a
reference B sits in the DPB: the writer then emits ref_pic_list_modification commands.
These CPU tests pin the plan (coding order, frame_num, sliding-window DPB, lists) and check
with the independent decoder (csrc/host/h264_decoder.cc) that a P picture whose MBs copy
reference ref_idx r (zero vector, no residual, no deblocking) reproduces exactly the picture
the plan put at list-0 position r.  No third-party decoder exists here: parity with x264's
own pyramid streams is unpinned.
"""
import numpy as np
import pytest

from govideocompressor_amd.models.gop import dpb_frames, fixed_types, h264_plan
from govideocompressor_amd.utils.h264_synth import HDR_BYTES, _intra_record, _levels

_KIND, _QP, _REF, _MV = 0, 2, 8, 16
P16x16, B16x16 = 2, 9


def test_fixed_types_and_plan_orders():
    assert fixed_types(9, 3) == "IBBBPBBBP"
    assert fixed_types(7, 3, anchors_at=[2]) == "IBPBPBP"  # the grid anchors stay
    plan = h264_plan("IBBBPBBBP", refs=3, pyramid=True)
    assert [(p.d, p.kind, p.ref) for p in plan] == [(0, "I", True), (4, "P", True), (2, "B", True), (1, "B", False),
                                                     (3, "B", False), (8, "P", True), (6, "B", True), (5, "B", False),
                                                     (7, "B", False)]
    by_d = {p.d: p for p in plan}
    # frame_num counts reference pictures; non-reference pictures share the next value
    assert [p.frame_num for p in plan] == [0, 1, 2, 3, 3, 3, 4, 5, 5]
    assert by_d[1].refs0 == (0,) and by_d[1].refs1 == (2,)
    assert by_d[3].refs0 == (2, 0) and by_d[3].refs1 == (4,)
    # P8: POC-distance order [P4, B2, I0] vs the default PicNum order [B2, P4, I0]
    assert by_d[8].refs0 == (4, 2, 0) and by_d[8].mod_l0 == ((0, 1), (1, 0), (0, 1))
    assert by_d[2].nal_ref_idc == 1 and by_d[1].nal_ref_idc == 0
    # buffers: a reference picture keeps its buffer while in the DPB, B pictures use the scratch one
    nref = dpb_frames(3, True, 3)
    assert all(p.buf == nref + 1 for p in plan if not p.ref)
    for p in plan:
        for r, b in zip(p.refs0, p.bufs0):
            assert by_d[r].buf == b
    # no pyramid: the x264 --b-adapt 0 order, no modification
    flat = h264_plan("IBBBPBBBP", refs=3, pyramid=False)
    assert [p.d for p in flat] == [0, 4, 1, 2, 3, 8, 5, 6, 7]
    assert not any(p.mod_l0 for p in flat) and not any(p.ref for p in flat if p.kind == "B")


def test_plan_sliding_window_never_references_an_evicted_picture():
    rng = np.random.default_rng(3)
    for _ in range(50):
        n = int(rng.integers(2, 40))
        ty = ["I"] + ["P" if rng.random() < 0.4 else "B" for _ in range(n - 2)] + ["P"]
        ty = "".join(ty)
        for pyr in (False, True):
            plan = h264_plan(ty, refs=3, pyramid=pyr, nref_frames=4)
            live: dict[int, int] = {}
            for p in plan:
                for r, b in zip(p.refs0 + p.refs1, p.bufs0 + ((p.buf1,) if p.refs1 else ())):
                    assert live.get(r) == b, (ty, pyr, p)
                if p.ref:
                    assert p.buf not in live.values()
                    live[p.d] = p.buf
                    if len(live) > 4:
                        oldest = min(live, key=lambda d: next(q.frame_num for q in plan if q.d == d))
                        del live[oldest]


def _pic_records(rng, nmb, wmb, kind, qp, nref=1, refs=None):
    hdr = np.zeros((nmb, HDR_BYTES), np.uint8)
    hdr[:, _REF:_REF + 8] = 0xFF
    coef = np.zeros((nmb, 408), np.int16)
    for mb in range(nmb):
        if kind == "I":
            _intra_record(rng, hdr[mb], coef[mb], mb % wmb, mb // wmb, qp, 0.2)
            continue
        hdr[mb, _QP] = qp
        if refs is not None:  # copy reference refs[mb]: zero vector, no residual
            hdr[mb, _KIND] = P16x16
            hdr[mb, _REF:_REF + 4] = refs[mb]
            continue
        hdr[mb, _KIND] = P16x16 if kind == "P" else B16x16
        hdr[mb, _REF:_REF + 4] = 0
        if kind == "B":
            hdr[mb, _REF + 4:_REF + 8] = 0  # bi-predicted
        hdr[mb, _MV:_MV + 32] = np.frombuffer(rng.integers(-12, 13, (2, 4, 2)).astype(np.int16).tobytes(), np.uint8)
        for b in range(16):
            coef[mb, b * 16:(b + 1) * 16] = _levels(rng, 16, 0.3)
    return hdr, coef


@pytest.mark.parametrize("seed", [1, 2])
def test_pyramid_stream_decodes_with_modified_lists(host, seed):
    rng = np.random.default_rng(seed)
    w, h = 64, 48
    wmb, hmb = w // 16, h // 16
    nmb = wmb * hmb
    refs = 3
    cfg = dict(width=w, height=h, qp=28, cabac=1, bframes=3, refs=refs, pyramid=1, deblock=0, weighted_bipred=0)
    plan = h264_plan("IBBBPBBBP", refs=refs, pyramid=True, nref_frames=dpb_frames(refs, True, 3))
    out = [host.parameter_sets(cfg)]
    copy_refs = None
    for p in plan:
        if p.d == 8:
            copy_refs = np.arange(nmb) % len(p.refs0)
            hdr, coef = _pic_records(rng, nmb, wmb, "P", 28, refs=copy_refs)
        else:
            hdr, coef = _pic_records(rng, nmb, wmb, p.kind, 28)
        fp = dict(idr=int(p.kind == "I"), qp=28, frame_num=p.frame_num, poc=p.poc, slice_type=p.slice_type,
                  nal_ref_idc=p.nal_ref_idc, direct_spatial=1)
        if p.kind != "I":
            fp["num_ref_l0"] = len(p.refs0)
            fp["num_ref_l1"] = 1
            if p.mod_l0:
                fp["mod_l0"] = list(p.mod_l0)
        out.append(host.write_slice(cfg, fp, hdr, coef)[0])
    pics = host.decode(b"".join(out))
    assert [q["poc"] // 2 for q in pics] == list(range(9))  # display order, every picture output
    p8 = next(p for p in plan if p.d == 8)
    y8 = np.asarray(pics[8]["y_coded"]).reshape(h, w)
    for mb in range(nmb):
        mx, my = mb % wmb, mb // wmb
        want = p8.refs0[copy_refs[mb]]
        blk = y8[my * 16:(my + 1) * 16, mx * 16:(mx + 1) * 16]
        for d, q in enumerate(pics):
            other = np.asarray(q["y_coded"]).reshape(h, w)[my * 16:(my + 1) * 16, mx * 16:(mx + 1) * 16]
            if d == want:
                assert np.array_equal(blk, other), (mb, want)


def test_pyramid_with_one_reference_keeps_both_anchors(host):
    """--ref 1 (veryfast / superfast presets) with a pyramid: the DPB must hold I0, P4 and the
    reference B2 at once, and P4 must survive the store of B6 while B2 is still in the window
    (round-4 review: a window of refs + 1 = 2 evicted I0 when B2 was stored, leaving B1
    without a list 0)."""
    assert dpb_frames(1, True, 3) == 4 and dpb_frames(1, False, 3) == 2 and dpb_frames(3, True, 3) == 4
    plan = h264_plan("IBBBPBBBP", refs=1, pyramid=True)
    by_d = {p.d: p for p in plan}
    assert by_d[1].refs0 == (0,) and by_d[1].refs1 == (2,)
    assert by_d[3].refs0 == (2,) and by_d[3].refs1 == (4,)
    assert by_d[5].refs0 == (4,) and by_d[7].refs1 == (8,)
    # the SPS max_num_ref_frames agrees (the decoder's sliding window is what the plan simulates)
    rng = np.random.default_rng(5)
    w, h = 48, 32
    wmb = w // 16
    nmb = wmb * (h // 16)
    cfg = dict(width=w, height=h, qp=28, cabac=1, bframes=3, refs=1, pyramid=1, deblock=0, weighted_bipred=0)
    out = [host.parameter_sets(cfg)]
    for p in plan:
        hdr, coef = _pic_records(rng, nmb, wmb, p.kind, 28)
        fp = dict(idr=int(p.kind == "I"), qp=28, frame_num=p.frame_num, poc=p.poc, slice_type=p.slice_type,
                  nal_ref_idc=p.nal_ref_idc, direct_spatial=1)
        if p.kind != "I":
            fp["num_ref_l0"] = len(p.refs0)
            fp["num_ref_l1"] = 1
            if p.mod_l0:
                fp["mod_l0"] = list(p.mod_l0)
        out.append(host.write_slice(cfg, fp, hdr, coef)[0])
    pics = host.decode(b"".join(out))
    assert [q["poc"] // 2 for q in pics] == list(range(9))
