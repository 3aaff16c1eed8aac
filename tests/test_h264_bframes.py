"""B pictures through the host CABAC writer and the independent decoder (CPU).

The GPU encoder codes B pictures with temporal direct prediction (B_Skip / B_Direct_16x16)
and B_16x16 L0 / L1 / Bi macroblocks.  These tests pin the writer, the decoder and the
numpy temporal-direct derivation (utils/h264_synth.temporal_direct, clause 8.4.1.2.3)
against each other on random records: stream I0 P2 B1 (coding order), POC type 0.
Reference parity: x264 --bframes / --direct temporal behind `-vcodec libx264`
(server.go:69-70); a third-party B stream is not available here (parity unpinned).
"""
import numpy as np
import pytest

from govideocompressor_amd.utils.h264_synth import (B16x16, BDIRECT, HDR_BYTES, P16x16, _intra_record, _levels,
                                                    temporal_direct)

_KIND, _QP, _FLAGS, _REF, _MV = 0, 2, 5, 8, 16


def _mv_bytes(mv):
    return np.frombuffer(np.asarray(mv, np.int16).reshape(-1).tobytes(), np.uint8)


def _b_stream(host, w, h, seed, skip_frac=0.3):
    rng = np.random.default_rng(seed)
    cfg = dict(width=w, height=h, qp=28, cabac=1, bframes=1)
    wmb, hmb = (w + 15) // 16, (h + 15) // 16
    nmb = wmb * hmb
    out = [host.parameter_sets(cfg)]
    # I0 (POC 0)
    hdr = np.zeros((nmb, HDR_BYTES), np.uint8)
    hdr[:, _REF:_REF + 8] = 0xFF
    coef = np.zeros((nmb, 408), np.int16)
    for mb in range(nmb):
        _intra_record(rng, hdr[mb], coef[mb], mb % wmb, mb // wmb, 28, 0.1)
    out.append(host.write_slice(cfg, dict(idr=1, qp=28, frame_num=0, poc=0), hdr, coef)[0])
    # P2 (POC 4): P16x16 with random vectors, some intra
    ph = np.zeros((nmb, HDR_BYTES), np.uint8)
    ph[:, _REF:_REF + 8] = 0xFF
    pc = np.zeros((nmb, 408), np.int16)
    for mb in range(nmb):
        if rng.random() < 0.15:
            _intra_record(rng, ph[mb], pc[mb], mb % wmb, mb // wmb, 28, 0.1)
            continue
        ph[mb, _KIND] = P16x16
        ph[mb, _QP] = 28
        ph[mb, _REF:_REF + 4] = 0
        ph[mb, _MV:_MV + 16] = _mv_bytes(np.tile(rng.integers(-40, 41, 2), 4))
        for b in range(16):
            pc[mb, b * 16:(b + 1) * 16] = _levels(rng, 16, 0.1) if rng.random() < 0.5 else 0
    out.append(host.write_slice(cfg, dict(idr=0, qp=28, frame_num=1, poc=4), ph, pc)[0])
    # B1 (POC 2), non-reference: L0 = P2's reference (I0), L1 = P2
    mv0, mv1 = temporal_direct(ph, 2, 0, 4)
    bh = np.zeros((nmb, HDR_BYTES), np.uint8)
    bh[:, _REF:_REF + 8] = 0xFF
    bc = np.zeros((nmb, 408), np.int16)
    kinds = []
    for mb in range(nmb):
        r = rng.random()
        if r < 0.1:
            _intra_record(rng, bh[mb], bc[mb], mb % wmb, mb // wmb, 30, 0.1)
            kinds.append("intra")
            continue
        bh[mb, _QP] = 30
        if r < 0.1 + skip_frac + 0.2:  # direct (B_Skip when nothing is coded)
            bh[mb, _KIND] = BDIRECT
            bh[mb, _REF:_REF + 8] = 0
            bh[mb, _MV:_MV + 32] = _mv_bytes(np.stack([mv0[mb], mv1[mb]]))
            kinds.append("direct")
            if r < 0.1 + skip_frac:
                continue
        else:
            lists = int(rng.integers(1, 4))  # 1 L0, 2 L1, 3 Bi
            bh[mb, _KIND] = B16x16
            mvs = np.zeros((2, 4, 2), np.int64)
            for li in range(2):
                if (lists >> li) & 1:
                    bh[mb, _REF + 4 * li:_REF + 4 * li + 4] = 0
                    mvs[li] = np.tile(rng.integers(-30, 31, 2), (4, 1))
            bh[mb, _MV:_MV + 32] = _mv_bytes(mvs)
            kinds.append(("L0", "L1", "Bi")[lists - 1])
        for b in range(16):
            bc[mb, b * 16:(b + 1) * 16] = _levels(rng, 16, 0.1) if rng.random() < 0.5 else 0
        bc[mb, 272:280] = _levels(rng, 8, 0.1)
    out.append(host.write_slice(cfg, dict(idr=0, slice_type=1, nal_ref_idc=0, qp=30, frame_num=2, poc=2,
                                          direct_spatial=0), bh, bc)[0])
    return b"".join(out), (ph, bh, bc, mv0, kinds)


@pytest.mark.parametrize("w,h,seed", [(64, 48, 1), (96, 80, 2), (176, 144, 3)])
def test_b_picture_roundtrip_temporal_direct(host, w, h, seed):
    s, (ph, bh, bc, mv0, kinds) = _b_stream(host, w, h, seed)
    pics = host.decode(s)
    assert [p["poc"] for p in pics] == [0, 2, 4]  # display order
    b = pics[1]
    assert b["slice_type"] == 1
    nmb = bh.shape[0]
    dec_mv = np.asarray(b["mv"]).reshape(nmb, 16, 2)
    for mb in range(nmb):
        k = kinds[mb]
        if k == "intra":
            continue
        if k in ("direct", "L0", "Bi"):
            # L0 motion of every 4x4 block: the quadrant's vector
            want = np.frombuffer(bh[mb, _MV:_MV + 16].tobytes(), np.int16).reshape(4, 2)
            for blk in range(16):
                bx, by = (blk % 4), (blk // 4)
                q = (by // 2) * 2 + bx // 2
                assert tuple(dec_mv[mb, blk]) == tuple(want[q]), (mb, k, blk)
    # the parse-only decoder recovers the B records (kinds, refs and both lists' vectors)
    seg = host.parse([s], 1)[0]
    assert seg["error"] is None
    got = seg["hdr"][2]  # coding order: I0, P2, B1
    for mb in range(nmb):
        if kinds[mb] == "intra":
            continue
        assert got[mb, _KIND] == bh[mb, _KIND], (mb, kinds[mb])
        assert np.array_equal(got[mb, _REF:_REF + 8].view(np.int8), bh[mb, _REF:_REF + 8].view(np.int8)), mb
        assert np.array_equal(got[mb, _MV:_MV + 32], bh[mb, _MV:_MV + 32]), (mb, kinds[mb])


def test_temporal_direct_scaling_matches_spec_example():
    """tb / td scaling with C division: POC distances 2 / 4 halve the co-located vector."""
    col = np.zeros((1, HDR_BYTES), np.uint8)
    col[0, _KIND] = P16x16
    col[0, _MV:_MV + 16] = _mv_bytes(np.tile([9, -7], 4))
    m0, m1 = temporal_direct(col, 2, 0, 4)
    # tx = (16384 + 2) / 4 = 4096; DSF = (2 * 4096 + 32) >> 6 = 128; mvL0 = (128 * mv + 128) >> 8
    assert tuple(m0[0, 0]) == ((128 * 9 + 128) >> 8, (128 * -7 + 128) >> 8)
    assert tuple(m1[0, 0]) == (m0[0, 0, 0] - 9, m0[0, 0, 1] + 7)
