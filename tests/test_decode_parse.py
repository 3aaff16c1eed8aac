"""Parse-only H.264 decoding (the host half of the GPU decode path).

``_host.parse`` turns CAVLC into the encoder's MbHeader records + packed levels.
Checked here on the CPU:

* round trip: records parsed from a stream, written again by the CAVLC writer,
  reproduce the original slice NALs bit for bit (so headers, motion vectors, QPs and
  every level survive the packed format);
* consistency with the full decoder (MB kinds, QPs, motion vectors, non-zero flags);
* the GPU-coverage flags (several slices per picture stay on the GPU path; I_PCM,
  constrained intra prediction and mmco 5 fall back to the CPU).
"""
import numpy as np
import pytest

from govideocompressor_amd.utils import yuv
from govideocompressor_amd.utils.h264_synth import random_stream, unpack_levels


@pytest.mark.parametrize("w,h,seed", [(64, 48, 1), (80, 64, 2), (50, 34, 3)])
def test_parse_rewrite_roundtrip(host, w, h, seed):
    frames = 4
    s = random_stream(host, w, h, frames, seed=seed)
    seg = host.parse([s], 1)[0]
    assert seg["error"] is None and seg["n"] == frames
    nals = host.parse_nals(s)
    slices = [n for n in nals if (n[4] & 31) in (1, 5)] if isinstance(nals[0], (bytes, bytearray)) else None
    cfg = dict(width=w, height=h, qp=28)
    for t in range(frames):
        hdr = seg["hdr"][t]
        coef = unpack_levels(seg, t)
        fp = dict(idr=int(t == 0), qp=int(seg["meta"][t, 5]), frame_num=t, idr_pic_id=0)
        nal, _ = host.write_slice(cfg, fp, np.ascontiguousarray(hdr), coef)
        if slices is not None:
            assert nal == slices[t], f"picture {t}: rewritten slice differs"
    rebuilt = host.parameter_sets(cfg) + b"".join(
        host.write_slice(cfg, dict(idr=int(t == 0), qp=int(seg["meta"][t, 5]), frame_num=t, idr_pic_id=0),
                         np.ascontiguousarray(seg["hdr"][t]), unpack_levels(seg, t))[0] for t in range(frames))
    assert rebuilt == s


def test_parse_matches_full_decode(host):
    w, h = 96, 64
    s = random_stream(host, w, h, 5, seed=7)
    pics = host.decode(s)
    seg = host.parse([s], 2)[0]
    nmb = (w // 16) * (h // 16)
    assert seg["hdr"].shape == (5, nmb, 64)
    for t, p in enumerate(pics):
        hd = seg["hdr"][t]
        kinds = hd[:, 0].astype(np.int8)
        assert np.array_equal(kinds, p["mb_kind"])
        assert np.array_equal(hd[:, 2].astype(np.int8), p["mb_qp"])
        mv = np.frombuffer(hd[:, 16:32].tobytes(), np.int16).reshape(nmb, 4, 2)
        dmv = p["mv"].reshape(nmb, 16, 2)
        for q, r in enumerate((0, 2, 8, 10)):
            assert np.array_equal(mv[:, q], dmv[:, r])
        assert all(seg["meta"][t, 10] == 1 for t in range(5))


def test_parse_encoder_stream_and_meta(host):
    c = yuv.synth_clip_cpu(6, 64, 48, seed=4)
    enc = host.CpuEncoder(dict(width=64, height=48, qp=30, keyint=3))
    es = enc.encode(c.i420(), c.frames, 0)
    seg = host.parse([es, es], 2)
    assert len(seg) == 2
    m = seg[0]["meta"]
    assert list(m[:, 3]) == [1, 0, 0, 1, 0, 0]            # idr
    assert list(m[:, 4] % 5) == [2, 0, 0, 2, 0, 0]        # slice types
    assert m[1, 1] == m[0, 0] and m[4, 1] == m[3, 0]       # P refs = previous picture
    assert np.array_equal(seg[0]["coef"], seg[1]["coef"])
    assert seg[0]["width"] == 64 and seg[0]["coded_height"] == 48


def test_parse_reports_errors(host):
    seg = host.parse([b"\x00\x00\x00\x01\x67garbage"], 1)[0]
    assert seg["error"] is not None or seg["n"] == 0


@pytest.mark.parametrize("cabac,rows", [(False, 2), (True, 1)])
def test_parse_multi_slice_rewrite_roundtrip(host, cabac, rows):
    """Pictures of several slices: the parsed records, rewritten slice by slice, reproduce
    the stream bit for bit; every picture stays on the GPU path and the records carry each
    MB's slice (MbHeader::pad0)."""
    w, h, frames = 96, 80, 3
    s = random_stream(host, w, h, frames, seed=31, slice_rows=rows, cabac=cabac, intra_in_p=0.3)
    seg = host.parse([s], 1)[0]
    assert seg["error"] is None and seg["n"] == frames
    assert all(seg["meta"][t, 10] == 1 for t in range(frames))
    wmb, hmb = w // 16, h // 16
    cfg = dict(width=w, height=h, qp=28, cabac=int(cabac))
    out = [host.parameter_sets(cfg)]
    for t in range(frames):
        hdr = np.ascontiguousarray(seg["hdr"][t])
        assert np.array_equal(hdr[:, 7], (np.arange(wmb * hmb) // (rows * wmb)).astype(np.uint8))
        hdr[:, 7] = 0
        fp = dict(idr=int(t == 0), qp=int(seg["meta"][t, 5]), frame_num=t, idr_pic_id=0)
        for r0 in range(0, hmb, rows):
            out.append(host.write_slice(cfg, dict(fp, first_mb=r0 * wmb, num_mbs=min(rows, hmb - r0) * wmb), hdr,
                                        unpack_levels(seg, t))[0])
    assert b"".join(out) == s
