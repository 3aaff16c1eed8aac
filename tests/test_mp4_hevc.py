"""HEVC MP4 container: Annex-B HEVC pieces -> ``hvc1``/``hvcC`` MP4 and
back, checked through the independent host HEVC decoder; merge of HEVC ``.mp4`` pieces.
The reference writes every piece as ``<idx>.mp4`` (client.go:54) whatever the codec."""
import os
import struct

import numpy as np
import pytest

from govideocompressor_amd.segment import merge, mp4_hevc
from govideocompressor_amd.utils.hevc_synth import random_stream


def _same_pics(a, b):
    assert len(a) == len(b)
    for p, q in zip(a, b):
        assert p["poc"] == q["poc"] and p["idr"] == q["idr"]
        for k in ("y", "u", "v"):
            assert np.array_equal(p[k], q[k])


@pytest.mark.parametrize("w,h,bd,wpp", [(64, 64, 8, 0), (80, 48, 10, 0), (160, 96, 8, 1)])
def test_hevc_mp4_roundtrip(host, w, h, bd, wpp):
    s, _ = random_stream(host, w, h, 3, seed=11, bit_depth=bd, host_cfg=dict(wpp=wpp, threads=2) if wpp else None)
    assert mp4_hevc.is_hevc_annexb(s)
    m = mp4_hevc.mux(s, 25.0)
    assert m[4:8] == b"ftyp" and mp4_hevc.is_hevc_mp4(m)
    info = mp4_hevc.parse_sps(mp4_hevc.split_nals(s)[1])
    assert (info["width"], info["height"], info["bit_depth_luma"]) == (w, h, bd)
    # hvcC: profile/level copied from the SPS, 4-byte NAL lengths, VPS+SPS+PPS arrays
    i = m.index(b"hvcC") + 4
    assert m[i] == 1 and m[i + 21] & 3 == 3 and m[i + 22] == 3 and m[i + 17] & 7 == bd - 8
    # 3 samples, the first (IDR) is the only sync sample
    st = m.index(b"stss") + 4
    assert struct.unpack(">II", m[st + 4:st + 12]) == (1, 1)
    back = mp4_hevc.demux(m)
    _same_pics(host.hevc_decode(back), host.hevc_decode(s))


def _hevc_stream(host, w, h, n):
    return random_stream(host, w, h, n, seed=5)[0]


def test_h264_streams_not_taken_for_hevc(host):
    assert not mp4_hevc.is_hevc_annexb(host.parameter_sets(dict(width=64, height=48)))
    assert not mp4_hevc.is_hevc_annexb(b"\x00\x00\x00\x01\x67\x42\xc0\x1e" + bytes(16))
    assert not mp4_hevc.is_hevc_annexb(b"\x00\x00\x00\x01\x09\xf0")
    assert not mp4_hevc.is_hevc_annexb(b"\x00\x00\x00\x01\x41\x9a\x02\x10")  # H.264 P slice (nal_ref_idc 2)


def test_hevc_mp4_merge(host, tmp_path):
    pieces = []
    ref = []
    for k in range(3):
        s, _ = random_stream(host, 64, 48, 2, seed=20 + k)
        p = tmp_path / f"{k}.mp4"
        p.write_bytes(mp4_hevc.mux(s, 30.0))
        pieces.append(str(p))
        ref += host.hevc_decode(s)
    merge.make_filelist(3, str(tmp_path))
    out = merge.merge_dir(str(tmp_path))
    data = open(out, "rb").read()
    assert mp4_hevc.is_hevc_mp4(data)
    pics = host.hevc_decode(mp4_hevc.demux(data))
    assert len(pics) == 6
    for p, q in zip(pics, ref):
        assert np.array_equal(p["y"], q["y"])
    assert os.path.getsize(out) == len(data)


def test_merge_keeps_piece_frame_rate(host, tmp_path):
    """merged HEVC .mp4 takes the pieces' mdhd/stts rate (not a 30 fps default)."""
    from govideocompressor_amd.segment import merge, mp4_hevc
    stream = _hevc_stream(host, 64, 64, 3)
    paths = []
    for i in range(2):
        p = tmp_path / f"{i}.mp4"
        p.write_bytes(mp4_hevc.mux(stream, 25.0))
        paths.append(str(p))
    out = tmp_path / "out.mp4"
    merge.merge_files(paths, str(out))
    data = out.read_bytes()
    assert abs(mp4_hevc.track_fps(data) - 25.0) < 1e-6


def test_mux_suffix_nals_and_trailing(host):
    """Suffix SEI / EOS stay with the picture they follow; a stray slice before any picture
    start is rejected."""
    from govideocompressor_amd.segment import mp4_hevc
    stream = _hevc_stream(host, 64, 64, 2)
    sei_suffix = b"\x00\x00\x00\x01" + bytes([40 << 1, 1]) + b"\x05\x01\xaa\x80"
    eos = b"\x00\x00\x00\x01" + bytes([36 << 1, 1])
    data = mp4_hevc.mux(stream + sei_suffix + eos, 30.0)
    back = mp4_hevc.demux(data)
    assert back.endswith(sei_suffix[4:] + b"\x00\x00\x00\x01" + eos[4:])
    nals = mp4_hevc.split_nals(stream)
    vcl = [n for n in nals if ((n[0] >> 1) & 0x3F) < 32]
    bad = b"\x00\x00\x00\x01" + vcl[0][:2] + bytes([vcl[0][2] & 0x7F]) + vcl[0][3:]
    import pytest
    with pytest.raises(ValueError):
        mp4_hevc.mux(b"".join(b"\x00\x00\x00\x01" + n for n in nals if ((n[0] >> 1) & 0x3F) >= 32) + bad, 30.0)


def test_merge_rejects_mixed_codecs(host, tmp_path):
    from govideocompressor_amd.segment import merge
    hevc = _hevc_stream(host, 64, 64, 2)
    h264 = host.parameter_sets(dict(width=64, height=64))
    a, b = tmp_path / "0.264", tmp_path / "1.264"
    a.write_bytes(hevc)
    b.write_bytes(h264)
    import pytest
    with pytest.raises(ValueError, match="mix codecs"):
        merge.merge_files([str(a), str(b)], str(tmp_path / "o.264"))


def test_probe_annexb_of_hevc_mp4(host, tmp_path):
    from govideocompressor_amd.segment import mp4_hevc, probe
    stream = _hevc_stream(host, 64, 64, 2)
    p = tmp_path / "x.mp4"
    p.write_bytes(mp4_hevc.mux(stream, 30.0))
    assert mp4_hevc.is_hevc_annexb(probe.annexb_of(str(p)))
