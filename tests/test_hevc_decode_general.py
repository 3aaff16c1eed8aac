"""General HEVC decode on the CPU (csrc/host/hevc_dec.cc) and its wiring into probe /
split / CPU transcode:

* syntax-exerciser streams (csrc/host/hevc_exerciser.cc: B slices + TMVP, AMP, CTB 16-64,
  tiles, WPP, several and dependent slice segments, long-term references, list
  modification, weighted prediction, scaling lists, transform skip, PCM,
  cu_transquant_bypass, deblocking overrides, SAO) decode, deterministically, and the
  GPU-record parse reconstructs the same samples;
* the IRAP splitter's pieces decode to exactly the pictures of the whole stream;
* ``server s`` on a ``.265`` / ``hvc1`` ``.mp4`` input writes HEVC pieces, and the CPU
  backend transcodes them (HEVC -> H.264).
"""
import numpy as np
import pytest


def _display(pics):
    return sorted((p for p in pics if p["display"] >= 0), key=lambda p: p["display"])


@pytest.mark.parametrize("seed", range(0, 48, 3))
def test_exerciser_streams_decode(host, seed):
    s = host.hevc_exercise(seed)
    a = host.hevc_decode_full(s, True, False)
    b = host.hevc_decode_full(s, True, False)
    assert len(a) >= 3
    for p, q in zip(a, b):
        assert np.array_equal(p["y"], q["y"]) and np.array_equal(p["u"], q["u"])
    info = host.hevc_stream_info(s)
    assert info["frames"] == len(a) and info["irap_frames"] == 1
    # the parse that feeds the GPU reconstructs the same pictures
    r = host.hevc_parse([s], 1, True)[0]
    assert r["n"] == len(a)
    for p, q in zip(r["pictures"], a):
        assert np.array_equal(p["y"], q["y"]) and np.array_equal(p["v"], q["v"])
    # records are self-consistent
    assert r["tu_off"][-1] == len(r["tus"]) and r["op_off"][-1] == len(r["ops"])
    assert r["coef_off"][-1] == len(r["coefs"])


def test_exerciser_covers_the_tool_set(host):
    """Across seeds the exerciser streams hit B pictures, non-32 CTBs, 10-bit and cropping."""
    ctbs, bds, types, crops = set(), set(), set(), 0
    for seed in range(40):
        pics = host.hevc_decode_full(host.hevc_exercise(seed), False, False)
        ctbs.add(pics[0]["log2_ctb"])
        bds.add(pics[0]["bit_depth"])
        types |= {p["slice_type"] for p in pics}
        crops += pics[0]["width"] != pics[0]["coded_width"] or pics[0]["height"] != pics[0]["coded_height"]
    assert ctbs == {4, 5, 6} and bds == {8, 10} and types == {0, 1, 2} and crops > 0


def test_hevc_split_pieces_decode_like_the_whole(host):
    from govideocompressor_amd.utils.hevc_synth import random_stream
    parts = [random_stream(host, 96, 64, 4, seed=70 + k, intra_in_p=0.2, mv_range=8)[0] for k in range(3)]
    whole = b"".join(parts)
    pieces = host.hevc_split_pieces(whole, 1)
    assert len(pieces) == 3
    ref = _display(host.hevc_decode_full(whole, True, False))
    got = [p for pc in pieces for p in _display(host.hevc_decode_full(pc, True, False))]
    assert len(got) == len(ref) == 12
    for p, q in zip(got, ref):
        assert np.array_equal(p["y"], q["y"])
    # min_frames groups IRAP pictures
    assert len(host.hevc_split_pieces(whole, 8)) == 2


def test_server_split_and_cpu_transcode_hevc_input(tmp_path, host):
    """``server s`` on HEVC (.265 and hvc1 .mp4) -> HEVC pieces; the CPU backend decodes them
    (hevc_dec.cc) and re-encodes H.264 (the reference worker: ffmpeg -i piece ... -vcodec libx264)."""
    from govideocompressor_amd.backends import get_backend
    from govideocompressor_amd.backends.common import PieceJob
    from govideocompressor_amd.jobs import ffargs
    from govideocompressor_amd.segment import mp4, probe as PR
    from govideocompressor_amd.segment.split import split
    from govideocompressor_amd.utils.hevc_synth import random_stream
    parts = [random_stream(host, 96, 64, 4, seed=90 + k, intra_in_p=0.2, mv_range=8)[0] for k in range(2)]
    src = tmp_path / "clip.265"
    src.write_bytes(b"".join(parts))
    info = PR.probe(str(src))
    assert (info.kind, info.codec, info.width, info.height, info.frames) == ("hevc", "hevc", 96, 64, 8)
    d, n = split(str(src), frames=4, out_root=str(tmp_path), log=lambda s: None)
    assert n == 2
    be = get_backend("cpu").impl
    job = PieceJob("0", str(tmp_path / d / "0.265"), str(tmp_path / "o0.264"), str(tmp_path / "o0.264.log"))
    res = be.transcode([job], ffargs.parse("-vcodec libx264 -qp 24"))
    assert res[0].ok, res[0].reason
    dec = host.decode((tmp_path / "o0.264").read_bytes())
    assert len(dec) == 4 and dec[0]["width"] == 96
    # MP4 (hvc1) input keeps the container per piece
    srcm = tmp_path / "clip.mp4"
    srcm.write_bytes(mp4.mux_video(b"".join(parts), 25.0, "hevc"))
    assert PR.probe(str(srcm)).codec == "hevc"
    d2, n2 = split(str(srcm), frames=4, out_root=str(tmp_path / "m"), log=lambda s: None)
    assert n2 == 2
    data = (tmp_path / "m" / d2 / "1.mp4").read_bytes()
    assert mp4.video_track(mp4.read(data)).codec in (b"hvc1", b"hev1")


@pytest.mark.parametrize("name", [f"p_bd{bd}_s{s}" for bd in (8, 10) for s in range(3)])
def test_decoder_matches_gpu_encoder_reconstruction(host, name):
    """Streams written by the GPU HEVC encoder (128x96, 5 pictures, AQ / cu_qp_delta, WPP,
    SAO, merge with 3 candidates; tools/dump_hevc_test_streams.py on an MI355X) decode to the
    encoder's own reconstruction (SHA-256 of its planes recorded with the streams).  This
    pinned the merge-candidate pruning rule (B0 / B2 are compared with availableB1, not with
    B1 after its own pruning, 8.5.3.2.3)."""
    import hashlib
    import json
    import os
    d = os.path.join(os.path.dirname(__file__), "data")
    want = json.load(open(os.path.join(d, "hevc_gpuenc_recon_sha256.json")))[name]
    s = open(os.path.join(d, f"hevc_gpuenc_{name}.265"), "rb").read()
    pics = _display(host.hevc_decode_full(s, True, False))
    planes = np.concatenate([np.concatenate([p["y"].ravel(), p["u"].ravel(), p["v"].ravel()]) for p in pics])
    assert hashlib.sha256(planes.astype(np.uint16).tobytes()).hexdigest() == want
