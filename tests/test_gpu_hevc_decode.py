"""GPU HEVC decode (csrc/kernels/hevc_decode.hip) vs the CPU reconstruction of the same
parse (csrc/host/hevc_dec.cc), bit-exact, on

* streams from the GPU HEVC encoder (I / P pictures, intra NxN + DST, cu_qp_delta, SAO,
  WPP, Main and Main 10);
* streams from the syntax exerciser (csrc/host/hevc_exerciser.cc): B slices with TMVP and
  combined merge candidates, AMP, CTB 16 / 64, tiles, several slices and dependent slice
  segments, long-term references, weighted prediction, scaling lists, transform skip,
  PCM, cu_transquant_bypass, deblocking overrides (when the exerciser is built).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cpu_display(host, stream: bytes):
    pics = host.hevc_decode_full(stream, True, False)
    return sorted((p for p in pics if p["display"] >= 0), key=lambda p: p["display"])


def _check(host, streams, dec_out):
    for i, (s, d) in enumerate(zip(streams, dec_out)):
        ref = _cpu_display(host, s)
        assert d.frames == len(ref), (i, d.frames, len(ref))
        for t, p in enumerate(ref):
            x0, y0, w, h = p["crop_x"], p["crop_y"], p["width"], p["height"]
            for name, g in (("y", d.y), ("u", d.u), ("v", d.v)):
                sc = 0 if name == "y" else 1
                want = p[name][y0 >> sc:(y0 + h) >> sc, x0 >> sc:(x0 + w) >> sc]
                got = g[t].cpu().numpy().astype(np.uint16)
                if not np.array_equal(got, want):
                    diff = np.argwhere(got != want)
                    raise AssertionError(f"segment {i} picture {t} plane {name}: {len(diff)} samples differ, first "
                                         f"{diff[0].tolist()} gpu {got[tuple(diff[0])]} cpu {want[tuple(diff[0])]}")


@pytest.mark.parametrize("bd", [8, 10])
def test_gpu_hevc_decode_encoder_streams(host, bd):
    from govideocompressor_amd.models.h264_gpu import synth_clip
    from govideocompressor_amd.models.hevc_decode_gpu import GpuHevcDecoder
    from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams
    W, H, B, F = 200, 120, 3, 6
    enc = GpuHevcEncoder(HevcParams(width=W, height=H, crf=27.0, bit_depth=bd), slots=B)
    y, u, v = synth_clip(B, F, W, H, seed=21, bit_depth=bd)
    res = enc.encode(y, u, v, metrics=False)
    enc.close()
    streams = [r.bitstream for r in res]
    dec = GpuHevcDecoder().decode(streams)
    _check(host, streams, dec)
    assert dec[0].y.dtype == (torch.uint8 if bd == 8 else torch.int16)


def test_gpu_hevc_decode_intra_nxn_no_filters(host):
    from govideocompressor_amd.models.h264_gpu import synth_clip
    from govideocompressor_amd.models.hevc_decode_gpu import GpuHevcDecoder
    from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams
    enc = GpuHevcEncoder(HevcParams(width=96, height=64, crf=None, qp=24, intra_only=True, sao=False, deblock=False),
                         slots=2)
    y, u, v = synth_clip(2, 2, 96, 64, seed=8)
    res = enc.encode(y, u, v, metrics=False)
    enc.close()
    streams = [r.bitstream for r in res]
    _check(host, streams, GpuHevcDecoder().decode(streams))


def test_gpu_hevc_decode_exerciser_streams(host):
    if not hasattr(host, "hevc_exercise"):
        pytest.skip("syntax exerciser not built")
    from govideocompressor_amd.models.hevc_decode_gpu import GpuHevcDecoder
    streams = [host.hevc_exercise(seed) for seed in range(12)]
    _check(host, streams, GpuHevcDecoder().decode(streams))


@pytest.mark.parametrize("src", ["h264", "hevc"])
def test_gpu_transcoder_round_trip(host, src):
    """models/transcode.py: pieces (H.264 or HEVC) -> GPU decode -> GPU H.264 encode, three
    pieces in batches of two (the host parse of batch 2 overlaps batch 1); every output piece
    decodes (CPU decoder) to its input's frame count at a reasonable PSNR."""
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip
    from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams
    from govideocompressor_amd.models.transcode import GpuTranscoder
    W, H, F = 192, 112, 9
    y, u, v = synth_clip(3, F, W, H, seed=12)
    enc = (GpuHevcEncoder(HevcParams(width=W, height=H, crf=22.0), slots=3) if src == "hevc"
           else GpuH264Encoder(H264Params(width=W, height=H, crf=20), slots=3))
    pieces = [r.bitstream for r in enc.encode(y, u, v, metrics=False)]
    enc.close()
    tc = GpuTranscoder(H264Params(width=W, height=H, crf=18.0), slots=2)
    outs = tc.run(pieces, 30.0)
    tc.close()
    assert len(outs) == 3 and tc.timings["decode_s"] > 0
    for b, o in enumerate(outs):
        pics = host.decode(o)
        assert len(pics) == F
        got = np.stack([p["i420"][:W * H].reshape(H, W) for p in pics]).astype(np.float64)
        ref = y[b].cpu().numpy().astype(np.float64)
        mse = np.mean((got - ref) ** 2)
        assert 10 * np.log10(255 ** 2 / max(mse, 1e-9)) > 30


def test_gpu_hevc_decode_kat_streams(host):
    """Streams of the independent known-answer writer (tests/hevc_kat.py): the CPU decoder
    matches the clause formulas there (tests/test_hevc_kat.py); the GPU matches the CPU."""
    from govideocompressor_amd.models.hevc_decode_gpu import GpuHevcDecoder
    from hevc_kat import sample_streams
    from test_hevc_kat import _content
    streams = sample_streams(_content)
    _check(host, streams, GpuHevcDecoder().decode(streams))
