"""GPU H.264 reconstruction (decode.hip + deblock.hip) against the CPU decoder, bit-exact.

Streams: random decision records (every macroblock type / partition / intra mode /
QP delta the CAVLC writer produces), CPU-encoder streams with several IDR periods,
and a GPU-encoder stream; segments of different lengths and sizes decode in one call.
"""
import numpy as np
import pytest

from govideocompressor_amd.utils import yuv
from govideocompressor_amd.utils.h264_synth import random_stream

pytestmark = pytest.mark.gpu


def _planes(pic):
    w, h = pic["width"], pic["height"]
    b = pic["i420"]
    ys, cs = w * h, (w // 2) * (h // 2)
    return (b[:ys].reshape(h, w), b[ys:ys + cs].reshape(h // 2, w // 2), b[ys + cs:].reshape(h // 2, w // 2))


def _check(host, dec, streams, expect_gpu=True):
    out = dec.decode(streams)
    for i, (s, d) in enumerate(zip(streams, out)):
        ref = host.decode(s)
        assert d.frames == len(ref)
        if expect_gpu:
            assert d.path == "gpu", f"segment {i} fell back to the CPU decoder"
        y, u, v = d.y.cpu().numpy(), d.u.cpu().numpy(), d.v.cpu().numpy()
        for t, p in enumerate(ref):
            ry, ru, rv = _planes(p)
            for name, a, b in (("y", y[t], ry), ("u", u[t], ru), ("v", v[t], rv)):
                if not np.array_equal(a, b):
                    diff = np.argwhere(a != b)
                    raise AssertionError(f"segment {i} picture {t} plane {name}: {len(diff)} samples differ, "
                                         f"first at {diff[0].tolist()} (gpu {a[tuple(diff[0])]}, cpu {b[tuple(diff[0])]})")
    return out


@pytest.fixture(scope="module")
def dec():
    from govideocompressor_amd.models.h264_decode_gpu import GpuH264Decoder
    return GpuH264Decoder()


def test_gpu_decode_random_records(host, dec):
    streams = [random_stream(host, 96, 64, 6, seed=11),
               random_stream(host, 96, 64, 3, seed=12, intra_in_p=0.3),
               random_stream(host, 96, 64, 5, seed=13, density=0.4, mv_range=200),
               random_stream(host, 96, 64, 7, seed=14, keyint=3)]
    _check(host, dec, streams)


def test_gpu_decode_cropped_and_mixed_sizes(host, dec):
    streams = [random_stream(host, 50, 34, 4, seed=21), random_stream(host, 176, 144, 3, seed=22),
               random_stream(host, 50, 34, 2, seed=23)]
    _check(host, dec, streams)


def test_gpu_decode_encoder_streams(host, dec):
    streams = []
    for k, (w, h, qp) in enumerate([(176, 144, 22), (176, 144, 34), (176, 144, 28)]):
        c = yuv.synth_clip_cpu(8, w, h, seed=30 + k)
        enc = host.CpuEncoder(dict(width=w, height=h, qp=qp, keyint=4))
        streams.append(enc.encode(c.i420(), c.frames, k))
    # a deblocking-disabled stream lands in its own batch
    c = yuv.synth_clip_cpu(4, 176, 144, seed=40)
    streams.append(host.CpuEncoder(dict(width=176, height=144, qp=30, deblock=0)).encode(c.i420(), 4, 0))
    _check(host, dec, streams)


def _gpu_encoder_streams(**kw):
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip
    enc = GpuH264Encoder(H264Params(width=320, height=240, crf=23, **kw), slots=3)
    y, u, v = synth_clip(3, 10, 320, 240, seed=5)
    res = enc.encode(y, u, v, metrics=False)
    streams = [r.bitstream for r in res]
    enc.close()
    torch.cuda.synchronize()
    return streams


def test_gpu_decode_gpu_encoder_stream(host, dec):
    # Constrained Baseline CAVLC (the round-1 encoder): P pictures, one reference
    _check(host, dec, _gpu_encoder_streams(cabac=False))


def test_gpu_decode_gpu_encoder_cabac_b_stream(host, dec):
    # the default encoder (Main CABAC + 3 B, temporal direct): B pictures from the DPB,
    # output in display order
    _check(host, dec, _gpu_encoder_streams())


def test_gpu_decode_multiref_high_cabac(host, dec):
    """CABAC streams with up to 4 references per P picture (per-partition ref_idx), 8x8
    transforms on inter MBs and Intra8x8 MBs (High profile)."""
    streams = [random_stream(host, 96, 64, 7, seed=31, cabac=True, refs=3),
               random_stream(host, 96, 64, 6, seed=32, cabac=True, refs=4, t8x8=True),
               random_stream(host, 176, 144, 5, seed=33, cabac=True, t8x8=True, intra_in_p=0.3),
               random_stream(host, 50, 34, 6, seed=34, cabac=True, refs=2, t8x8=True, keyint=3)]
    out = _check(host, dec, streams)
    assert dec.stats["segments_cpu"] == 0


def test_gpu_decode_b_records(host, dec):
    """B pictures with L0 / L1 / bi-predicted 16x16 MBs, direct and skipped MBs."""
    from tests.test_h264_bframes import _b_stream
    streams = [_b_stream(host, w, h, seed)[0] for w, h, seed in ((64, 48, 1), (96, 80, 2), (176, 144, 3))]
    _check(host, dec, streams)


def test_gpu_decode_multi_slice_pictures(host, dec):
    """Pictures coded as several slices (2-row / 1-row slices, CAVLC and CABAC, High 8x8
    with Intra8x8) reconstruct on the GPU: intra prediction treats MBs of another slice as
    unavailable (MbHeader::pad0 carries the slice), deblocking filters across the slices."""
    streams = [random_stream(host, 96, 64, 4, seed=61, slice_rows=2, intra_in_p=0.3),
               random_stream(host, 112, 80, 4, seed=62, slice_rows=1, cabac=True, t8x8=True, intra_in_p=0.4),
               random_stream(host, 96, 64, 3, seed=63, slice_rows=3, cabac=True)]
    _check(host, dec, streams)


def test_gpu_decode_pcm_constrained_intra_scaling_lists(host, dec):
    """Coding tools that used to drop a segment to the CPU decoder now reconstruct on the GPU:
    I_PCM macroblocks (samples through the level pool, deblocking QP 0), constrained intra
    prediction (inter neighbours unavailable to intra MBs of P pictures), and scaling matrices
    (SPS lists; PPS lists with fall-back rule B; CAVLC and CABAC; 4x4 and 8x8)."""
    rng = np.random.default_rng(5)
    cqm4 = rng.integers(6, 60, (6, 16)).astype(np.uint8)
    cqm8 = rng.integers(6, 60, (2, 64)).astype(np.uint8)
    streams = [random_stream(host, 96, 64, 5, seed=31, pcm=0.25, intra_in_p=0.3),
               random_stream(host, 96, 64, 5, seed=32, constrained_intra=True, intra_in_p=0.4, density=0.3),
               random_stream(host, 96, 64, 5, seed=33, t8x8=True, cqm=dict(cqm=1, cqm4=cqm4, cqm8=cqm8), density=0.3),
               random_stream(host, 96, 64, 5, seed=34, t8x8=True, cabac=True, intra_in_p=0.3,
                             cqm=dict(cqm=3, cqm4=cqm4, cqm8=cqm8, cqm_coded=0x5A), density=0.3)]
    _check(host, dec, streams)


def test_gpu_decode_high10_segments(host, dec):
    """High 10 segments (the CPU decoder's 16-bit path) come back as int16 planes of the
    decoded samples next to 8-bit segments reconstructed on the GPU in the same call, and a
    transcode of High 10 pieces (models/transcode.py) rounds them to the 8-bit encoder's input."""
    import torch
    from govideocompressor_amd.models.h264_gpu import H264Params
    from govideocompressor_amd.models.transcode import GpuTranscoder
    s10 = random_stream(host, 96, 64, 4, seed=71, bit_depth=10, intra_in_p=0.3, t8x8=True, cabac=True)
    s8 = random_stream(host, 96, 64, 4, seed=72)
    out = dec.decode([s10, s8])
    assert out[0].path == "cpu" and out[0].bit_depth == 10 and out[0].y.dtype == torch.int16
    assert out[1].path == "gpu"
    for t, p in enumerate(host.decode(s10)):
        ry, ru, rv = _planes(p)
        assert np.array_equal(out[0].y[t].cpu().numpy(), ry.astype(np.int16))
        assert np.array_equal(out[0].u[t].cpu().numpy(), ru.astype(np.int16))
        assert np.array_equal(out[0].v[t].cpu().numpy(), rv.astype(np.int16))
    tc = GpuTranscoder(H264Params(width=96, height=64, crf=20.0), slots=2)
    outs = tc.run([s10, s10], 30.0)
    tc.close()
    assert [len(host.decode(o)) for o in outs] == [4, 4]


def test_gpu_decode_high12_to_main10(host):
    """A 12-bit High 10-family segment feeding a Main 10 output (keep_high_bit) is rescaled to
    10 bits with rounding (DecodedSegment.bit_depth 10) instead of reaching the encoder unscaled;
    a 10-bit segment passes through untouched."""
    import torch
    from govideocompressor_amd.backends.gpu import GpuBackend
    s12 = random_stream(host, 96, 64, 3, seed=81, bit_depth=12, intra_in_p=0.3, cabac=True)
    s10 = random_stream(host, 96, 64, 3, seed=82, bit_depth=10, intra_in_p=0.3, cabac=True)
    b = GpuBackend()
    out = b.decode_streams([s12, s10], 30.0, keep_high_bit=True)
    assert out[0].bit_depth == 10 and out[0].y.dtype == torch.int16
    for t, p in enumerate(host.decode(s12)):
        ry, ru, rv = _planes(p)
        for got, ref in ((out[0].y[t], ry), (out[0].u[t], ru), (out[0].v[t], rv)):
            want = np.clip((ref.astype(np.int32) + 2) >> 2, 0, 1023)
            assert np.array_equal(got.cpu().numpy().astype(np.int32), want)
    for t, p in enumerate(host.decode(s10)):
        assert np.array_equal(out[1].y[t].cpu().numpy(), _planes(p)[0].astype(np.int16))
