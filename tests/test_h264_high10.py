"""High 10 H.264 decode (CPU decoder, csrc/host/h264_decoder.cc): 9..14-bit 4:2:0 streams
written by the host record writer (profile_idc 110, bit_depth_*_minus8, PCM samples of
BitDepth bits, QPs down to -QpBdOffsetY).

No High 10 decoder exists in this image to compare against (no ffmpeg), so the checks are
analytic, from the clauses rather than from the decoder's code paths:

* I_PCM samples come back exactly (7.3.5 pcm_sample_* of BitDepth bits);
* zero-residual P pictures equal a numpy model of the quarter-sample interpolation
  (8.4.2.2.1 / 8.4.2.2.2, Clip1 at 2^BitDepth - 1) and of explicit weighted prediction with
  offsets scaled by 2^(BitDepth - 8) (8.4.2.3.2), at QP < 0 where the loop filter is a no-op;
* Intra16x16 DC-only macroblocks equal a model of 8.3.3 (DC default 2^(BitDepth-1)) and 8.5.10
  with QP'Y = QPY + QpBdOffsetY;
* random High 10 streams (every MB type, CAVLC and CABAC, deblocking on) decode within
  [0, 2^BitDepth) and are flagged for the CPU path of the batched GPU decoder.

Parity with another decoder beyond these is unpinned.
"""
import numpy as np
import pytest

from govideocompressor_amd.utils.h264_synth import HDR_BYTES, random_stream

_KIND, _QP, _I16, _REF, _MV = 0, 2, 3, 8, 16
IPCM, I16x16, P16x16 = 4, 1, 2
_ZZ4 = [0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15]


def _pcm_picture(rng, wmb, hmb, bd):
    """Records of an all-I_PCM picture and the planes they code."""
    nmb = wmb * hmb
    hdr = np.zeros((nmb, HDR_BYTES), np.uint8)
    hdr[:, _KIND] = IPCM
    hdr[:, _REF:_REF + 8] = 0xFF
    coef = np.zeros((nmb, 408), np.int16)
    Y = np.zeros((hmb * 16, wmb * 16), np.int64)
    U = np.zeros((hmb * 8, wmb * 8), np.int64)
    V = np.zeros_like(U)
    for mb in range(nmb):
        mx, my = mb % wmb, mb // wmb
        s = rng.integers(0, 1 << bd, 384)
        coef[mb, :384] = s
        Y[my * 16:my * 16 + 16, mx * 16:mx * 16 + 16] = s[:256].reshape(16, 16)
        U[my * 8:my * 8 + 8, mx * 8:mx * 8 + 8] = s[256:320].reshape(8, 8)
        V[my * 8:my * 8 + 8, mx * 8:mx * 8 + 8] = s[320:].reshape(8, 8)
    return hdr, coef, (Y, U, V)


def _tap(a, b, c, d, e, f):
    return a - 5 * b + 20 * c + 20 * d - 5 * e + f


def _luma_mc(ref, X0, Y0, mvx, mvy, bd):
    """16x16 luma prediction block at (X0, Y0) displaced by a quarter-sample vector (8.4.2.2.1)."""
    H, W = ref.shape
    mx = (1 << bd) - 1

    def G(x, y):
        return int(ref[min(max(y, 0), H - 1), min(max(x, 0), W - 1)])

    def clip(v):
        return min(max(v, 0), mx)

    def b1(x, y):
        return _tap(*(G(x + k, y) for k in range(-2, 4)))

    def b(x, y):
        return clip((b1(x, y) + 16) >> 5)

    def h(x, y):
        return clip((_tap(*(G(x, y + k) for k in range(-2, 4))) + 16) >> 5)

    def j(x, y):
        return clip((_tap(*(b1(x, y + k) for k in range(-2, 4))) + 512) >> 10)

    xf, yf = mvx & 3, mvy & 3
    out = np.zeros((16, 16), np.int64)
    for yy in range(16):
        for xx in range(16):
            x, y = X0 + xx + (mvx >> 2), Y0 + yy + (mvy >> 2)
            g = G(x, y)
            # Table 8-12: (xFrac, yFrac) -> sample; m = h one column right, s = b one row down
            v = {(0, 0): lambda: g, (0, 1): lambda: (g + h(x, y) + 1) >> 1, (0, 2): lambda: h(x, y),
                 (0, 3): lambda: (G(x, y + 1) + h(x, y) + 1) >> 1, (1, 0): lambda: (g + b(x, y) + 1) >> 1,
                 (1, 1): lambda: (b(x, y) + h(x, y) + 1) >> 1, (1, 2): lambda: (h(x, y) + j(x, y) + 1) >> 1,
                 (1, 3): lambda: (h(x, y) + b(x, y + 1) + 1) >> 1, (2, 0): lambda: b(x, y),
                 (2, 1): lambda: (b(x, y) + j(x, y) + 1) >> 1, (2, 2): lambda: j(x, y),
                 (2, 3): lambda: (j(x, y) + b(x, y + 1) + 1) >> 1, (3, 0): lambda: (G(x + 1, y) + b(x, y) + 1) >> 1,
                 (3, 1): lambda: (b(x, y) + h(x + 1, y) + 1) >> 1, (3, 2): lambda: (j(x, y) + h(x + 1, y) + 1) >> 1,
                 (3, 3): lambda: (h(x + 1, y) + b(x, y + 1) + 1) >> 1}[(xf, yf)]()
            out[yy, xx] = v
    return out


def _chroma_mc(ref, X0, Y0, mvx, mvy):
    """8x8 chroma block (4:2:0: the luma vector in eighth chroma samples, 8.4.2.2.2)."""
    H, W = ref.shape
    xf, yf = mvx & 7, mvy & 7

    def P(x, y):
        return int(ref[min(max(y, 0), H - 1), min(max(x, 0), W - 1)])

    out = np.zeros((8, 8), np.int64)
    for yy in range(8):
        for xx in range(8):
            x, y = X0 + xx + (mvx >> 3), Y0 + yy + (mvy >> 3)
            out[yy, xx] = ((8 - xf) * (8 - yf) * P(x, y) + xf * (8 - yf) * P(x + 1, y) + (8 - xf) * yf * P(x, y + 1) +
                           xf * yf * P(x + 1, y + 1) + 32) >> 6
    return out


def _weigh(p, w, o, logwd, bd):
    o = o << (bd - 8)
    v = ((p * w + (1 << (logwd - 1))) >> logwd) + o if logwd >= 1 else p * w + o
    return np.clip(v, 0, (1 << bd) - 1)


def _planes(pic):
    return [np.asarray(pic[k]).astype(np.int64) for k in ("y_coded", "u_coded", "v_coded")]


@pytest.mark.parametrize("bd", [9, 10, 12])
@pytest.mark.parametrize("wp", [None, [5, 4, 40, -7, 21, 3, 13, -2]])
def test_high10_pcm_and_motion_compensation(host, bd, wp):
    """I_PCM picture, then a P picture of P_L0_16x16 MBs without residual at QP -QpBdOffsetY
    (the loop filter's indexA clips to 0: alpha = 0 filters nothing)."""
    rng = np.random.default_rng(bd)
    w, h, wmb, hmb = 64, 48, 4, 3
    cfg = dict(width=w, height=h, bit_depth=bd, weightp=int(wp is not None))
    qmin = -6 * (bd - 8)
    hdr0, coef0, ref = _pcm_picture(rng, wmb, hmb, bd)
    nal0, _ = host.write_slice(cfg, dict(idr=1, qp=qmin, frame_num=0), hdr0, coef0)
    nmb = wmb * hmb
    hdr1 = np.zeros((nmb, HDR_BYTES), np.uint8)
    hdr1[:, _KIND] = P16x16
    hdr1[:, _QP] = qmin & 0xFF
    hdr1[:, _REF:_REF + 8] = 0xFF
    hdr1[:, _REF:_REF + 4] = 0
    mvs = rng.integers(-23, 24, (nmb, 2))
    mv4 = np.repeat(mvs[:, None, :], 4, axis=1).astype(np.int16)
    hdr1[:, _MV:_MV + 16] = np.frombuffer(mv4.tobytes(), np.uint8).reshape(nmb, 16)
    fp = dict(idr=0, qp=qmin, frame_num=1)
    if wp is not None:
        fp["wp"] = wp
    nal1, _ = host.write_slice(cfg, fp, hdr1, np.zeros((nmb, 408), np.int16))
    pics = host.decode(host.parameter_sets(cfg) + nal0 + nal1)
    assert len(pics) == 2 and pics[0]["bit_depth"] == bd
    for got, want in zip(_planes(pics[0]), ref):
        np.testing.assert_array_equal(got, want)
    Y, U, V = ref
    for mb in range(nmb):
        mx, my = mb % wmb, mb // wmb
        vx, vy = int(mvs[mb, 0]), int(mvs[mb, 1])
        py = _luma_mc(Y, mx * 16, my * 16, vx, vy, bd)
        pu = _chroma_mc(U, mx * 8, my * 8, vx, vy)
        pv = _chroma_mc(V, mx * 8, my * 8, vx, vy)
        if wp is not None:
            py = _weigh(py, wp[2], wp[3], wp[0], bd)
            pu = _weigh(pu, wp[4], wp[5], wp[1], bd)
            pv = _weigh(pv, wp[6], wp[7], wp[1], bd)
        gy, gu, gv = _planes(pics[1])
        np.testing.assert_array_equal(gy[my * 16:my * 16 + 16, mx * 16:mx * 16 + 16], py, err_msg=f"MB {mb} luma")
        np.testing.assert_array_equal(gu[my * 8:my * 8 + 8, mx * 8:mx * 8 + 8], pu, err_msg=f"MB {mb} Cb")
        np.testing.assert_array_equal(gv[my * 8:my * 8 + 8, mx * 8:mx * 8 + 8], pv, err_msg=f"MB {mb} Cr")


def test_high10_intra16x16_dc_scaling(host):
    """Intra16x16 DC prediction with luma DC levels only, per-MB QPs from -12 to 40:
    8.3.3.3 (DC of the neighbours, 512 without any) + 8.5.10 at QP'Y = QPY + 12 + 8.5.12
    (a DC-only 4x4 block adds (dcY + 32) >> 6 to every sample), clipped to 1023."""
    bd = 10
    rng = np.random.default_rng(5)
    w, h, wmb, hmb = 48, 32, 3, 2
    nmb = wmb * hmb
    hdr = np.zeros((nmb, HDR_BYTES), np.uint8)
    hdr[:, _KIND] = I16x16
    hdr[:, _I16] = 2
    hdr[:, _REF:_REF + 8] = 0xFF
    hdr[:, 48:64] = 2
    qps = np.array([-12, -5, 0, 17, 33, 40])
    hdr[:, _QP] = qps & 0xFF
    coef = np.zeros((nmb, 408), np.int16)
    coef[:, 256:272] = rng.integers(-40, 41, (nmb, 16))
    coef[0, 256] = 900  # drives the first MB into the 1023 clip
    cfg = dict(width=w, height=h, bit_depth=bd, deblock=0)
    nal, _ = host.write_slice(cfg, dict(idr=1, qp=qps[0], frame_num=0), hdr, coef)
    pics = host.decode(host.parameter_sets(cfg) + nal)
    got = _planes(pics[0])[0]
    A = np.array([[1, 1, 1, 1], [1, 1, -1, -1], [1, -1, -1, 1], [1, -1, 1, -1]])
    v0 = [10, 11, 13, 14, 16, 18]
    Y = np.zeros((h, w), np.int64)
    for mb in range(nmb):
        mx, my = mb % wmb, mb // wmb
        X0, Y0 = mx * 16, my * 16
        top = Y[Y0 - 1, X0:X0 + 16] if my else None
        left = Y[Y0:Y0 + 16, X0 - 1] if mx else None
        if top is not None and left is not None:
            pred = (top.sum() + left.sum() + 16) >> 5
        elif left is not None:
            pred = (left.sum() + 8) >> 4
        elif top is not None:
            pred = (top.sum() + 8) >> 4
        else:
            pred = 1 << (bd - 1)
        c = np.zeros(16, np.int64)
        c[_ZZ4] = coef[mb, 256:272]
        F = A @ c.reshape(4, 4) @ A
        qp = int(qps[mb]) + 6 * (bd - 8)
        ls = 16 * v0[qp % 6]
        for by in range(4):
            for bx in range(4):
                f = int(F[by, bx])
                dc = (f * ls) << (qp // 6 - 6) if qp >= 36 else (f * ls + (1 << (5 - qp // 6))) >> (6 - qp // 6)
                Y[Y0 + by * 4:Y0 + by * 4 + 4, X0 + bx * 4:X0 + bx * 4 + 4] = np.clip(pred + ((dc + 32) >> 6), 0, 1023)
    np.testing.assert_array_equal(got, Y)
    assert got.max() == 1023


@pytest.mark.parametrize("cabac", [False, True])
def test_high10_random_streams_decode(host, cabac):
    """Every MB type, partitions, residual and deblocking at QPs on both sides of 0: the
    stream decodes, samples stay inside 10 bits, the batched decoder's parse flags the
    pictures for its CPU path (the GPU reconstruction kernels are 8-bit)."""
    kw = dict(frames=5, seed=41, cabac=cabac, t8x8=True, intra_in_p=0.3, bit_depth=10)
    if not cabac:
        kw["pcm"] = 0.05
    for qp in (2, 30):
        s = random_stream(host, 80, 48, qp=qp, **kw)
        pics = host.decode(s)
        assert len(pics) == 5
        for p in pics:
            assert p["bit_depth"] == 10 and p["y_coded"].dtype == np.uint16
            assert int(p["y_coded"].max()) <= 1023 and int(p["u_coded"].max()) <= 1023
        assert min(int(np.min(p["mb_qp"])) for p in pics) < 0 if qp == 2 else True
        again = host.decode(s)
        assert all(np.array_equal(a["i420"], b["i420"]) for a, b in zip(pics, again))
        seg = host.parse([s])[0]
        assert not np.all(seg["meta"][:, 10] == 1)  # gpu_ok column (models/h264_decode_gpu.py _META)


def test_mixed_luma_chroma_depth_refused(host):
    """BitDepthC != BitDepthY is refused at the SPS (the picture records carry one depth; the
    old path emitted an empty 8-bit plane set for bdY 8 / bdC 10 and mis-scaled chroma)."""
    from govideocompressor_amd.utils.h264_synth import random_stream
    ok = random_stream(host, 32, 32, 1, seed=3, bit_depth=10)
    ps_ok = host.parameter_sets(dict(width=32, height=32, bit_depth=10))
    assert ok.startswith(ps_ok)
    bad = host.parameter_sets(dict(width=32, height=32, bit_depth=10, bit_depth_chroma=12)) + ok[len(ps_ok):]
    with pytest.raises(Exception, match="bit depths differ"):
        host.decode(bad)
    assert len(host.decode(ok)) == 1


def test_rescale_bits_model():
    from govideocompressor_amd.utils import yuv
    a = np.array([0, 1, 2, 3, 4095, 2048], np.int16)
    assert yuv.rescale_bits(a, 12, 10).tolist() == [0, 0, 1, 1, 1023, 512]
    assert yuv.rescale_bits(np.array([0, 511, 300], np.int16), 9, 10).tolist() == [0, 1022, 600]
    assert yuv.rescale_bits(a, 10, 10) is a
