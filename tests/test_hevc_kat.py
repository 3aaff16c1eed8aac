"""Known-answer tests of the HEVC decoder (csrc/host/hevc_dec.cc), independent of its code.

The streams come from tests/hevc_kat.py, a small writer that shares nothing with the repo's
C++ (own CABAC encoder, own context init values, own syntax); the expected pictures are
computed here from the clause formulas of ITU-T H.265:

* PCM CUs reproduce their samples exactly (7.3.8.7, 8.4.4.2.7) -- the writer's self-check;
* fractional luma / chroma interpolation with reference padding (8.5.3.3.3.1 / .3.3.3.2);
* explicit weighted prediction: luma / chroma weights, the chroma offset derivation of 7.4.7.3
  and the rounding of 8.5.3.3.4.3 at 8 and 10 bits;
* TMVP motion scaling (8.5.3.2.8: tx, distScaleFactor, rounding) through a merge candidate;
* merge candidates of the second PU of AMP / symmetric partitions (8.5.3.2.3: A1 or B1 of
  the first PU excluded);
* dequantisation with explicit scaling lists, including the 16x16 DC coefficient
  (7.3.4 / 7.4.5, 8.6.2 - 8.6.4).

CPU decoder only; the GPU reconstruction is compared with the CPU decoder elsewhere
(tests/test_gpu_hevc_decode.py)."""
import numpy as np
import pytest

from hevc_kat import DEFAULT_8x8_INTER, KatStream

FL = {1: [-1, 4, -10, 58, 17, -5, 1, 0], 2: [-1, 4, -11, 40, 40, -11, 4, -1], 3: [0, 1, -5, 17, 58, -10, 4, -1]}
FC = {1: [-2, 58, 10, -2], 2: [-4, 54, 16, -2], 3: [-6, 46, 28, -4], 4: [-4, 36, 36, -4], 5: [-4, 28, 46, -6],
      6: [-2, 16, 54, -4], 7: [-2, 10, 58, -2]}


def _content(w, h, bd, seed):
    r = np.random.default_rng(seed)
    hi = (1 << bd) - 1
    yy, xx = np.mgrid[0:h, 0:w]
    y = (hi * (0.5 + 0.35 * np.sin(xx / 3.1 + yy / 5.3))).astype(np.int64) + r.integers(-hi // 16, hi // 16, (h, w))
    u = r.integers(0, hi + 1, (h // 2, w // 2))
    v = (hi - u // 2 + r.integers(-8, 8, (h // 2, w // 2))).clip(0, hi)
    return y.clip(0, hi), u, v


def _decode(host, data):
    pics = host.hevc_decode_full(data, True, False)
    pics = sorted((p for p in pics if p["display"] >= 0), key=lambda p: p["display"])
    return [(p["y"].astype(np.int64), p["u"].astype(np.int64), p["v"].astype(np.int64)) for p in pics]


def _pred(ref, x0, y0, w, h, mv, chroma, bd):
    """8.5.3.3.3: fractional sample interpolation of one block -> 14-bit intermediate samples."""
    H, W = ref.shape
    shift1, shift2, shift3 = min(4, bd - 8), 6, 14 - bd
    if chroma:
        fx, fy, filt, taps = mv[0] & 7, mv[1] & 7, FC, 4
        ix, iy = x0 + (mv[0] >> 3), y0 + (mv[1] >> 3)
    else:
        fx, fy, filt, taps = mv[0] & 3, mv[1] & 3, FL, 8
        ix, iy = x0 + (mv[0] >> 2), y0 + (mv[1] >> 2)
    half = taps // 2 - 1

    def at(x, y):
        return ref[np.clip(y, 0, H - 1)][:, np.clip(x, 0, W - 1)]

    xs, ys = np.arange(w) + ix, np.arange(h) + iy
    if fx == 0 and fy == 0:
        return at(xs, ys) << shift3
    if fy == 0:
        return sum(filt[fx][i] * at(xs + i - half, ys) for i in range(taps)) >> shift1
    if fx == 0:
        return sum(filt[fy][i] * at(xs, ys + i - half) for i in range(taps)) >> shift1
    tmp = [sum(filt[fx][i] * at(xs + i - half, ys + n - half) for i in range(taps)) >> shift1 for n in range(taps)]
    return sum(filt[fy][n] * tmp[n] for n in range(taps)) >> shift2


def _default_weighted(p, bd):
    s = 14 - bd
    return np.clip((p + (1 << (s - 1))) >> s, 0, (1 << bd) - 1)


def _explicit_weighted(p, bd, log2wd_denom, w, o):
    """8.5.3.3.4.3, uni-prediction."""
    log2wd = log2wd_denom + 14 - bd
    o = o << (bd - 8)
    if log2wd >= 1:
        r = ((p * w + (1 << (log2wd - 1))) >> log2wd) + o
    else:
        r = p * w + o
    return np.clip(r, 0, (1 << bd) - 1)


def _predict_picture(ref, mv_of_block, bd, blocks, weights=None):
    """blocks: list of (x, y, w, h) luma PBs with their mv; weights: None or
    ((denom, w, o), (cdenom, [(cw, co)] * 2))."""
    ry, ru, rv = ref
    oy, ou, ov = np.zeros_like(ry), np.zeros_like(ru), np.zeros_like(rv)
    for (x, y, w, h), mv in zip(blocks, mv_of_block):
        py = _pred(ry, x, y, w, h, mv, False, bd)
        pu = _pred(ru, x // 2, y // 2, w // 2, h // 2, mv, True, bd)
        pv = _pred(rv, x // 2, y // 2, w // 2, h // 2, mv, True, bd)
        if weights is None:
            oy[y:y + h, x:x + w] = _default_weighted(py, bd)
            ou[y // 2:(y + h) // 2, x // 2:(x + w) // 2] = _default_weighted(pu, bd)
            ov[y // 2:(y + h) // 2, x // 2:(x + w) // 2] = _default_weighted(pv, bd)
        else:
            (d, lw, lo), (cd, cw) = weights
            oy[y:y + h, x:x + w] = _explicit_weighted(py, bd, d, lw, lo)
            ou[y // 2:(y + h) // 2, x // 2:(x + w) // 2] = _explicit_weighted(pu, bd, cd, *cw[0])
            ov[y // 2:(y + h) // 2, x // 2:(x + w) // 2] = _explicit_weighted(pv, bd, cd, *cw[1])
    return oy, ou, ov


def _assert_pic(got, want):
    for g, w_, name in zip(got, want, "yuv"):
        assert g.shape == w_.shape, name
        bad = np.argwhere(g != w_)
        assert bad.size == 0, f"{name}: {len(bad)} samples differ, first at {tuple(bad[0])}: {g[tuple(bad[0])]} != {w_[tuple(bad[0])]}"


@pytest.mark.parametrize("bd,ctb", [(8, 4), (10, 5), (8, 6)])
def test_kat_pcm_pictures_are_exact(host, bd, ctb):
    w, h = 2 << ctb, 1 << ctb
    y, u, v = _content(w, h, bd, 1)
    s = KatStream(w, h, bit_depth=bd, ctb_log2=ctb)
    s.idr_pcm(y, u, v)
    (got,) = _decode(host, s.bytes())
    _assert_pic(got, (y, u, v))


MVS = [(0, 0), (1, 0), (0, 2), (3, 3), (-5, 6), (13, -7), (-9, -14), (22, 1), (-70, 3), (2, 75)]


@pytest.mark.parametrize("bd", [8, 10])
def test_kat_skip_cus_inherit_the_first_vector(host, bd):
    """An AMVP CU then skip CUs: each skip CU's merge candidate 0 is its left (A1) or, at the
    start of a CTB row, above (B1) neighbour, so one fractional vector covers the picture."""
    w, h = 64, 32
    ref = _content(w, h, bd, 2)
    s = KatStream(w, h, bit_depth=bd, ctb_log2=4)
    s.idr_pcm(*ref)
    mvs = [(13, -7)]
    blocks = [(x, y, 16, 16) for y in range(0, h, 16) for x in range(0, w, 16)]
    cus = [{"mvd": mvs[0]}] + [{"skip": True}] * 7
    s.p_picture(1, [0], cus)
    got = _decode(host, s.bytes())
    want = _predict_picture(ref, [mvs[0]] * len(blocks), bd, blocks)
    _assert_pic(got[1], want)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("mv", MVS)
def test_kat_interpolation_single_vector(host, bd, mv):
    w, h = 32, 32
    ref = _content(w, h, bd, 3)
    s = KatStream(w, h, bit_depth=bd, ctb_log2=5)
    s.idr_pcm(*ref)
    s.p_picture(1, [0], [{"mvd": mv}])
    got = _decode(host, s.bytes())
    _assert_pic(got[1], _predict_picture(ref, [mv], bd, [(0, 0, 32, 32)]))


WP = [
    # (luma denom, luma weight, luma offset, chroma denom delta, [(cw, delta_chroma_offset)] * 2)
    (0, 1, 0, 0, [(1, 0), (1, 0)]),
    (6, 64, 0, 0, [(64, 0), (64, 0)]),
    (5, 40, -7, 1, [(70, 3), (50, -20)]),
    (7, 100, 20, -3, [(20, 10), (12, -9)]),
    (2, -3, 127, 0, [(-2, -128), (7, 127)]),
    (0, 3, -128, 7, [(200, 60), (100, -60)]),
]


def _chroma_offset(cw, cdenom, delta):
    """7.4.7.3: ChromaOffsetL0 from delta_chroma_offset_l0 (wpOffsetHalfRangeC = 128)."""
    half = 128
    return int(np.clip(half - ((half * cw) >> cdenom) + delta, -half, half - 1))


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("k", range(len(WP)))
def test_kat_weighted_prediction(host, bd, k):
    d, lw, lo, cdd, cws = WP[k]
    cd = d + cdd
    w, h = 32, 32
    ref = _content(w, h, bd, 4 + k)
    s = KatStream(w, h, bit_depth=bd, ctb_log2=4, weighted=True)
    s.idr_pcm(*ref)
    wp = {"denom": d, "w": lw, "o": lo, "cdenom_delta": cdd, "cw": cws}
    mv = (5, -3)
    s.p_picture(1, [0], [{"mvd": mv}] + [{"skip": True}] * 3, wp=wp)
    got = _decode(host, s.bytes())
    cw = [(c, _chroma_offset(c, cd, off)) for c, off in cws]
    blocks = [(x, y, 16, 16) for y in (0, 16) for x in (0, 16)]
    want = _predict_picture(ref, [mv] * 4, bd, blocks, weights=((d, lw, lo), (cd, cw)))
    _assert_pic(got[1], want)
    if k > 1:  # non-trivial weights: default weighting would differ in every plane
        dflt = _predict_picture(ref, [mv] * 4, bd, blocks)
        assert all(not np.array_equal(a_, b_) for a_, b_ in zip(dflt, want))


def _scale_mv(mv, td, tb):
    """8.5.3.2.8 with C-style division."""
    td, tb = int(np.clip(td, -128, 127)), int(np.clip(tb, -128, 127))
    tx = int((16384 + (abs(td) >> 1)) / td)
    dsf = int(np.clip((tb * tx + 32) >> 6, -4096, 4095))

    def one(m):
        p = dsf * m
        return int(np.clip((1 if p >= 0 else -1) * ((abs(p) + 127) >> 8), -32768, 32767))

    return one(mv[0]), one(mv[1])


@pytest.mark.parametrize("mv,pocs", [
    ((12, 0), (3, 4)),        # td 3, tb 1
    ((-7, 21), (3, 8)),       # td 3, tb 5
    ((33, -17), (5, 6)),      # td 5, tb 1
    ((64, 40), (2, 9)),       # td 2, tb 7
    ((-3, -1), (7, 20)),      # td 7, tb 13
    ((9, 9), (4, 4 + 100)),   # tb 100: distScaleFactor clipped? (tx 4096, 100 * 4096 >> 6)
])
def test_kat_tmvp_scaling(host, mv, pocs):
    """P1 (POC a) codes one vector from the IDR (POC 0); P2 (POC b) is one skip CU whose only
    merge candidate is the temporal one, collocated in P1, scaled from distance a to b - a."""
    a, b = pocs
    w = h = 32
    ref = _content(w, h, 8, 9)
    s = KatStream(w, h, ctb_log2=5)
    s.idr_pcm(*ref)
    s.p_picture(a, [0], [{"mvd": mv}])
    s.p_picture(b, [a], [{"skip": True}], tmvp=True)
    got = _decode(host, s.bytes())
    p1 = _predict_picture(ref, [mv], 8, [(0, 0, 32, 32)])
    _assert_pic(got[1], p1)
    smv = _scale_mv(mv, a - 0, b - a)
    want = _predict_picture(p1, [smv], 8, [(0, 0, 32, 32)])
    _assert_pic(got[2], want)
    # the case discriminates: the unscaled vector predicts differently
    assert not np.array_equal(_predict_picture(p1, [mv], 8, [(0, 0, 32, 32)])[0], want[0])


@pytest.mark.parametrize("part,geom", [
    ("nLx2N", [(0, 0, 8, 32), (8, 0, 24, 32)]),
    ("nRx2N", [(0, 0, 24, 32), (24, 0, 8, 32)]),
    ("2NxnU", [(0, 0, 32, 8), (0, 8, 32, 24)]),
    ("2NxnD", [(0, 0, 32, 24), (0, 24, 32, 8)]),
    ("Nx2N", [(0, 0, 16, 32), (16, 0, 16, 32)]),
    ("2NxN", [(0, 0, 32, 16), (0, 16, 32, 16)]),
])
def test_kat_second_pu_merge_excludes_first_pu(host, part, geom):
    """The second PU of a vertical split must not merge the first PU's motion through A1, nor
    that of a horizontal split through B1; with no other neighbour (one CTU picture, TMVP
    off) its only candidate is the zero vector."""
    w = h = 32
    ref = _content(w, h, 8, 11)
    s = KatStream(w, h, ctb_log2=5)
    s.idr_pcm(*ref)
    mv = (-6, 5)
    s.p_picture(1, [0], [{"part": part, "pus": [("mvd", mv), ("merge",)]}])
    got = _decode(host, s.bytes())
    want = _predict_picture(ref, [mv, (0, 0)], 8, geom)
    _assert_pic(got[1], want)
    assert not np.array_equal(_predict_picture(ref, [mv, mv], 8, geom)[0], want[0])


LEVEL_SCALE = [40, 45, 51, 57, 64, 72]


def _dc_residual(level, m, qp, log2, bd):
    """8.6.2 - 8.6.4.2 for a block whose only coefficient is the DC one."""
    bds = bd + log2 - 5
    d = int(np.clip(((level * m * LEVEL_SCALE[qp % 6] << (qp // 6)) + (1 << (bds - 1))) >> bds, -32768, 32767))
    g = int(np.clip((64 * d + 64) >> 7, -32768, 32767))
    s2 = 20 - bd
    return (64 * g + (1 << (s2 - 1))) >> s2


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("case", ["flat", "list8", "dc16", "default8"])
def test_kat_scaling_list_dequant(host, bd, case):
    """One 2Nx2N inter CU (zero vector) with a DC level per luma transform block: flat
    dequantisation (scaling lists off), an explicit 8x8 inter-luma list, an explicit 16x16 list
    whose DC entry is scaling_list_dc_coef, and the default 8x8 inter list (Table 7-6)."""
    w = h = 16
    ref = _content(w, h, bd, 13)
    qp = 31
    coefs8 = [(8 + 3 * i) % 97 + 9 for i in range(64)]
    if case == "flat":
        kw, log2, m = dict(), 4, 16
    elif case == "list8":
        kw, log2, m = dict(scaling={(1, 3): (coefs8, None)}, max_tb_log2=3), 3, coefs8[0]
    elif case == "dc16":
        kw, log2, m = dict(scaling={(2, 3): (coefs8, 37)}), 4, 37
    else:
        kw, log2, m = dict(scaling={}, max_tb_log2=3), 3, DEFAULT_8x8_INTER[0]
    s = KatStream(w, h, bit_depth=bd, ctb_log2=4, **kw)
    s.idr_pcm(*ref)
    levels = [3, -2, 5, -6] if log2 == 3 else [-4]
    s.p_picture(1, [0], [{"mvd": (0, 0), "dc": levels}], qp=qp)
    got = _decode(host, s.bytes())
    qpp = qp + 6 * (bd - 8)
    y = ref[0].copy()
    n = 1 << log2
    tbs = [(x, yy) for yy in range(0, 16, n) for x in range(0, 16, n)]
    for (x, yy), L in zip(tbs, levels):
        y[yy:yy + n, x:x + n] += _dc_residual(L, m, qpp, log2, bd)
    want = (np.clip(y, 0, (1 << bd) - 1), ref[1], ref[2])
    _assert_pic(got[1], want)
    if m != 16:  # the scaling factor matters: flat dequantisation gives another residual
        assert any(_dc_residual(L, 16, qpp, log2, bd) != _dc_residual(L, m, qpp, log2, bd) for L in levels)
