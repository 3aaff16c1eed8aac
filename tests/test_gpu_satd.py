"""The 4x4 SATD primitives of the decision kernels (csrc/kernels/kcommon.h) against a numpy
fp32 model of x264's satd (sum of |4x4 Hadamard of the residual| / 2), bit-exact: the
packed 16-bit form (satd4x4_u8) is what b_decide, p_mv_refine, p_part8x8 and encode_inter
price candidates with, so any difference would change decisions and bytes."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

H4 = np.array([[1, 1, 1, 1], [1, 1, -1, -1], [1, -1, -1, 1], [1, -1, 1, -1]], np.float32)


def _satd_ref(s, p):
    r = s.astype(np.float32).reshape(-1, 4, 4) - p.astype(np.float32).reshape(-1, 4, 4)
    t = np.einsum("ij,njk,lk->nil", H4, r, H4)
    return (np.abs(t).sum(axis=(1, 2)) / 2).astype(np.int64)


@pytest.mark.parametrize("mode", [0, 1])
def test_satd_primitives_match_numpy(mode):
    from govideocompressor_amd.ops import native
    hip = native.hip()
    rng = np.random.default_rng(3)
    n = 64 * 97
    s = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    p = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    # extremes: full-scale residuals of both signs, flat blocks, one-sample spikes
    s[:64], p[:64] = 255, 0
    s[64:128], p[64:128] = 0, 255
    s[128:192] = p[128:192]
    s[192:256], p[192:256] = 0, 0
    s[192:256, 5] = 255
    s[256:320] = np.where(np.arange(16) % 2, 255, 0)
    p[256:320] = np.where(np.arange(16) % 3, 0, 255)
    dev = torch.device("cuda")
    ts, tp = torch.from_numpy(s).to(dev), torch.from_numpy(p).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    hip.satd_blocks(ts.data_ptr(), tp.data_ptr(), out.data_ptr(), n, mode, torch.cuda.current_stream().cuda_stream)
    got = out.cpu().numpy().astype(np.int64)
    want = _satd_ref(s, p)
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]


# ---------------------------------------------------------------- trellis forms (h264_trellis.h)
CF = np.array([[1, 1, 1, 1], [2, 1, -1, -2], [1, -1, -1, 1], [1, -2, 2, -1]], np.int64)
ZZ = [0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15]
MF = [[13107, 5243, 8066], [11916, 4660, 7490], [10082, 4194, 6554], [9362, 3647, 5825], [8192, 3355, 5243],
      [7282, 2893, 4559]]


def _cls(r):
    x, y = r & 3, r >> 2
    return 0 if ((x | y) & 1) == 0 else (1 if (x & y) & 1 else 2)


def _trellis_ref(w, qp, start):
    """float64 model of the serial greedy pass (trellis_lite4x4)."""
    qbits, mf = 15 + qp // 6, MF[qp % 6]
    lam = 0.85 * 2.0 ** ((qp - 12) / 3)
    inv = [1 / 16, 1 / 100, 1 / 40]

    def bits(level, seen):
        b = 1.35 + (0.25 if seen else 2.2) + 1.0
        if level == 1:
            return b + 0.6
        b += 1.7 + 0.9 * min(level - 2, 13)
        if level > 15:
            b += 2.0 * (int(level - 14).bit_length() - 1) + 1.0
        return b

    out = np.zeros(16, np.int64)
    seen = False
    for i in range(15, start - 1, -1):
        r = ZZ[i]
        a, m = abs(int(w[r])), mf[_cls(r)]
        zr = (a * m + (1 << (qbits - 1))) >> qbits
        step = (1 << qbits) / m
        best, bl = a * a * inv[_cls(r)] + lam * (0.55 if seen else 0.0), 0
        for level in (zr - 1, zr):
            if level < 1:
                continue
            j = (a - level * step) ** 2 * inv[_cls(r)] + lam * bits(level, seen)
            if j < best:
                best, bl = j, level
        out[r] = -bl if w[r] < 0 else bl
        seen |= bl != 0
    return out


@pytest.mark.parametrize("qp", [12, 24, 33, 45])
@pytest.mark.parametrize("skip_dc", [0, 1])
def test_trellis_parallel_form_matches_serial(qp, skip_dc):
    """grp_trellis4x4 (4 lanes per block, `seen` resolved by one max-reduction: the intra
    kernel's form) gives the levels of the serial pass (the inter kernel's), bit-exact, and
    both follow a float64 model (ties aside)."""
    from govideocompressor_amd.ops import native
    hip = native.hip()
    rng = np.random.default_rng(qp * 2 + skip_dc)
    n = 16 * 301
    amp = rng.choice([2, 6, 20, 60, 255], size=(n, 1, 1))
    res = np.clip(np.round(rng.laplace(0, 1, (n, 4, 4)) * amp / 3), -255, 255).astype(np.int64)
    w = np.einsum("ij,njk,lk->nil", CF, res, CF).reshape(n, 16)
    dev = torch.device("cuda")
    tw = torch.from_numpy(w.astype(np.int32)).to(dev)
    outs = []
    for mode in (0, 1):
        out = torch.empty(n, 16, dtype=torch.int32, device=dev)
        hip.trellis_blocks(tw.data_ptr(), out.data_ptr(), n, qp, mode, skip_dc, torch.cuda.current_stream().cuda_stream)
        outs.append(out.cpu().numpy().astype(np.int64))
    assert np.array_equal(outs[0], outs[1]), np.argwhere((outs[0] != outs[1]).any(axis=1))[:5]
    want = np.stack([_trellis_ref(w[b], qp, skip_dc) for b in range(n)])
    bad = (want != outs[1]).any(axis=1).mean()
    assert bad < 2e-3, bad
    # the levels stay within one of the rounded quotient and the dead zone never grows a level
    qbits, mf = 15 + qp // 6, np.array([MF[qp % 6][_cls(r)] for r in range(16)])
    zr = (np.abs(w) * mf + (1 << (qbits - 1))) >> qbits
    assert (np.abs(outs[1]) <= zr).all()
    assert (np.abs(outs[1])[zr == 0] == 0).all()
    if skip_dc:
        assert (outs[1][:, 0] == 0).all()
    assert np.abs(outs[1]).sum() > 0
