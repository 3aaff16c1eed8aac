"""T1 kernel golden test: the gfx950 motion-estimation kernel (csrc/kernels/me.hip)
against an independent numpy statement of the same search -- candidate centre,
(2R+1)^2 integer SAD search on the edge-extended reference, half- then
quarter-sample SATD refinement with H.264 6-tap interpolation, the final luma
prediction and the open-loop Intra16x16 estimate.  Every output must match exactly.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PAD = 64


def _ue_bits(v):
    return 2 * int(np.floor(np.log2(v + 1))) + 1


def _se_bits(v):
    return _ue_bits(-2 * v if v <= 0 else 2 * v - 1)


_H4 = np.array([[1, 1, 1, 1], [1, 1, -1, -1], [1, -1, -1, 1], [1, -1, 1, -1]])


def _hsum(r):
    return int(np.abs(_H4 @ r @ _H4.T).sum())


def _satd(r):
    return _hsum(r) >> 1


class _Planes:
    """Edge-extended reference + full-frame half-sample planes (8.4.2.2.1)."""

    def __init__(self, ref):
        g = np.pad(ref.astype(np.int64), PAD, mode="edge")
        self.G = g

        def tap(a, axis, k):
            sl = lambda o: np.roll(a, -o, axis=axis)  # noqa: E731
            return sl(k - 2) - 5 * sl(k - 1) + 20 * sl(k) + 20 * sl(k + 1) - 5 * sl(k + 2) + sl(k + 3)
        b1 = tap(g, 1, 0)               # b1[y, x] = half position between x and x+1
        h1 = tap(g, 0, 0)
        self.b = np.clip((b1 + 16) >> 5, 0, 255)
        self.h = np.clip((h1 + 16) >> 5, 0, 255)
        j1 = tap(b1, 0, 0)
        self.j = np.clip((j1 + 512) >> 10, 0, 255)

    def qpel(self, x, y, xf, yf):
        """sample at integer (x, y) (frame coords) + quarter phase (xf, yf)"""
        X, Y = x + PAD, y + PAD
        G, b, h, j = self.G, self.b, self.h, self.j
        tab = {
            (0, 0): (G[Y, X], G[Y, X]), (1, 0): (G[Y, X], b[Y, X]), (2, 0): (b[Y, X], b[Y, X]),
            (3, 0): (G[Y, X + 1], b[Y, X]), (0, 1): (G[Y, X], h[Y, X]), (1, 1): (b[Y, X], h[Y, X]),
            (2, 1): (j[Y, X], b[Y, X]), (3, 1): (b[Y, X], h[Y, X + 1]), (0, 2): (h[Y, X], h[Y, X]),
            (1, 2): (j[Y, X], h[Y, X]), (2, 2): (j[Y, X], j[Y, X]), (3, 2): (j[Y, X], h[Y, X + 1]),
            (0, 3): (G[Y + 1, X], h[Y, X]), (1, 3): (b[Y + 1, X], h[Y, X]), (2, 3): (j[Y, X], b[Y + 1, X]),
            (3, 3): (b[Y + 1, X], h[Y, X + 1]),
        }
        a, c = tab[(xf, yf)]
        return int(a), int(c)

    def block(self, x0, y0, mvx, mvy, rounded=True):
        """prediction (A + B + 1) >> 1, or the unrounded tap sum A + B (rounded=False)"""
        out = np.zeros((16, 16), dtype=np.int64)
        ix, iy, xf, yf = mvx >> 2, mvy >> 2, mvx & 3, mvy & 3
        for y in range(16):
            for x in range(16):
                a, c = self.qpel(x0 + x + ix, y0 + y + iy, xf, yf)
                out[y, x] = (a + c + 1) >> 1 if rounded else a + c
        return out


def _ring(c, step):
    idx = 4 if c == 0 else (c - 1 if c <= 4 else c)
    return (idx % 3 - 1) * step, (idx // 3 - 1) * step


def _me_ref(src, ref, pred_mv, qp, R, lam_tab, wmb, hmb):
    H, W = src.shape
    lam = lam_tab[qp]
    pl = _Planes(ref)
    G = pl.G
    out_mv = np.zeros((hmb * wmb, 2), dtype=np.int64)
    out_cost = np.zeros(hmb * wmb, dtype=np.int64)
    out_pred = np.zeros((hmb * wmb, 256), dtype=np.int64)
    out_intra = np.zeros(hmb * wmb, dtype=np.int64)
    s = src.astype(np.int64)
    for mb in range(wmb * hmb):
        mx, my = mb % wmb, mb // wmb
        X0, Y0 = mx * 16, my * 16
        S = s[Y0:Y0 + 16, X0:X0 + 16]
        pmx, pmy = int(pred_mv[mb, 0]), int(pred_mv[mb, 1])
        cands = [((pmx + 2) >> 2, (pmy + 2) >> 2)]
        cands.append(((int(pred_mv[mb - 1, 0]) + 2) >> 2, (int(pred_mv[mb - 1, 1]) + 2) >> 2) if mx > 0 else (0, 0))
        cands.append(((int(pred_mv[mb - wmb, 0]) + 2) >> 2, (int(pred_mv[mb - wmb, 1]) + 2) >> 2) if my > 0 else (0, 0))
        cands.append(((int(pred_mv[mb + 1, 0]) + 2) >> 2, (int(pred_mv[mb + 1, 1]) + 2) >> 2)
                     if mx < wmb - 1 else (0, 0))
        cands.append((0, 0))

        def sad(dx, dy):
            blk = G[PAD + Y0 + dy:PAD + Y0 + dy + 16, PAD + X0 + dx:PAD + X0 + dx + 16]
            return int(np.abs(S - blk).sum())
        best, cx, cy = None, 0, 0
        for (dx, dy) in cands:
            dx, dy = max(-128, min(128, dx)), max(-128, min(128, dy))
            c = sad(dx, dy) + lam * (_se_bits(dx * 4 - pmx) + _se_bits(dy * 4 - pmy))
            if best is None or c < best:
                best, cx, cy = c, dx, dy
        side = 2 * R + 1
        bkey = None
        for dy in range(side):
            for dx in range(side):
                mvx, mvy = (cx + dx - R) * 4, (cy + dy - R) * 4
                c = sad(cx + dx - R, cy + dy - R) + lam * (_se_bits(mvx - pmx) + _se_bits(mvy - pmy))
                key = (c << 12) | (dy * side + dx)
                bkey = key if bkey is None else min(bkey, key)
        if abs(cx) > R or abs(cy) > R:
            c = sad(0, 0) + lam * (_se_bits(-pmx) + _se_bits(-pmy))
            bkey = min(bkey, (c << 12) | 4095)
        bp = bkey & 4095
        bx, by = (0, 0) if bp == 4095 else (cx + bp % side - R, cy + bp // side - R)

        def cost_q(mvx, mvy):
            # the MFMA form of me.hip: (sum over the MB of |H (2 (S - P))| + 2) / 4
            T = S - pl.block(X0, Y0, mvx, mvy)
            sat = (sum(_hsum(T[y:y + 4, x:x + 4]) for y in range(0, 16, 4) for x in range(0, 16, 4)) + 1) >> 1
            return sat + lam * (_se_bits(mvx - pmx) + _se_bits(mvy - pmy))
        bm = (bx * 4, by * 4)
        hk = min(((cost_q(bm[0] + _ring(c, 2)[0], bm[1] + _ring(c, 2)[1]) << 4) | c) for c in range(9))
        hx, hy = _ring(hk & 15, 2)
        qk = hk & ~15
        for c in range(1, 9):
            ox, oy = _ring(c, 1)
            qk = min(qk, (cost_q(bm[0] + hx + ox, bm[1] + hy + oy) << 4) | c)
        qx, qy = _ring(qk & 15, 1)
        mv = (bm[0] + hx + qx, bm[1] + hy + qy)
        out_mv[mb] = mv
        out_cost[mb] = qk >> 4
        out_pred[mb] = pl.block(X0, Y0, mv[0], mv[1]).reshape(-1)
        # open-loop Intra16x16 on source neighbours
        top = s[Y0 - 1, X0:X0 + 16] if my > 0 else np.zeros(16, dtype=np.int64)
        left = s[Y0:Y0 + 16, X0 - 1] if mx > 0 else np.zeros(16, dtype=np.int64)
        tl = int(s[Y0 - 1, X0 - 1]) if mx > 0 and my > 0 else 0
        modes = []
        if my > 0:
            modes.append(np.tile(top, (16, 1)))
        if mx > 0:
            modes.append(np.tile(left[:, None], (1, 16)))
        st, sl = int(top.sum()), int(left.sum())
        dc = (st + sl + 16) >> 5 if (mx > 0 and my > 0) else ((sl + 8) >> 4 if mx > 0 else ((st + 8) >> 4 if my > 0 else 128))
        modes.append(np.full((16, 16), dc))
        if mx > 0 and my > 0:
            Hh = sum((i + 1) * (int(top[8 + i]) - (tl if i == 7 else int(top[6 - i]))) for i in range(8))
            Vv = sum((i + 1) * (int(left[8 + i]) - (tl if i == 7 else int(left[6 - i]))) for i in range(8))
            a, b, c = 16 * (int(left[15]) + int(top[15])), (5 * Hh + 32) >> 6, (5 * Vv + 32) >> 6
            yy, xx = np.mgrid[0:16, 0:16]
            modes.append(np.clip((a + b * (xx - 7) + c * (yy - 7) + 16) >> 5, 0, 255))
        best_i = min((sum(_hsum(S[y:y + 4, x:x + 4] - M[y:y + 4, x:x + 4]) for y in range(0, 16, 4)
                          for x in range(0, 16, 4)) + 1) >> 1 for M in modes)
        out_intra[mb] = best_i + lam * 4
    return out_mv, out_cost, out_pred, out_intra


@pytest.mark.parametrize("R,seed,with_pred", [(8, 1, False), (8, 2, True), (4, 3, True)])
def test_me_matches_numpy_reference(host, R, seed, with_pred):
    import torch
    from govideocompressor_amd.ops import native
    hip = native.hip()
    rng = np.random.default_rng(seed)
    wmb, hmb = 4, 3
    W, H = wmb * 16, hmb * 16
    base = rng.integers(0, 256, size=(H + 40, W + 40)).astype(np.float64)
    k = np.ones(5) / 5
    base = np.apply_along_axis(lambda r: np.convolve(r, k, "same"), 1, base)
    base = np.apply_along_axis(lambda r: np.convolve(r, k, "same"), 0, base)
    ref = base[10:10 + H, 12:12 + W]
    src = base[13:13 + H, 10:10 + W] + rng.normal(0, 2, size=(H, W))
    # np.apply_along_axis leaves a Fortran-ordered array: force C order before the upload
    ref = np.ascontiguousarray(np.clip(ref, 0, 255).astype(np.uint8))
    src = np.ascontiguousarray(np.clip(src, 0, 255).astype(np.uint8))
    pred = np.ascontiguousarray(
        (rng.integers(-24, 24, size=(wmb * hmb, 2)) if with_pred else np.zeros((wmb * hmb, 2))).astype(np.int16))
    qp = 27
    dev = torch.device("cuda")
    ts, tr = torch.from_numpy(src).to(dev), torch.from_numpy(ref).to(dev)
    tp = torch.from_numpy(pred).to(dev)
    mv = torch.zeros((wmb * hmb, 2), dtype=torch.int16, device=dev)
    cost = torch.zeros(wmb * hmb, dtype=torch.int32, device=dev)
    outp = torch.zeros((wmb * hmb, 256), dtype=torch.uint8, device=dev)
    intra = torch.zeros(wmb * hmb, dtype=torch.int32, device=dev)
    tq = torch.tensor([qp], dtype=torch.int32, device=dev)
    hip.me(1, wmb, hmb, ts.data_ptr(), tr.data_ptr(), tp.data_ptr(), mv.data_ptr(), cost.data_ptr(), outp.data_ptr(),
           intra.data_ptr(), tq.data_ptr(), R, 2, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    lam = host.table("lambda")[0]
    rmv, rcost, rpred, rintra = _me_ref(src, ref, pred, qp, R, lam, wmb, hmb)
    assert np.array_equal(mv.cpu().numpy(), rmv), (mv.cpu().numpy(), rmv)
    assert np.array_equal(cost.cpu().numpy(), rcost)
    assert np.array_equal(outp.cpu().numpy().astype(np.int64), rpred)
    assert np.array_equal(intra.cpu().numpy(), rintra)


@pytest.mark.parametrize("W,H", [(64, 48), (176, 144)])
def test_me_halfpel_planes_match_numpy(W, H):
    """Frame-level b / h / j planes (margin 4) against the numpy 6-tap statement."""
    import torch
    from govideocompressor_amd.ops import native
    hip = native.hip()
    rng = np.random.default_rng(W)
    refs = rng.integers(0, 256, size=(2, H, W)).astype(np.uint8)
    dev = torch.device("cuda")
    tr = torch.from_numpy(refs).to(dev)
    M = 4
    hp = torch.zeros((2, 3, H + 2 * M, W + 2 * M), dtype=torch.uint8, device=dev)
    hip.me_halfpel(2, W, H, tr.data_ptr(), hp.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = hp.cpu().numpy().astype(np.int64)
    for b in range(2):
        pl = _Planes(refs[b])
        sl = (slice(PAD - M, PAD + H + M), slice(PAD - M, PAD + W + M))
        for k, plane in enumerate((pl.b, pl.h, pl.j)):
            d = np.argwhere(got[b, k] != plane[sl])
            assert len(d) == 0, (b, "bhj"[k], len(d), d[:8], [(int(got[b, k][tuple(e)]), int(plane[sl][tuple(e)])) for e in d[:8]])


def _refine_ref(src, planes, mv_in, cost, pm, pred, qps, lam_tab, wmb, hmb):
    """One Jacobi pass of the P_Skip-aware vector choice (bframe.hip p_mv_refine) in numpy:
    each MB is offered the P_Skip predictor of its neighbours' current vectors (8.4.1.1) and
    takes it when SATD <= its own SATD + lambda * (mvd bits vs that predictor + 1)."""
    B = src.shape[0]
    mv_out, cost, pred = mv_in.copy(), cost.copy(), pred.copy()
    for b in range(B):
        lam = lam_tab[int(qps[b])]
        for mb in range(wmb * hmb):
            mx, my = mb % wmb, mb // wmb
            cx, cy = (int(v) for v in mv_in[b, mb])
            sx = sy = 0
            if mx > 0 and my > 0:
                A, Bn = mv_in[b, mb - 1], mv_in[b, mb - wmb]
                if A.any() and Bn.any():
                    C = mv_in[b, mb - wmb + 1] if mx < wmb - 1 else mv_in[b, mb - wmb - 1]
                    sx, sy = (int(np.median([A[i], Bn[i], C[i]])) for i in range(2))
            if (sx, sy) == (cx, cy):
                continue
            X0, Y0 = mx * 16, my * 16
            P = planes[b].block(X0, Y0, sx, sy)
            R = src[b, Y0:Y0 + 16, X0:X0 + 16].astype(np.int64) - P
            satd = sum(_satd(R[y:y + 4, x:x + 4]) for y in range(0, 16, 4) for x in range(0, 16, 4))
            pmx, pmy = (int(v) for v in pm[b, mb])
            satd_me = int(cost[b, mb]) - lam * (_se_bits(cx - pmx) + _se_bits(cy - pmy))
            if satd <= satd_me + lam * (_se_bits(cx - sx) + _se_bits(cy - sy) + 1):
                mv_out[b, mb] = (sx, sy)
                cost[b, mb] = satd + lam * (_se_bits(sx - pmx) + _se_bits(sy - pmy))
                pred[b, mb] = P.reshape(256)
    return mv_out, cost, pred


@pytest.mark.parametrize("masks", [False, True])
def test_p_refine_matches_numpy(host, masks):
    """p_mv_refine (four MBs per wave, one 4x4 block per lane) against the numpy statement of
    the pass, over four passes on a near-uniform field; 117 MBs leave a partial last wave.
    ``masks``: passes after the first skip MBs whose own and whose neighbours' vectors did not
    move in the previous pass (change masks) -- the fields must still equal the full passes'."""
    import torch
    from govideocompressor_amd.ops import native
    hip = native.hip()
    rng = np.random.default_rng(5)
    B, wmb, hmb = 2, 13, 9
    W, H, nmb = wmb * 16, hmb * 16, wmb * hmb
    dev = torch.device("cuda")
    s = torch.cuda.current_stream().cuda_stream
    k = np.ones(5) / 5
    refs, srcs = [], []
    for _ in range(B):
        base = rng.integers(0, 256, size=(H + 40, W + 40)).astype(np.float64)
        base = np.apply_along_axis(lambda r: np.convolve(r, k, "same"), 1, base)
        base = np.apply_along_axis(lambda r: np.convolve(r, k, "same"), 0, base)
        refs.append(np.clip(base[10:10 + H, 12:12 + W], 0, 255))
        srcs.append(np.clip(base[12:12 + H, 13:13 + W] + rng.normal(0, 3, size=(H, W)), 0, 255))
    refs = np.ascontiguousarray(np.stack(refs).astype(np.uint8))
    srcs = np.ascontiguousarray(np.stack(srcs).astype(np.uint8))
    ref, src = torch.from_numpy(refs).to(dev), torch.from_numpy(srcs).to(dev)
    hp = torch.zeros((B, 3, H + 8, W + 8), dtype=torch.uint8, device=dev)
    hip.me_halfpel(B, W, H, ref.data_ptr(), hp.data_ptr(), s)
    planes = [_Planes(refs[b]) for b in range(B)]
    # a near-uniform field (4, 8) with scattered quarter-sample deviations
    mv = np.tile(np.array([4, 8], dtype=np.int16), (B, nmb, 1))
    dmask = rng.random((B, nmb)) < 0.6
    mv[dmask] += rng.integers(-3, 4, size=(int(dmask.sum()), 2)).astype(np.int16)
    cost = rng.integers(400, 4000, size=(B, nmb)).astype(np.int32)
    pred = rng.integers(0, 256, size=(B, nmb, 256)).astype(np.uint8)
    pm = np.zeros((B, nmb, 2), dtype=np.int16)
    qps = np.array([26, 32], dtype=np.int32)
    t_mv = [torch.from_numpy(mv.copy()).to(dev), torch.zeros((B, nmb, 2), dtype=torch.int16, device=dev)]
    t_cost, t_pred = torch.from_numpy(cost.copy()).to(dev), torch.from_numpy(pred.copy()).to(dev)
    t_pm, t_qp = torch.from_numpy(pm).to(dev), torch.from_numpy(qps).to(dev)
    lam = host.table("lambda")[0]
    took = 0
    chg = [torch.zeros((B, nmb), dtype=torch.uint8, device=dev) for _ in range(2)]
    for it in range(4):
        a_, b_ = t_mv[it % 2], t_mv[(it + 1) % 2]
        cin = chg[(it - 1) % 2].data_ptr() if (masks and it > 0) else 0
        cout = chg[it % 2].data_ptr() if masks else 0
        hip.p_refine(B, wmb, hmb, src.data_ptr(), ref.data_ptr(), hp.data_ptr(), a_.data_ptr(), b_.data_ptr(),
                     t_cost.data_ptr(), t_pm.data_ptr(), t_pred.data_ptr(), t_qp.data_ptr(), 0, s, 0, 0, cin, cout)
        torch.cuda.synchronize()
        r_mv, r_cost, r_pred = _refine_ref(srcs, planes, mv, cost, pm, pred, qps, lam, wmb, hmb)
        took += int((r_mv != mv).any(axis=2).sum())
        assert np.array_equal(b_.cpu().numpy(), r_mv), it
        assert np.array_equal(t_cost.cpu().numpy(), r_cost), it
        assert np.array_equal(t_pred.cpu().numpy(), r_pred.astype(np.uint8)), it
        mv, cost, pred = r_mv, r_cost, r_pred
    assert took > 0
