"""T1 kernel golden test: the gfx950 lookahead (csrc/kernels/lookahead.hip: 2x2
downscale, lowres integer search, DC/H/V intra, 8x8 Hadamard SATD as an int8 MFMA
GEMM) against the plain numpy statement in rc/lookahead.py.  Per-block intra/inter
costs and the per-frame sums must match exactly; the MFMA operand layout is checked
with content whose Hadamard spectrum is asymmetric (random texture + moving blocks).
"""
import numpy as np
import pytest

from govideocompressor_amd.rc.lookahead import lookahead_reference
from govideocompressor_amd.rc.ratecontrol import crf_qps, crf_qps_batch


def _clip(B, F, h, w, seed):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, size=(B, h + 64, w + 64), dtype=np.int64)
    # smooth it a little so the search has a real minimum, keep high-frequency detail
    base = (base + np.roll(base, 1, 1) + np.roll(base, 1, 2) + np.roll(base, (1, 1), (1, 2))) // 4
    out = np.zeros((B, F, h, w), dtype=np.uint8)
    for b in range(B):
        vx, vy = int(rng.integers(-5, 6)), int(rng.integers(-3, 4))
        for f in range(F):
            ox, oy = 32 + vx * f, 32 + vy * f
            fr = np.roll(base[b], (-oy, -ox), (0, 1))[:h, :w].copy()
            fr += rng.integers(-2, 3, size=fr.shape)
            fr[8:24, 8 + 3 * f:40 + 3 * f] = 255 - fr[8:24, 8 + 3 * f:40 + 3 * f]  # a moving object
            out[b, f] = np.clip(fr, 0, 255)
    out[0, :, -6:, :] = 0          # saturated edges
    out[-1, :, :, -10:] = 255
    return out


def test_reference_model_basics():
    y = _clip(1, 3, 48, 80, 0)
    frame, blk = lookahead_reference(y, search_range=4)
    assert frame.shape == (1, 3, 2) and blk.shape == (1, 3, 2, 3, 5)
    assert np.all(frame[:, 0, 0] == frame[:, 0, 1])       # key frame: intra only
    assert np.all(frame[:, 1:, 1] <= frame[:, 1:, 0])     # P cost <= intra cost
    # a static clip: inter cost collapses to the noise floor
    ys = np.repeat(y[:, :1], 3, axis=1)
    fs, _ = lookahead_reference(ys, search_range=4)
    assert fs[0, 1, 1] < fs[0, 1, 0] // 4


def test_crf_batch_matches_scalar():
    rng = np.random.default_rng(3)
    costs = rng.uniform(2e5, 2e6, size=(4, 12, 2))
    costs[:, :, 1] = np.minimum(costs[:, :, 1], costs[:, :, 0])
    q = crf_qps_batch(costs, 23.0, 8160)
    for b in range(4):
        ref = crf_qps(costs[b, :, 0], costs[b, :, 1], 23.0, 8160, keyint=12)
        assert np.array_equal(q[b], ref)


@pytest.mark.gpu
@pytest.mark.parametrize("R", [4, 6, 8])
@pytest.mark.parametrize("shape", [(2, 3, 64, 96), (1, 2, 70, 300)])
def test_lookahead_matches_reference(R, shape):
    import torch

    from govideocompressor_amd.rc.lookahead import GpuLookahead

    B, F, h, w = shape
    y = _clip(B, F, h, w, seed=R * 10 + w)
    la = GpuLookahead("cuda:0", search_range=R, hierarchical=False)
    yd = torch.from_numpy(y).to("cuda:0")
    frame, blk = la.frame_costs(yd, block_costs=True)
    torch.cuda.synchronize()
    ref_frame, ref_blk = lookahead_reference(y, search_range=R)
    got_blk = blk.cpu().numpy().astype(np.int64)
    bad = np.argwhere(got_blk != ref_blk)
    assert bad.size == 0, f"{len(bad)} block mismatches, first {bad[:4].tolist()}"
    assert np.array_equal(frame.cpu().numpy(), ref_frame)


@pytest.mark.gpu
def test_encoder_uses_lookahead_qps():
    import torch

    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip

    p = H264Params(width=320, height=240, crf=23)
    enc = GpuH264Encoder(p, slots=2, device="cuda:0")
    y, u, v = synth_clip(2, 4, 320, 240, seed=5, device="cuda:0")
    q = enc.crf_qps(y)
    assert q.shape == (2, 4) and q.dtype == np.int32
    assert np.all(q[:, 0] <= q[:, 1])          # IDR gets the I/P offset
    res = enc.encode(y, u, v, metrics=False)
    assert all(len(r.bitstream) > 0 for r in res)
    assert "lookahead_s" in enc.timings
    enc.close()
    torch.cuda.synchronize()


def _mbtree_reference(blk, mv, strength):
    """numpy statement of csrc/kernels/mbtree.hip (x264 macroblock_tree_propagate)."""
    B, F, _, lbh, lbw = blk.shape
    prop = np.zeros((B, F, lbh, lbw))
    for b in range(B):
        for t in range(F - 1, 0, -1):
            for by in range(lbh):
                for bx in range(lbw):
                    intra = float(blk[b, t, 0, by, bx])
                    inter = min(float(blk[b, t, 1, by, bx]), intra)
                    if intra <= 0 or inter >= intra:
                        continue
                    amount = (prop[b, t, by, bx] + intra) * (intra - inter) / intra
                    m = int(mv[b, t, by, bx])
                    dx = ((m & 0xFFFF) ^ 0x8000) - 0x8000
                    dy = m >> 16
                    x, y = bx * 8 + dx, by * 8 + dy
                    x0, y0, fx, fy = x >> 3, y >> 3, x & 7, y & 7
                    for cy, wy in ((y0, 8 - fy), (y0 + 1, fy)):
                        for cx, wx in ((x0, 8 - fx), (x0 + 1, fx)):
                            if wx * wy and 0 <= cx < lbw and 0 <= cy < lbh:
                                prop[b, t - 1, cy, cx] += amount * wx * wy / 64.0
    intra = np.maximum(blk[:, :, 0].astype(np.float64), 1.0)
    return -strength * np.log2((intra + prop) / intra)


@pytest.mark.gpu
def test_mbtree_matches_reference():
    import torch

    from govideocompressor_amd.models.h264_gpu import synth_clip
    from govideocompressor_amd.rc.lookahead import GpuLookahead

    y, _, _ = synth_clip(2, 5, 160, 96, seed=3, device="cuda:0")
    la = GpuLookahead("cuda:0", 6, hierarchical=False)
    _, blk, mv = la.frame_costs(y, block_costs=True, block_mvs=True)
    _, off = la.mbtree(y, 2.0)
    torch.cuda.synchronize()
    ref = _mbtree_reference(blk.cpu().numpy().astype(np.int64), mv.cpu().numpy(), 2.0)
    got = off.cpu().numpy().reshape(ref.shape)
    assert np.allclose(got, ref, rtol=1e-4, atol=1e-3)
    assert (got[:, -1] == 0).all() and got[:, 0].mean() < -0.1  # early frames are referenced


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(2, 6, 64, 96), (1, 5, 70, 300)])
def test_lookahead_multi_matches_reference(shape):
    """x264 --b-adapt costs (la_multi): P at distances 2..4 and B between the neighbours,
    from small searches around the scaled distance-1 vectors -- exact against the numpy model
    (search clamps at the plane borders included: the 300-wide clip moves 5 px / frame)."""
    import torch
    from govideocompressor_amd.rc.lookahead import GpuLookahead, multi_reference

    y = _clip(*shape, seed=11)
    la = GpuLookahead("cuda", 6, hierarchical=False)
    yd = torch.from_numpy(y).cuda()
    _, blk, mv = la.frame_costs(yd, block_costs=True, block_mvs=True)
    got = la.multi_costs(yd, blk, mv, 4).cpu().numpy()
    got_intra = la.last_multi_intra.cpu().numpy()
    ref, ref_intra = multi_reference(y, 6, 4, with_intra=True)
    assert np.array_equal(got, ref), (got[..., :5], ref[..., :5])
    assert np.array_equal(got_intra, ref_intra), (got_intra[..., :5], ref_intra[..., :5])
    assert (ref[:, 2:, 2] > 0).all() and (ref[:, 1:-1, 0] > 0).all()


@pytest.mark.gpu
def test_hierarchical_lookahead_follows_fast_pans():
    """A texture panning 24 px / frame (12 lowres px, twice the lowres window of 6): the
    quarter-resolution search finds the motion, the lowres vectors follow it and inter costs
    stay far below intra; the window-only search cannot and prices the frames as new scenes."""
    import torch
    from govideocompressor_amd.rc.lookahead import GpuLookahead

    rng = np.random.default_rng(3)
    tex = rng.integers(0, 256, (40, 120)).astype(np.float64)
    tex = np.kron(tex, np.ones((4, 4)))  # 4-pixel texels: coarse enough to survive the downscales
    tex = (tex + np.roll(tex, 1, 0) + np.roll(tex, 1, 1)) / 3
    B, F, h, w = 1, 4, 128, 256
    y = np.stack([tex[:h, 24 * t:24 * t + w] for t in range(F)])[None].astype(np.uint8)
    yd = torch.from_numpy(np.ascontiguousarray(y)).cuda()
    out = {}
    for hier in (False, True):
        la = GpuLookahead("cuda", 6, hierarchical=hier)
        cost, blk, mv = la.frame_costs(yd, block_costs=True, block_mvs=True)
        torch.cuda.synchronize()
        c = cost.cpu().numpy()[0]
        m = mv.cpu().numpy()[0]
        dx = ((m & 0xFFFF) ^ 0x8000) - 0x8000
        out[hier] = (c[1:, 1].sum() / c[1:, 0].sum(), np.median(dx[1:, 2:-2, 2:-4]))
    ratio_h, dx_h = out[True]
    assert dx_h == 12, out          # frame t matches frame t - 1 twelve lowres pixels to the right
    assert ratio_h < 0.35, out      # inter prediction works
    assert out[False][0] > 2 * ratio_h, out


@pytest.mark.gpu
@pytest.mark.parametrize("R", [4, 6])
def test_weighted_lookahead_matches_reference_on_a_fade(R):
    """Lowres weighting: on a fade (brightness and contrast scaled per frame) the weights of
    every (picture, distance) pair equal the numpy model's, the weighted block costs match
    the model exactly (search and SATD on the inverse-weighted source, SATD scaled back), and
    the P costs drop well below the unweighted ones -- the fade stops looking like new content."""
    import torch

    from govideocompressor_amd.rc.lookahead import GpuLookahead, lowres_weights

    B, F, h, w = 2, 4, 64, 96
    y = _clip(B, F, h, w, seed=R + 7).astype(np.float64)
    gain = np.array([1.0, 0.8, 0.62, 0.47])[None, :, None, None]
    y = np.clip(np.rint(16 + (y - 16) * gain + 6 * np.arange(F)[None, :, None, None]), 0, 255).astype(np.uint8)
    yd = torch.from_numpy(y).to("cuda:0")
    plain = GpuLookahead("cuda:0", search_range=R, hierarchical=False)
    la = GpuLookahead("cuda:0", search_range=R, hierarchical=False, weighted=True)
    frame0 = plain.frame_costs(yd).cpu().numpy()
    frame, blk = la.frame_costs(yd, block_costs=True)
    torch.cuda.synchronize()
    wt_ref = lowres_weights(y)
    wt = la.last_weights.cpu().numpy()
    assert (wt_ref[:, 1:, 1, 0] > 0).all(), "every picture of the fade is weighted"
    np.testing.assert_allclose(wt, wt_ref, rtol=1e-6, atol=1e-4)
    ref_frame, ref_blk = lookahead_reference(y, search_range=R, weights=wt)
    got_blk = blk.cpu().numpy().astype(np.int64)
    bad = np.argwhere(got_blk != ref_blk)
    assert bad.size == 0, f"{len(bad)} block mismatches, first {bad[:4].tolist()}"
    frame = frame.cpu().numpy()
    assert np.array_equal(frame, ref_frame)
    # P costs (min(intra, inter)) of the faded pictures: weighted well below unweighted
    assert (frame[:, 1:, 1] < 0.8 * frame0[:, 1:, 1]).all(), (frame[:, :, 1], frame0[:, :, 1])


@pytest.mark.gpu
def test_weighted_lookahead_leaves_steady_content_alone():
    """No brightness or contrast change (the headline content class): no pair is weighted and
    the costs equal the unweighted lookahead's, so the default encode is unchanged."""
    import torch

    from govideocompressor_amd.rc.lookahead import GpuLookahead

    y = _clip(2, 4, 64, 96, seed=5)
    yd = torch.from_numpy(y).to("cuda:0")
    a = GpuLookahead("cuda:0", 6, hierarchical=True).frame_costs(yd).cpu().numpy()
    la = GpuLookahead("cuda:0", 6, hierarchical=True, weighted=True)
    b = la.frame_costs(yd).cpu().numpy()
    assert (la.last_weights.cpu().numpy()[..., 0] == 0).all()
    assert np.array_equal(a, b)
