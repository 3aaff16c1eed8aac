"""GPU H.264 encoder: the reconstruction the kernels produce must equal what the
independent CPU decoder reconstructs from the emitted bitstream, bit for bit
(SURVEY.md §4.2 tiers T1/T2)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(width, height, slots, frames, **kw):
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip

    p = H264Params(width=width, height=height, **kw)
    enc = GpuH264Encoder(p, slots=slots)
    y, u, v = synth_clip(slots, frames, width, height, seed=3)
    res = enc.encode(y, u, v, keep_recon=True)
    torch.cuda.synchronize()
    return enc, res, (y, u, v)


def _check_roundtrip(host, enc, res, width, height):
    for b, r in enumerate(res):
        pics = host.decode(r.bitstream)
        assert len(pics) == r.frames
        for t, pic in enumerate(pics):
            ry, ru, rv = (x[b].cpu().numpy() for x in enc.last_recon[t])
            dy, du, dv = pic["y_coded"], pic["u_coded"], pic["v_coded"]
            assert np.array_equal(dy, ry), f"slot {b} frame {t}: luma mismatch ({(dy != ry).sum()} px)"
            assert np.array_equal(du, ru), f"slot {b} frame {t}: Cb mismatch"
            assert np.array_equal(dv, rv), f"slot {b} frame {t}: Cr mismatch"


@pytest.mark.parametrize("qp", [22, 30])
def test_gpu_h264_roundtrip_small(host, qp):
    enc, res, _ = _run(176, 144, slots=2, frames=4, crf=None, qp=qp)
    _check_roundtrip(host, enc, res, 176, 144)
    for r in res:
        assert r.psnr_y > 30


def test_gpu_h264_roundtrip_no_deblock_no_i4(host):
    enc, res, _ = _run(176, 144, slots=2, frames=3, crf=None, qp=26, deblock=False, i4x4=False)
    _check_roundtrip(host, enc, res, 176, 144)


def test_gpu_h264_cavlc_roundtrip(host):
    enc, res, _ = _run(176, 144, slots=2, frames=4, crf=None, qp=26, cabac=False)
    _check_roundtrip(host, enc, res, 176, 144)


@pytest.mark.parametrize("bframes", [0, 3])
def test_gpu_h264_partitions_roundtrip(host, bframes):
    """P_8x8 / P_16x8 / P_8x16 (x264 --partitions p8x8): quadrant vectors from p_part8x8,
    chroma MC per quadrant, partition mvds through the GPU CABAC binariser -- the CPU
    decoder reconstructs the same pictures, and the split shapes actually occur."""
    enc, res, _ = _run(352, 288, slots=2, frames=9, crf=None, qp=24, bframes=bframes, part_overhead=0,
                          part_min_satd=0)
    _check_roundtrip(host, enc, res, 352, 288)
    kinds = np.concatenate([np.asarray(p["mb_kind"]).ravel() for r in res for p in host.decode(r.bitstream)])
    assert np.isin(kinds, [5, 6, 7]).sum() > 0, np.bincount(kinds.astype(np.int64) + 1)


def test_gpu_h264_partitions_cut_bits(host):
    """The split is taken only where it pays: same QP, fewer bits than 16x16-only P MBs
    at no PSNR cost beyond noise."""
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip

    y, u, v = synth_clip(4, 8, 640, 368, seed=21)
    out = {}
    for part in (True, False):
        enc = GpuH264Encoder(H264Params(width=640, height=368, crf=None, qp=26, bframes=0, partitions=part), slots=4)
        rs = enc.encode(y, u, v)
        out[part] = (sum(r.nbytes() for r in rs), float(np.mean([r.psnr_y for r in rs])))
        enc.close()
    torch.cuda.synchronize()
    (b1, p1), (b0, p0) = out[True], out[False]
    assert b1 < b0 * 1.005 and p1 > p0 - 0.05, out


def test_gpu_cabac_smaller_than_cavlc(host):
    """Same decisions, CABAC vs CAVLC: CABAC saves bits (x264 documents ~10-15 %)."""
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip

    y, u, v = synth_clip(2, 6, 352, 288, seed=5)
    size = {}
    for cabac in (True, False):
        enc = GpuH264Encoder(H264Params(width=352, height=288, crf=None, qp=27, cabac=cabac, bframes=0), slots=2)
        size[cabac] = sum(r.nbytes() for r in enc.encode(y, u, v))
        enc.close()
    torch.cuda.synchronize()
    assert size[True] < 0.97 * size[False], size


def test_gpu_h264_roundtrip_1080p(host):
    enc, res, _ = _run(1920, 1080, slots=2, frames=3, crf=23)
    _check_roundtrip(host, enc, res, 1920, 1080)
    for r in res:
        assert r.psnr_y > 33


@pytest.mark.parametrize("cabac", [True, False])
def test_gpu_entropy_matches_host_writer(host, cabac):
    """GPU CABAC / CAVLC bitstreams must be byte-identical to the host writer's for the same
    decisions (the CABAC kernel runs the shared csrc/common/h264_cabac.h coder)."""
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip

    for (w, h, qp) in [(176, 144, 24), (352, 288, 32), (1920, 1080, 23)]:
        p = H264Params(width=w, height=h, crf=None, qp=qp, cabac=cabac)
        y, u, v = synth_clip(3, 4, w, h, seed=11)
        out = {}
        for mode in ("cpu", "gpu"):
            enc = GpuH264Encoder(p, slots=3, entropy=mode)
            out[mode] = [r.bitstream for r in enc.encode(y, u, v, idr_base=5)]
            enc.close()
        for b in range(3):
            assert out["gpu"][b] == out["cpu"][b], f"{w}x{h} slot {b}: GPU entropy coder differs from host writer"
        torch.cuda.synchronize()


@pytest.mark.parametrize("group", [1, 2, 3])
def test_gpu_cabac_groups_match_host_writer(host, group):
    """The arithmetic coder runs over groups of frame steps from a double-buffered symbol
    pool: group sizes that wrap the ring several times (and leave a partial last group)
    give the host writer's bytes."""
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip

    w, h, B, F = 176, 144, 3, 7
    p = H264Params(width=w, height=h, crf=None, qp=26)
    y, u, v = synth_clip(B, F, w, h, seed=13)
    out = {}
    for mode in ("cpu", "gpu"):
        enc = GpuH264Encoder(p, slots=B, entropy=mode, cabac_group=group)
        out[mode] = [r.bitstream for r in enc.encode(y, u, v)]
        enc.close()
    assert out["gpu"] == out["cpu"]
    torch.cuda.synchronize()


@pytest.mark.parametrize("cabac", [True, False])
def test_gpu_per_frame_qps(host, cabac):
    """Rate-control QPs per (slot, frame): GPU entropy coder == host writer, and the recon roundtrips."""
    import numpy as np
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip

    w, h, B, F = 176, 144, 3, 5
    rng = np.random.default_rng(4)
    qps = rng.integers(18, 40, size=(B, F))
    p = H264Params(width=w, height=h, aq_strength=0.0, cabac=cabac)  # every MB at its frame's QP
    y, u, v = synth_clip(B, F, w, h, seed=2)
    out = {}
    for mode in ("cpu", "gpu"):
        enc = GpuH264Encoder(p, slots=B, entropy=mode)
        res = enc.encode(y, u, v, qps=qps, keep_recon=(mode == "gpu"))
        out[mode] = [r.bitstream for r in res]
        if mode == "gpu":
            _check_roundtrip(host, enc, res, w, h)
        enc.close()
    assert out["gpu"] == out["cpu"]
    for b in range(B):
        pics = host.decode(out["gpu"][b])
        assert [int(np.median(p["mb_qp"])) for p in pics] == qps[b].tolist()
    torch.cuda.synchronize()


def test_gpu_scenecut_codes_cut_frames_intra(host):
    """A hard cut inside a segment: the lookahead flags it (x264 --scenecut 40), the frame
    is coded with every MB intra at the I-frame QP, and the recon still roundtrips."""
    import numpy as np
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip

    # past keyint_min (25) from the IDR, where x264's scene-cut bias allows a cut at an inter
    # cost of 90 % of the intra cost (right after a key frame it needs ~97.5 %)
    w, h, B, F, cut = 176, 144, 2, 30, 27
    y, u, v = _cut_clip(B, F, w, h, cut, seed=2)
    enc = GpuH264Encoder(H264Params(width=w, height=h), slots=B)
    res = enc.encode(y, u, v, keep_recon=True)
    torch.cuda.synchronize()
    assert enc._scenecuts[:, cut].all() and enc.stats["scenecuts"] >= B
    _check_roundtrip(host, enc, res, w, h)
    for r in res:
        pics = host.decode(r.bitstream)
        kinds = np.asarray(pics[cut]["mb_kind"])
        assert np.isin(kinds, [0, 1, 4, 8]).all()       # I4x4 / I16x16 / I_PCM / I8x8 only
        inter = [2, 3, 5, 6, 7, 9, 10, 11, 12, 13]  # P and B kinds: the cut is an anchor
        assert np.isin(np.asarray(pics[cut + 1]["mb_kind"]), inter).mean() > 0.5
        assert r.psnr_y > 25   # (uniform noise after the cut)
    enc.close()


def test_gpu_adaptive_quant(host):
    """x264-style variance AQ: per-MB QPs differ inside a picture, MBs without
    mb_qp_delta carry QP_pred in their records (deblocking stays bit-exact), and the GPU
    CAVLC equals the host writer on the same records."""
    import numpy as np
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip

    w, h, B, F = 176, 144, 2, 4
    y, u, v = synth_clip(B, F, w, h, seed=11)
    out = {}
    for mode in ("cpu", "gpu"):
        enc = GpuH264Encoder(H264Params(width=w, height=h, crf=None, qp=28, aq_strength=1.0), slots=B, entropy=mode)
        res = enc.encode(y, u, v, keep_recon=(mode == "gpu"))
        out[mode] = [r.bitstream for r in res]
        if mode == "gpu":
            _check_roundtrip(host, enc, res, w, h)
            offs = enc.aq.cpu().numpy()
            assert offs.std() > 0.5 and abs(int(offs.max())) <= 24
            # golden: x264 ac_energy (luma 16x16 + chroma 8x8 variances) of the last frame
            sy, su, sv = (x.cpu().numpy().astype(np.int64) for x in enc.src)
            for bb in range(B):
                for my in range(enc.hmb):
                    for mx in range(enc.wmb):
                        e = 0
                        for pl, n in ((sy[bb, my * 16:my * 16 + 16, mx * 16:mx * 16 + 16], 8),
                                      (su[bb, my * 8:my * 8 + 8, mx * 8:mx * 8 + 8], 6),
                                      (sv[bb, my * 8:my * 8 + 8, mx * 8:mx * 8 + 8], 6)):
                            e += int((pl * pl).sum()) - ((int(pl.sum()) ** 2) >> n)
                        ref = int(np.rint(1.0397 * (np.log2(max(e, 1)) - 14.427)))
                        assert abs(int(offs[bb, my * enc.wmb + mx]) - max(-24, min(24, ref))) <= 1
        enc.close()
    assert out["gpu"] == out["cpu"]
    for b in range(B):
        pics = host.decode(out["gpu"][b])
        assert any(np.unique(np.asarray(p["mb_qp"])).size > 3 for p in pics)
    torch.cuda.synchronize()


def test_gpu_h264_wide_multiband_roundtrip(host):
    """Rows wider than the deblocking waves' combined ring slack, over several 32-row bands
    (the band-boundary hand-off of deblock.hip): bit-exact and no wavefront stall."""
    enc, res, _ = _run(4096, 544, slots=1, frames=2, crf=None, qp=30)
    _check_roundtrip(host, enc, res, 4096, 544)
    assert int(enc.err.item()) == 0


@pytest.mark.parametrize("bframes,frames", [(3, 9), (2, 7), (1, 4)])
def test_gpu_bframes_roundtrip(host, bframes, frames):
    """B pictures (temporal direct, B_16x16 L0 / L1 / Bi): decoder output == GPU recon for
    every picture in display order; slice types follow the I P B.. coding order."""
    enc, res, _ = _run(176, 144, slots=3, frames=frames, crf=None, qp=27, bframes=bframes)
    _check_roundtrip(host, enc, res, 176, 144)
    from govideocompressor_amd.models.h264_gpu import gop_plan
    plan = gop_plan(frames, bframes)
    pics = host.decode(res[0].bitstream)
    kinds = {p.d: p.kind for p in plan}
    assert [{"I": 2, "P": 0, "B": 1}[kinds[d]] for d in range(frames)] == [p["slice_type"] % 5 for p in pics]
    assert res[0].order == [p.d for p in plan]


def test_gpu_bframes_save_bits(host):
    """x264's --bframes 3 on 1080p bench content in CRF mode (B pictures at their references'
    QP + pbratio): a real saving -- the rate at equal PSNR-Y, interpolated between CRF 21 and
    27 (log rate vs PSNR), at least 10 % below P-only (the content suite measures -36 % on this
    class: profiles/r4_bframes_rd.md)."""
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip

    y, u, v = synth_clip(2, 25, 1920, 1080, seed=7)
    pts = {}
    for nb in (0, 3):
        enc = GpuH264Encoder(H264Params(width=1920, height=1080, crf=21.0, bframes=nb), slots=2)
        pts[nb] = []
        for crf in (21.0, 27.0):
            enc.p.crf = crf
            res = enc.encode(y, u, v)
            pts[nb].append((float(np.log(sum(len(r.bitstream) for r in res))), float(np.mean([r.psnr_y for r in res]))))
        enc.close()
    torch.cuda.synchronize()
    # log rate of the B configuration at the P-only configuration's mean PSNR
    (r0a, q0a), (r0b, q0b) = pts[0]
    (r3a, q3a), (r3b, q3b) = pts[3]
    q = 0.5 * (q0a + q0b)
    lr0 = r0a + (r0b - r0a) * (q - q0a) / (q0b - q0a)
    lr3 = r3a + (r3b - r3a) * (q - q3a) / (q3b - q3a)
    assert np.exp(lr3 - lr0) < 0.90, pts


def test_gpu_short_segment_display_prefix(host):
    """A segment shorter than the batch ends on a forced anchor: its display prefix is a
    decodable stream of exactly its pictures (the worker backend's padded chunks)."""
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip

    y, u, v = synth_clip(2, 10, 176, 144, seed=9)
    enc = GpuH264Encoder(H264Params(width=176, height=144, crf=None, qp=28, bframes=3), slots=2)
    res = enc.encode(y, u, v, keep_recon=True, anchors_at=[5])
    torch.cuda.synchronize()
    ps = enc.parameter_sets()
    pics = host.decode(ps + b"".join(res[1].display_prefix(6)))
    assert len(pics) == 6
    for t, pic in enumerate(pics):
        assert np.array_equal(pic["y_coded"], enc.last_recon[t][0][1].cpu().numpy())
    enc.close()


def test_nonref_b_deblock_skip_keeps_bytes():
    """Without metrics / keep_recon the non-reference B pictures skip the in-loop filter;
    the bitstream must not change (nothing predicts from them)."""
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip
    enc = GpuH264Encoder(H264Params(width=176, height=144, crf=24, bframes=3), slots=2)
    y, u, v = synth_clip(2, 9, 176, 144, seed=8)
    a = enc.encode(y, u, v, metrics=True)
    b = enc.encode(y, u, v, metrics=False)
    enc.close()
    assert [r.bitstream for r in a] == [r.bitstream for r in b]


@pytest.mark.parametrize("qp", [20, 30])
def test_gpu_h264_intra8x8(host, qp):
    """x264's Intra8x8 (High profile, --partitions i8x8): filtered reference samples, 9
    modes ranked on sa8d, the 8x8 transform in the closed loop.  The CPU decoder
    reconstructs the same pictures (8x8-transform-aware deblocking included), I8x8 MBs
    occur, and the IDR pictures get no bigger than with Intra4x4 / Intra16x16 alone."""
    enc, res, _ = _run(352, 288, slots=2, frames=3, crf=None, qp=qp, bframes=0)
    _check_roundtrip(host, enc, res, 352, 288)
    kinds = np.concatenate([np.asarray(p["mb_kind"]).ravel() for r in res for p in host.decode(r.bitstream)[:1]])
    assert (kinds == 8).sum() > 0
    enc0, res0, _ = _run(352, 288, slots=2, frames=3, crf=None, qp=qp, bframes=0, i8x8=False)
    i8 = sum(len(r.nals[0]) for r in res)
    i4 = sum(len(r.nals[0]) for r in res0)
    assert i8 <= 1.01 * i4
    enc.close()
    enc0.close()


@pytest.mark.parametrize("bframes", [0, 3])
def test_gpu_h264_multiref_roundtrip(host, bframes):
    """x264 --ref 3: P macroblocks choose among the three latest anchors (ref_idx through the
    GPU CABAC binariser, chroma MC from the chosen picture, deblocking across different
    references) and B pictures' temporal direct follows the co-located block's reference
    (per-reference DistScaleFactor and implicit weights) -- bit-exact against the CPU decoder,
    and farther pictures are actually chosen."""
    # ref_gate 0: every MB searches the farther pictures (the default gate 3000 leaves this
    # small clip on the nearest one)
    enc, res, _ = _run(352, 288, slots=2, frames=13, crf=None, qp=26, bframes=bframes, refs=3, ref_gate=0)
    _check_roundtrip(host, enc, res, 352, 288)
    assert enc.stats.get("p_far_ref_ratio", 0.0) > 0.0, enc.stats


def test_gpu_h264_multiref_gate_and_one_ref(host):
    """refs=1 keeps the single-reference path (no override in the slice headers); a gate that
    skips every MB's far search leaves the decisions on RefPicList0[0] and decodes the same."""
    enc, res, _ = _run(176, 144, slots=2, frames=9, crf=None, qp=28, bframes=3, refs=1)
    _check_roundtrip(host, enc, res, 176, 144)
    enc, res, _ = _run(176, 144, slots=2, frames=9, crf=None, qp=28, bframes=0, refs=2, ref_gate=1 << 20)
    _check_roundtrip(host, enc, res, 176, 144)
    assert enc.stats.get("p_far_ref_ratio", 1.0) == 0.0, enc.stats


def _fade_clip(slots, frames, w, h, seed=5):
    import torch
    from govideocompressor_amd.models.h264_gpu import synth_clip
    y, u, v = synth_clip(slots, frames, w, h, seed=seed)
    f = torch.linspace(1.0, 0.35, frames, device=y.device).view(1, frames, 1, 1)
    y = (y.float() * f + 0.5).clamp(0, 255).to(torch.uint8)
    u = ((u.float() - 128) * f + 128.5).clamp(0, 255).to(torch.uint8)
    v = ((v.float() - 128) * f + 128.5).clamp(0, 255).to(torch.uint8)
    return y.contiguous(), u.contiguous(), v.contiguous()


@pytest.mark.parametrize("bframes,refs", [(0, 1), (3, 3)])
def test_gpu_h264_weightp_fade(host, bframes, refs):
    """x264 --weightp on a fade to black: P pictures carry pred_weight_table() (explicit luma
    and chroma weights of RefPicList0[0], inverse-weighted source for the motion search,
    forward weights on the chosen prediction in encode_inter) -- bit-exact against the CPU
    decoder, and fewer bits than the unweighted encode at the same QP."""
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params
    y, u, v = _fade_clip(2, 9, 352, 288)
    out = {}
    for wpon in (True, False):
        enc = GpuH264Encoder(H264Params(width=352, height=288, crf=None, qp=26, bframes=bframes, refs=refs,
                                        weightp=wpon), slots=2)
        res = enc.encode(y, u, v, keep_recon=True)
        torch.cuda.synchronize()
        _check_roundtrip(host, enc, res, 352, 288)
        out[wpon] = (sum(r.nbytes() for r in res), enc.stats.get("weightp_pictures", 0))
        enc.close()
    assert out[True][1] > 0 and out[False][1] == 0, out
    assert out[True][0] < out[False][0] * 0.97, out


def test_gpu_h264_segment_bytes_independent_of_batch_neighbours():
    """A segment's bytes do not depend on what else its batch holds: a static segment encoded
    next to a fading one (whose P pictures get explicit weights, so the step runs the
    weighted path) equals its encode alone -- no identity pred_weight_table.  Segment-parallel
    jobs (bench/run.py config 3 over any rank count) rely on it."""
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip
    fy, fu, fv = _fade_clip(1, 8, 320, 192)
    sy, su, sv = synth_clip(1, 8, 320, 192, seed=9)
    both = [torch.cat([a, b]).contiguous() for a, b in ((sy, fy), (su, fu), (sv, fv))]
    out = []
    for clip, B in ((both, 2), ((sy, su, sv), 1)):
        enc = GpuH264Encoder(H264Params(width=320, height=192, crf=23.0), slots=B)
        out.append(enc.encode(*clip, idr_ids=[0] * B, metrics=False)[0].bitstream)
        if B == 2:
            assert enc.stats.get("weightp_pictures", 0) > 0, enc.stats
        enc.close()
    assert out[0] == out[1]


def test_gpu_h264_weightp_static_content_unweighted(host):
    """Content without brightness changes gets no weights (no pred_weight_table entries)."""
    enc, res, _ = _run(176, 144, slots=2, frames=5, crf=None, qp=28, bframes=0)
    _check_roundtrip(host, enc, res, 176, 144)
    assert enc.stats.get("weightp_pictures", 0) == 0, enc.stats


def test_gpu_h264_b_partitions_roundtrip(host):
    """x264 --partitions b8x8: B macroblocks whose quadrants prefer different candidates
    (direct, L0, L1, bi) are coded as B_16x8 / B_8x16 / B_8x8 (with B_Direct_8x8 quadrants);
    the CPU decoder reconstructs the same pictures and the split shapes occur."""
    enc, res, _ = _run(352, 288, slots=2, frames=9, crf=None, qp=24, bframes=3, b_gate=0)
    _check_roundtrip(host, enc, res, 352, 288)
    kinds = np.concatenate([np.asarray(p["mb_kind"]).ravel() for r in res for p in host.decode(r.bitstream)])
    assert np.isin(kinds, [10, 11, 12]).sum() > 0, np.bincount(kinds.astype(np.int64) + 1)
    enc, res, _ = _run(352, 288, slots=2, frames=9, crf=None, qp=24, bframes=3, b_gate=-150, bpartitions=False)
    _check_roundtrip(host, enc, res, 352, 288)


@pytest.mark.parametrize("refs", [1, 3])
def test_gpu_h264_spatial_direct_roundtrip(host, refs):
    """x264 --direct spatial: the direct MBs' motion derived from their final neighbours in an
    MB wavefront (MinPositive reference indices, the 16x16 predictor, colZeroFlag per quadrant)
    and weighed there against each MB's explicit candidate -- bit-exact against the CPU decoder (direct_spatial_mv_pred_flag
    1 in the B slice headers), with and without several reference pictures."""
    enc, res, _ = _run(352, 288, slots=2, frames=13, crf=None, qp=26, bframes=3, refs=refs, direct="spatial")
    _check_roundtrip(host, enc, res, 352, 288)


@pytest.mark.parametrize("pyramid", [False, True])
def test_gpu_h264_per_slot_plans_roundtrip(host, pyramid):
    """Every slot follows its own GOP plan (csrc/kernels/route.h): at one coding step slot 0
    codes a P picture while slot 1 codes a B picture and slot 2 a reference B (b-pyramid),
    each predicting from its own pool buffers.  Every slot's stream is bit-exact against
    the CPU decoder, the plans really differ, and a P picture after a reference B carries a
    ref_pic_list_modification (its list 0 is POC-distance ordered)."""
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip

    W, H, F = 176, 144, 13
    p = H264Params(width=W, height=H, crf=None, qp=26, bframes=3, refs=3, pyramid=pyramid,
                   direct="spatial" if pyramid else "temporal", part_overhead=0, part_min_satd=0)
    enc = GpuH264Encoder(p, slots=3)
    y, u, v = synth_clip(3, F, W, H, seed=5)
    res = enc.encode(y, u, v, keep_recon=True, anchors_at=[[], [2, 3, 7], [5, 6, 10]])
    torch.cuda.synchronize()
    plans = enc.last_plans
    assert len({tuple(q.d for q in pl) for pl in plans}) == 3
    mixed = [t for t in range(F) if len({plans[b][t].kind for b in range(3)}) > 1]
    assert mixed, "no coding step mixed picture types"
    if pyramid:
        assert any(q.kind == "B" and q.ref for pl in plans for q in pl)
        assert any(q.mod_l0 for pl in plans for q in pl)
    _check_roundtrip(host, enc, res, W, H)
    enc.close()


def test_gpu_h264_pyramid_spatial_roundtrip_b8x8(host):
    """b-pyramid with spatial direct at the default partitions (B_8x8 with direct quadrants):
    the co-located picture of the non-reference B pictures is a reference B, whose list-1-only
    blocks give their list-1 motion to colZeroFlag (8.4.1.2.1) -- bit-exact vs the CPU decoder."""
    # b-adapt 0: x264's fixed pattern, so the runs of 3 B pictures (and their reference B) occur
    enc, res, _ = _run(352, 288, slots=2, frames=17, crf=24, bframes=3, refs=3, pyramid=True, direct="spatial",
                       b_adapt=0)
    _check_roundtrip(host, enc, res, 352, 288)
    assert any(q.kind == "B" and q.ref for q in enc.last_plans[0])
    enc.close()


@pytest.mark.parametrize("wavefront", [False, True])
def test_gpu_h264_spatial_direct_modes_roundtrip(host, wavefront):
    """Spatial direct, both decision paths: the fast one (parallel pricing of an estimate, then
    the exact decoding-order derivation + re-prediction) and the wavefront one -- every B
    picture bit-exact against the CPU decoder, with direct MBs present."""
    enc, res, _ = _run(352, 288, slots=2, frames=9, crf=26, bframes=3, direct="spatial",
                       spatial_wavefront=wavefront)
    _check_roundtrip(host, enc, res, 352, 288)
    kinds = np.concatenate([np.asarray(p["mb_kind"]).ravel() for r in res for p in host.decode(r.bitstream)])
    assert (kinds == 13).sum() > 0
    enc.close()


@pytest.mark.parametrize("entropy", ["gpu", "cpu"])
def test_gpu_h264_slices_roundtrip(host, entropy):
    """--slices 4 (whole MB rows): the intra wavefront treats every slice's first row as having
    nothing above, QP prediction restarts per slice, the GPU CABAC codes one slice per lane --
    the CPU decoder reconstructs the encoder's pictures from the multi-slice stream (with
    B pictures, AQ and intra MBs in P / B pictures), and the picture really holds 4 slices."""
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip
    w, h = 352, 288  # 18 MB rows -> slices of 5, 5, 5, 3 rows
    p = H264Params(width=w, height=h, crf=24.0, slices=4)
    assert p.eff_slices() == 4 and p.slice_rows() == 5
    enc = GpuH264Encoder(p, slots=3, entropy=entropy)
    y, u, v = synth_clip(3, 9, w, h, seed=11, kind="cuts")
    res = enc.encode(y, u, v, keep_recon=True)
    torch.cuda.synchronize()
    _check_roundtrip(host, enc, res, w, h)
    for r in res:
        for nal in r.nals:
            assert nal.count(b"\x00\x00\x01") == 4   # four slice NAL units per picture


def test_gpu_h264_slices_spatial_direct_roundtrip(host):
    """Spatial direct over slices: the exact decoding-order derivation (b_spatial_exact) treats a
    slice's first MB row as having no neighbours above, as the decoder does."""
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip
    p = H264Params(width=352, height=288, crf=24.0, slices=3, direct="spatial")
    enc = GpuH264Encoder(p, slots=2)
    y, u, v = synth_clip(2, 9, 352, 288, seed=12)
    res = enc.encode(y, u, v, keep_recon=True)
    torch.cuda.synchronize()
    _check_roundtrip(host, enc, res, 352, 288)


def test_gpu_async_lookahead_same_bytes():
    """analyse_async (the next batch's lookahead on a side stream while the current one
    encodes, bench.py) must give the bytes of the inline lookahead."""
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip

    enc = GpuH264Encoder(H264Params(width=320, height=240, crf=23), slots=3)
    a = synth_clip(3, 12, 320, 240, seed=5, kind="cuts")
    b = synth_clip(3, 12, 320, 240, seed=6)
    ref = [[r.bitstream for r in enc.encode(*c, metrics=False)] for c in (a, b)]
    side = torch.cuda.Stream()
    fa = enc.analyse_async(a[0])
    with torch.cuda.stream(side):
        ev = torch.cuda.Event()
        ev.record(side)
    fb = enc.analyse_async(b[0], after=ev)
    got_a = [r.bitstream for r in enc.encode(*a, metrics=False, analysis=fa)]
    got_b = [r.bitstream for r in enc.encode(*b, metrics=False, analysis=fb)]
    assert got_a == ref[0] and got_b == ref[1]
    assert enc.timings.get("lookahead_async_s", 0) > 0


def _cut_clip(B, F, w, h, cut, seed):
    """synth_clip frames, then from frame ``cut`` a new scene: uniform noise panning by whole
    pixels -- the old scene predicts none of it (the cut frame's inter cost is ~intra, a cut
    even right after a key frame under x264's scene-cut bias), while the frames after the cut
    predict each other exactly."""
    import numpy as np
    import torch
    from govideocompressor_amd.models.h264_gpu import synth_clip
    a = synth_clip(B, F, w, h, seed=seed)
    rng = np.random.default_rng(seed)
    out = []
    for c, pa in enumerate(a):
        ph, pw = pa.shape[2], pa.shape[3]
        sh = 1 if c == 0 else 2
        canvas = rng.integers(0, 256, (B, ph + 2 * F, pw + 4 * F), dtype=np.uint8)
        new = np.stack([canvas[:, t // sh:t // sh + ph, (2 * t) // sh:(2 * t) // sh + pw] for t in range(F)], axis=1)
        new = torch.from_numpy(np.ascontiguousarray(new)).to(pa.device)
        out.append(torch.cat([pa[:, :cut], new[:, cut:]], dim=1).contiguous())
    return out


@pytest.mark.parametrize("tiny_pool", [False, True])
def test_gpu_encode_async_same_bytes(monkeypatch, tiny_pool):
    """encode_async (bench.py: batch k's entropy tail overlaps batch k + 1's first kernels;
    the CABAC rings, error flags and counters cross the batch boundary) gives the bytes of
    the synchronous encode, batch by batch -- also when a batch overflows the symbol pool
    and is re-encoded with a grown pool while the next one is in flight."""
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip

    clips = [synth_clip(3, 10, 320, 240, seed=s, kind=k) for s, k in ((11, "default"), (12, "cuts"), (13, "fade"))]
    ref_enc = GpuH264Encoder(H264Params(width=320, height=240, crf=23), slots=3)
    ref = [[r.bitstream for r in ref_enc.encode(*c, metrics=False)] for c in clips]
    ref_enc.close()
    if tiny_pool:
        monkeypatch.setenv("MIVC_CABAC_SYMS_PER_MB", "2")
        monkeypatch.setenv("MIVC_CABAC_PEAK_SYMS_PER_MB", "4")
    enc = GpuH264Encoder(H264Params(width=320, height=240, crf=23), slots=3)
    pend = [enc.encode_async(*c, metrics=False) for c in clips]
    got = [[r.bitstream for r in p.result()] for p in pend]
    torch.cuda.synchronize()
    assert got == ref
    if tiny_pool:
        assert enc.stats.get("cabac_pool_regrow", 0) >= 1
    enc.close()


def test_gpu_intra_in_p_rows_of_one_wave(host):
    """Intra MBs in a P picture, in two rows the same wave codes (rows y and y + 16 of the
    16-wave encoder, y and y + 8 / y + 16 of the 8-wave decoder): the second row's first intra
    MB is one column right of the first row's last one.  The LDS copy of the left MB's
    right edge must not be taken for it (it used to be keyed by the column alone, which
    showed as different bytes from the 8- and 16-wave intra kernels): the encoder's recon
    equals the CPU decoder's, and the GPU decoder reconstructs the same pictures."""
    from tests.test_gpu_decode import _check

    w, h = 320, 288
    enc, res, spots = _intra_spots_encode(w, h)
    pics = host.decode(res[0].bitstream)
    kinds = np.asarray(pics[1]["mb_kind"]).reshape(h // 16, w // 16)
    intra = np.isin(kinds, [0, 1, 4, 8])
    assert all(intra[my, mx] for mx, my in spots), kinds
    for my in (0, 1):  # nothing between the spots that would refresh the cache legitimately
        assert not intra[my, spots[2 * my][0] + 1:].any() and not intra[my + 16, :spots[2 * my + 1][0]].any(), kinds
    _check_roundtrip(host, enc, res, w, h)
    enc.close()
    from govideocompressor_amd.models.h264_decode_gpu import GpuH264Decoder
    _check(host, GpuH264Decoder(), [res[0].bitstream])


def _intra_spots_encode(w=320, h=288):
    """Noise background, static; in the second (P) picture four MBs whose rows repeat the
    sample left of the MB (Intra16x16 H predicts them, the reference does not)."""
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params

    rng = np.random.default_rng(17)
    planes = []
    for ph, pw in ((h, w), (h // 2, w // 2), (h // 2, w // 2)):
        bg = rng.integers(0, 256, (ph, pw), dtype=np.uint8)
        planes.append(np.stack([bg, bg.copy()])[None])
    y1 = planes[0][0, 1]
    spots = [(3, 0), (4, 16), (10, 1), (11, 17)]
    for mx, my in spots:
        rows = slice(my * 16, my * 16 + 16)
        y1[rows, mx * 16:mx * 16 + 16] = y1[rows, mx * 16 - 1:mx * 16]
    y, u, v = (torch.from_numpy(np.ascontiguousarray(p)).cuda() for p in planes)
    enc = GpuH264Encoder(H264Params(width=w, height=h, crf=None, qp=26, bframes=0), slots=1)
    res = enc.encode(y, u, v, keep_recon=True)
    torch.cuda.synchronize()
    return enc, res, spots


@pytest.mark.parametrize("waves", ["8", "16"])
def test_gpu_intra_waves_knob_keeps_bytes(waves):
    """MIVC_INTRA_WAVES=8 / 16 (the other intra kernel instances) is a speed knob: same bytes
    as the default 12-wave instance (the launcher reads the variable once, so the other run is
    a child process)."""
    import hashlib
    import os
    import subprocess
    import sys

    enc, res, _ = _intra_spots_encode()
    here = hashlib.sha256(res[0].bitstream).hexdigest()
    enc.close()
    code = ("import hashlib; from tests.test_gpu_h264 import _intra_spots_encode; "
            "print(hashlib.sha256(_intra_spots_encode()[1][0].bitstream).hexdigest())")
    env = dict(os.environ, MIVC_INTRA_WAVES=waves)
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.split()[-1] == here


def _multi_wg_bytes():
    import hashlib
    import torch
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip
    enc = GpuH264Encoder(H264Params(width=320, height=240, crf=None, qp=24), slots=8)
    y, u, v = synth_clip(8, 3, 320, 240, seed=29)
    res = enc.encode(y, u, v, keep_recon=True)
    torch.cuda.synchronize()
    return enc, res, hashlib.sha256(b"".join(r.bitstream for r in res)).hexdigest()


def test_gpu_intra_multi_workgroup_wavefront(host):
    """I pictures of a batch with few slice wavefronts deal each slice's MB rows to several
    workgroups (device-scope progress counters, 8 slots -> 4 workgroups per slot here): the
    reconstruction still equals the CPU decoder's, and the bytes equal the one-workgroup
    wavefront's (MIVC_INTRA_WG=1 in a child process)."""
    import os
    import subprocess
    import sys
    enc, res, here = _multi_wg_bytes()
    _check_roundtrip(host, enc, res, 320, 240)
    enc.close()
    code = "from tests.test_gpu_h264 import _multi_wg_bytes; print(_multi_wg_bytes()[2])"
    out = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, MIVC_INTRA_WG="1"), capture_output=True,
                         text=True, timeout=110, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.split()[-1] == here
