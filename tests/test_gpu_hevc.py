"""HEVC GPU encoder against the independent CPU decoder, bit-exact.

The GPU reconstruction (intra analysis + wavefront reconstruction, deblocking, SAO)
must equal what csrc/host/hevc_decoder.cc decodes from the CABAC bitstream the host
writer produced from the GPU's decision records -- for Main and Main 10 and with the
loop filters toggled (localises a mismatch to a stage).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _encode(w, h, F, B, bd=8, **kw):
    from govideocompressor_amd.models.h264_gpu import synth_clip
    from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams
    y, u, v = synth_clip(B, F, w, h, seed=7, bit_depth=bd)
    enc = GpuHevcEncoder(HevcParams(width=w, height=h, bit_depth=bd, **kw), slots=B)
    res = enc.encode(y, u, v, keep_recon=True)
    rec = enc.last_recon
    enc.close()
    return res, rec


def test_synth_10bit_is_native_10bit():
    """The 10-bit synth path renders the 8-bit content at 10-bit precision (low bits used),
    within the sensor-noise amplitude of 4x the 8-bit picture."""
    from govideocompressor_amd.models.h264_gpu import synth_clip
    y8, u8, v8 = synth_clip(2, 3, 200, 120, seed=4)
    y10, u10, v10 = synth_clip(2, 3, 200, 120, seed=4, bit_depth=10)
    assert y10.dtype == torch.int16 and y10.shape == y8.shape and u10.shape == u8.shape
    for a8, a10 in ((y8, y10), (u8, u10), (v8, v10)):
        assert int(a10.min()) >= 0 and int(a10.max()) <= 1023
        d = (a10.to(torch.int32) - 4 * a8.to(torch.int32)).abs().float()
        assert float(d.mean()) < 8.0
    frac = (y10 % 4 != 0).float().mean().item()
    assert frac > 0.5          # not 8-bit x 4: the two low bits carry content
    assert torch.equal(y10, synth_clip(2, 3, 200, 120, seed=4, bit_depth=10)[0])   # deterministic


def _compare(host, res, rec, skip_filters=False):
    for b, r in enumerate(res):
        pics = host.hevc_decode(r.bitstream, skip_filters)
        assert len(pics) == r.frames
        for t, p in enumerate(pics):
            for k, name in enumerate(("y", "u", "v")):
                g = rec[t][k][b].cpu().numpy().astype(np.uint16)
                d = p[name]
                if not np.array_equal(g, d):
                    diff = np.argwhere(g != d)
                    raise AssertionError(f"slot {b} pic {t} plane {name}: {len(diff)} samples differ, first "
                                         f"{diff[0].tolist()} gpu {g[tuple(diff[0])]} cpu {d[tuple(diff[0])]}")


@pytest.mark.parametrize("deblock,sao", [(False, False), (True, False), (True, True)])
def test_gpu_hevc_intra_matches_decoder(host, deblock, sao):
    res, rec = _encode(96, 64, 2, 2, intra_only=True, deblock=deblock, sao=sao, crf=None, qp=30)
    _compare(host, res, rec)


def test_gpu_hevc_intra_main10_cropped(host):
    res, rec = _encode(120, 68, 2, 2, bd=10, intra_only=True, crf=None, qp=27)
    _compare(host, res, rec)
    assert all(r.psnr_y > 30 for r in res)


@pytest.mark.parametrize("bd", [8, 10])
def test_gpu_hevc_p_pictures_match_decoder(host, bd):
    res, rec = _encode(128, 96, 5, 3, bd=bd, crf=None, qp=30, bframes=0)
    _compare(host, res, rec)
    for r in res:
        assert all(b > 0 for b in r.bits)
        assert sum(r.bits[1:]) / (r.frames - 1) < r.bits[0]   # P pictures are cheaper than the IDR


@pytest.mark.parametrize("bd,tmvp,pyramid", [(8, True, True), (10, True, True), (8, False, True), (8, True, False)])
def test_gpu_hevc_b_pictures_match_decoder(host, bd, tmvp, pyramid):
    """x265-style GOP: I, P anchors every 4 pictures and non-reference B pictures between
    them (list 0 / list 1 / bi-predicted CUs, bi-prediction averaging at 14-bit precision,
    B-aware deblocking strengths, TMVP candidates from the collocated anchor).  The GPU
    reconstruction equals the CPU decoder's, every inter direction occurs, and the B
    pictures cost less than the P anchors.  ``pyramid``: the middle B is a reference picture
    (coded first, at half the B QP offset) for the b pictures beside it."""
    res, rec = _encode(192, 128, 9, 2, bd=bd, crf=None, qp=28, bframes=3, tmvp=tmvp, pyramid=pyramid)
    _compare(host, res, rec)
    dirs = set()
    for r in res:
        assert r.order == ([0, 4, 2, 1, 3, 8, 6, 5, 7] if pyramid else [0, 4, 1, 2, 3, 8, 5, 6, 7])
        pics = host.hevc_decode(r.bitstream)
        for p in pics:
            inter = p["cu"][:, 0] == 1
            dirs |= set(p["cu"][inter, 12].tolist())
        assert [p["slice_type"] for p in pics] == [2, 0, 0, 0, 1, 0, 0, 0, 1]
        bits = dict(zip(r.order, r.bits))
        pb = np.mean([bits[d] for d in (4, 8)])
        bb = np.mean([bits[d] for d in (1, 2, 3, 5, 6, 7)])
        assert bb < 0.8 * pb
    assert {1, 2, 3} <= dirs


def test_gpu_hevc_b_segment_prefix(host):
    """A segment shorter than the batch ends on an anchor (anchors_at), so its pictures
    form a coding-order prefix that decodes on its own."""
    from govideocompressor_amd.models.h264_gpu import synth_clip
    from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams
    y, u, v = synth_clip(2, 9, 128, 96, seed=3)
    enc = GpuHevcEncoder(HevcParams(width=128, height=96, crf=None, qp=30), slots=2)
    res = enc.encode(y, u, v, keep_recon=True, anchors_at=[5])
    rec = enc.last_recon
    enc.close()
    _compare(host, res, rec)
    nals = res[0].display_prefix(6)
    pics = host.hevc_decode(enc.parameter_sets() + b"".join(nals))
    assert [p["poc"] for p in pics] == list(range(6))
    for t, p in enumerate(pics):
        assert np.array_equal(p["y"], rec[t][0][0].cpu().numpy().astype(np.uint16))


def test_gpu_backend_hevc_preset(host, tmp_path):
    """The reference's "265" preset through the GPU backend: pieces -> HEVC streams."""
    from govideocompressor_amd.backends import get_backend
    from govideocompressor_amd.jobs import ffargs
    from govideocompressor_amd.utils import yuv
    be = get_backend("gpu")
    clips = [(str(i), yuv.synth_clip_cpu(6, 160, 96, seed=i)) for i in range(3)]
    out = be.impl.encode_clips(clips, ffargs.parse(ffargs.expand_preset("265")))
    for key, c in clips:
        stream, st = out[key]
        pics = host.hevc_decode(stream)
        assert len(pics) == 6 and st["codec"] == "hevc"
        ref = c.y.astype(np.float64)
        dec = np.stack([p["y"][:96, :160] for p in pics]).astype(np.float64)
        mse = np.mean((ref - dec) ** 2)
        # cutree's CRF compensation ((1 - qcomp) * 13.5 QP, as x265) dominates a 6-frame piece
        assert 10 * np.log10(255 ** 2 / mse) > 27
    be.close()


def test_gpu_backend_hevc_mp4_piece(host, tmp_path):
    """Job path with the reference's piece naming (``<idx>.mp4``, client.go:54): the HEVC
    piece is written as an hvc1 MP4 that demuxes back to a decodable stream."""
    from govideocompressor_amd.backends import PieceJob, get_backend
    from govideocompressor_amd.segment import mp4_hevc
    from govideocompressor_amd.utils import yuv
    c = yuv.synth_clip_cpu(5, 160, 96, seed=3)
    src = tmp_path / "0.y4m"
    yuv.write_y4m(str(src), c)
    be = get_backend("gpu")
    (r,) = be.run([PieceJob("0", str(src), str(tmp_path / "c0.mp4"))], "-c:v libx265 -crf 26")
    be.close()
    assert r.ok, r.reason
    data = open(tmp_path / "c0.mp4", "rb").read()
    assert mp4_hevc.is_hevc_mp4(data)
    pics = host.hevc_decode(mp4_hevc.demux(data))
    assert len(pics) == 5 and pics[0]["idr"]


def test_gpu_hevc_scenecut(host):
    """A hard cut inside a segment is detected by the lookahead and the cut picture is
    coded with intra CUs only; the reconstruction stays bit-exact with the decoder."""
    from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams
    # the cut lies past keyint_min (25) from the IDR: x264 / x265's scene-cut bias makes a cut
    # right after a key frame need an inter cost of ~97.5 % of the intra cost, which a motion
    # search over hundreds of candidates undercuts even on unrelated noise
    w, h, B, F, cut = 128, 96, 2, 30, 27
    y, u, v = _cut_clip(B, F, w, h, cut, seed=7)
    enc = GpuHevcEncoder(HevcParams(width=w, height=h), slots=B)
    res = enc.encode(y, u, v, keep_recon=True)
    rec = enc.last_recon
    assert enc._scenecuts[:, cut].all() and enc.stats["scenecuts"] >= B
    enc.close()
    _compare(host, res, rec)
    for r in res:
        bits = dict(zip(r.order, r.bits))
        pics = host.hevc_decode(r.bitstream)
        assert not (pics[cut]["cu"][:, 0] == 1).any()   # intra CUs only
        assert bits[cut] > 1.3 * bits[cut + 1]        # the all-intra cut picture costs more than the next one


@pytest.mark.parametrize("wpp", [True, False])
def test_gpu_hevc_adaptive_qp(host, wpp):
    """Per-CTB QPs (variance AQ + cutree, cu_qp_delta): the reconstruction stays bit-exact
    with the decoder (dequantisation and deblocking at each CU's QpY), the decoded CTB QPs
    equal the GPU's records after the QP fix-up, and they actually vary."""
    from govideocompressor_amd.models.h264_gpu import synth_clip
    from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams
    w, h, B, F = 160, 128, 2, 4
    y, u, v = synth_clip(B, F, w, h, seed=5)
    enc = GpuHevcEncoder(HevcParams(width=w, height=h, wpp=wpp), slots=B)
    assert enc.p.host_cfg()["cu_qp_delta"] == 1
    res = enc.encode(y, u, v, keep_recon=True)
    rec = enc.last_recon
    ctu_last = enc.ctu.cpu().numpy()  # records of the last picture in coding order
    enc.close()
    _compare(host, res, rec)
    qps = set()
    for b, r in enumerate(res):
        pics = host.hevc_decode(r.bitstream)
        q = pics[r.order[-1]]["ctu"][:, 1].view(np.int8)
        assert np.array_equal(q, ctu_last[b][:, 1].view(np.int8))
        for p in pics:
            qps |= set(p["ctu"][:, 1].view(np.int8).tolist())
    assert len(qps) > 3


@pytest.mark.parametrize("bd", [8, 10])
def test_gpu_hevc_intra_nxn(host, bd):
    """Intra PART_NxN (four 4x4 PUs, DST luma TUs) is chosen on detailed content at a low QP,
    in I and P pictures, and the reconstruction stays bit-exact with the decoder."""
    res, rec = _encode(128, 96, 3, 2, bd=bd, crf=None, qp=22)
    _compare(host, res, rec)
    n = 0
    for r in res:
        for p in host.hevc_decode(r.bitstream):
            n += int(((p["cu"][:, 3] & 8) != 0).sum())
    assert n > 0


@pytest.mark.parametrize("bd", [8, 10])
def test_gpu_hevc_inter_tu_split(host, bd):
    """tu_inter_depth 1: inter CUs pick one TU or four quarter TUs by RD; the split CUs
    (split_transform_flag, per-quarter cbfs, transform edges inside the CU for deblocking)
    decode bit-exactly, and some CUs do split."""
    res, rec = _encode(128, 96, 5, 2, bd=bd, crf=None, qp=24, tu_inter_depth=1)
    _compare(host, res, rec)
    n = sum(int(((p["cu"][:, 3] & 16) != 0).sum()) for r in res for p in host.hevc_decode(r.bitstream))
    assert n > 0


def test_gpu_hevc_sign_data_hiding(host):
    """sign_data_hiding_enabled_flag: the GPU quantiser's parity fix (intra 4x4 / 8x8 mode
    dependent scans, inter diagonal) keeps the decoder bit-exact in I and P pictures."""
    res, rec = _encode(128, 96, 4, 2, crf=None, qp=22, sdh=True)
    _compare(host, res, rec)


@pytest.mark.parametrize("ctu64", [False, True])
@pytest.mark.parametrize("wpp", [True, False])
def test_gpu_hevc_ctu64(host, ctu64, wpp):
    """x265 --ctu 64: the 32x32 record blocks are reconstructed in z-order inside 64x64 CTUs
    (intra availability across blocks and CTUs), each block is a quantization group whose QP
    prediction uses the left / above block of the same CTU (AQ on: CRF with variance AQ and
    cutree), one SAO parameter set per CTU, partial CTUs at the right and bottom edges, with
    and without WPP -- bit-exact against the CPU decoder."""
    res, rec = _encode(160, 96, 5, 2, crf=26, bframes=1, wpp=wpp, ctu64=ctu64)
    _compare(host, res, rec)
    res, rec = _encode(96, 64, 2, 2, intra_only=True, crf=None, qp=27, ctu64=ctu64, wpp=wpp)
    _compare(host, res, rec)


@pytest.mark.parametrize("ctu64", [False, True])
def test_gpu_hevc_1080p_matches_decoder(host, ctu64):
    """Full-HD pictures: a 1080p-only fault (a non-inlined recon call site faulted at 1920x1080
    and never at the small test sizes) must show up here.  CTU 32 and 64 (x265 --ctu),
    2 slots x 4 pictures with the default GOP (B + P), bit-exact with the CPU decoder; then the
    GPU decoder reproduces the same pictures from the bitstreams."""
    from govideocompressor_amd.models.hevc_decode_gpu import GpuHevcDecoder
    res, rec = _encode(1920, 1080, 4, 2, crf=26, ctu64=ctu64)
    _compare(host, res, rec)
    dec = GpuHevcDecoder().decode([r.bitstream for r in res])
    for b, (r, d) in enumerate(zip(res, dec)):
        pics = sorted((p for p in host.hevc_decode_full(r.bitstream, True, False) if p["display"] >= 0),
                      key=lambda p: p["display"])
        assert d.frames == len(pics) == r.frames
        for t, p in enumerate(pics):
            assert np.array_equal(d.y[t].cpu().numpy().astype(np.uint16), p["y"][:1080]), (b, t)
            assert np.array_equal(d.v[t].cpu().numpy().astype(np.uint16), p["v"][:540]), (b, t)


def test_gpu_hevc_weightp_fade_matches_decoder(host):
    """x265 --weightp: on a fade the P pictures carry explicit weights (pred_weight_table,
    luma and chroma offsets) and the GPU reconstruction stays bit-exact with the CPU decoder;
    the weighted stream is smaller than the unweighted one."""
    from govideocompressor_amd.models.h264_gpu import synth_clip
    from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams
    y, u, v = synth_clip(2, 8, 192, 128, seed=9, kind="fade")
    sizes = {}
    for wp in (False, True):
        enc = GpuHevcEncoder(HevcParams(width=192, height=128, crf=27.0, bframes=0, weightp=wp), slots=2)
        res = enc.encode(y, u, v, keep_recon=True)
        rec = enc.last_recon
        if wp:
            assert enc.stats.get("weightp_pictures", 0) > 0
            _compare(host, res, rec)
        sizes[wp] = sum(len(r.bitstream) for r in res)
        enc.close()
    assert sizes[True] < sizes[False], sizes


def test_gpu_hevc_weightp_main10_fade_matches_decoder(host):
    """Main 10 weightp: statistics of the 16-bit planes (wp_stats16), offsets coded in 8-bit
    units and scaled by 4 in the prediction -- GPU reconstruction bit-exact with the CPU
    decoder, and the weighted stream smaller than the unweighted one."""
    from govideocompressor_amd.models.h264_gpu import synth_clip
    from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams
    y, u, v = synth_clip(2, 8, 192, 128, seed=9, kind="fade", bit_depth=10)
    sizes = {}
    for wp in (False, True):
        enc = GpuHevcEncoder(HevcParams(width=192, height=128, crf=27.0, bframes=0, weightp=wp, bit_depth=10), slots=2)
        res = enc.encode(y, u, v, keep_recon=True)
        rec = enc.last_recon
        if wp:
            assert enc.stats.get("weightp_pictures", 0) > 0
            _compare(host, res, rec)
        sizes[wp] = sum(len(r.bitstream) for r in res)
        enc.close()
    assert sizes[True] < sizes[False], sizes


def test_gpu_hevc_weightp_fade_to_flat_matches_decoder(host):
    """A fade to a flat picture: the current plane's variance collapses, so the luma / chroma
    weight quantises towards 0.  The slot must stay weighted (weight >= 1, the kernels read 0 as
    "not weighted") so encoder and decoder predict the same samples (round-4 review)."""
    from govideocompressor_amd.models.h264_gpu import synth_clip
    from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams
    y, u, v = synth_clip(2, 8, 192, 128, seed=11)
    a = torch.tensor([1.0, 0.7, 0.4, 0.15, 0.0, 0.0, 0.0, 0.0], device=y.device).view(1, 8, 1, 1)
    y = (16 + (y.float() - 16) * a).round().clamp(0, 255).to(torch.uint8)
    u = (128 + (u.float() - 128) * a).round().clamp(0, 255).to(torch.uint8)
    v = (128 + (v.float() - 128) * a).round().clamp(0, 255).to(torch.uint8)
    enc = GpuHevcEncoder(HevcParams(width=192, height=128, crf=27.0, bframes=0, weightp=True, wp_min_scale=0.05),
                         slots=2)
    res = enc.encode(y, u, v, keep_recon=True)
    rec = enc.last_recon
    assert enc.stats.get("weightp_pictures", 0) > 0
    _compare(host, res, rec)
    enc.close()


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


@pytest.mark.parametrize("entropy", ["host", "gpu"])
def test_gpu_hevc_encode_async_same_bytes(entropy):
    """encode_async + analyse_async (bench/run.py config 4: batch k's CABAC jobs and result
    assembly overlap batch k + 1's GPU work, the next batch's lookahead runs on a side stream;
    the pinned host buffer sets, record double buffers and copy events cross the batch boundary)
    give the bytes of the synchronous encode, batch by batch -- host or GPU entropy stage."""
    from govideocompressor_amd.models.h264_gpu import synth_clip
    from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams
    clips = [synth_clip(2, 9, 192, 128, seed=s, kind=k) for s, k in ((21, "default"), (22, "cuts"), (23, "fade"))]
    ref_enc = GpuHevcEncoder(HevcParams(width=192, height=128, crf=27.0), slots=2, entropy=entropy)
    ref = [[r.bitstream for r in ref_enc.encode(*c, metrics=False)] for c in clips]
    ref_enc.close()
    enc = GpuHevcEncoder(HevcParams(width=192, height=128, crf=27.0), slots=2, entropy=entropy)
    side = torch.cuda.Stream()
    pend = []
    for c in clips:
        ana = enc.analyse_async(c[0], stream=side)
        pend.append(enc.encode_async(*c, metrics=False, analysis=ana))
    got = [[r.bitstream for r in p.result()] for p in pend]
    torch.cuda.synchronize()
    assert got == ref
    enc.close()


def test_gpu_hevc_ctb32_config4_shape(host):
    """-preset ultrafast's geometry (32x32 CTBs, ctu64=False) at config-4 shape with B pictures:
    16 slots x 8 pictures of 1080p in one batch (the round-4 scratch log had hevc_intra_recon
    fault here when its per-CTB call was not inlined: a 544 B call frame on a 147 KB-LDS
    workgroup; the call is now inlined and each component is its own workgroup).  Three slots
    are compared bit-exactly with the CPU decoder, every slot must decode."""
    res, rec = _encode(1920, 1080, 8, 16, crf=26, ctu64=False, bframes=1)
    assert len(res) == 16
    pick = [0, 7, 15]
    _compare(host, [res[b] for b in pick], [tuple(plane[pick] for plane in t) for t in rec])
    for r in res:
        assert r.frames == 8 and len(r.bitstream) > 0


@pytest.mark.parametrize("bframes,kind,ctu64", [(0, 0, True), (1, 0, False), (1, "fade", True)])
def test_gpu_hevc_multiref_matches_decoder(host, bframes, kind, ctu64):
    """x265 --ref 3: P pictures search their farther list-0 pictures (scaled-vector seeds), pick
    per block at cost + ref_idx bins, and the merge passes carry candidates' refIdx (zero
    candidates counting through the list); motion compensation, deblocking (refIdx in the
    boundary strength), TMVP from multi-reference collocated pictures and explicit weights on
    RefPicList0[0] only (fade) -- bit-exact with the CPU decoder.  Content that repeats every
    second anchor makes the farther pictures win, so refIdx > 0 must occur."""
    from govideocompressor_amd.models.h264_gpu import synth_clip
    from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams
    w, h, F, B = 160, 96, 8, 3
    y, u, v = synth_clip(B, F, w, h, seed=9, kind=kind)
    # anchors of equal content every other anchor: d -> source frame
    step = bframes + 1
    perm = [d if d % step else (0 if (d // step) % 2 == 0 else step) for d in range(F)]
    idx = torch.tensor(perm, device=y.device)
    y, u, v = (t.index_select(1, idx).contiguous() for t in (y, u, v))
    enc = GpuHevcEncoder(HevcParams(width=w, height=h, crf=28, bframes=bframes, refs=3, ref_gate=0, ctu64=ctu64),
                         slots=B)
    res = enc.encode(y, u, v, keep_recon=True)
    rec = enc.last_recon
    enc.close()
    _compare(host, res, rec)
    far = 0
    for r in res:
        for p in host.hevc_decode(r.bitstream):
            if p["slice_type"] == 1:
                cu = p["cu"]
                far += int(((cu[:, 0] == 1) & (cu[:, 13] > 0)).sum())
    assert far > 0


@pytest.mark.parametrize("bd,ctu64", [(8, True), (10, False)])
def test_gpu_hevc_inter8_matches_decoder(host, bd, ctu64):
    """8x8 inter CUs in P pictures (per-quadrant vectors from the HEVC form of p_part8x8): the
    split quadrant's four CUs are predicted, transformed (8x8 luma / 4x4 chroma TUs) and
    reconstructed one after another in hevc_inter_cu, deblocked on the 8x8 grid, and the writer
    codes them with their own merge / AMVP decisions -- bit-exact with the CPU decoder, and
    some 8x8 inter CUs must occur (split overhead 0, no SATD floor)."""
    res, rec = _encode(160, 96, 6, 3, bd=bd, crf=24, bframes=1, ctu64=ctu64, inter8=True, inter8_overhead=0,
                       inter8_min_satd=0)
    _compare(host, res, rec)
    n8 = 0
    for r in res:
        for p in host.hevc_decode(r.bitstream):
            cu = p["cu"]
            n8 += int(((cu[:, 0] == 1) & (((cu[:, 3] >> 1) & 3) == 0)).sum())
    assert n8 > 0


def test_gpu_hevc_badapt_matches_decoder(host):
    """x265 --b-adapt (one lowres-cost placement per batch, runs of up to 3 B pictures with the
    pyramid's reference B, 3 list-0 pictures): bit-exact with the CPU decoder, and the placement
    is not the fixed pattern on static content (longer runs)."""
    from govideocompressor_amd.models.h264_gpu import synth_clip
    from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams
    w, h, F, B = 160, 96, 10, 2
    y, u, v = synth_clip(B, F, w, h, seed=11, kind="static")
    enc = GpuHevcEncoder(HevcParams(width=w, height=h, crf=28, bframes=3, b_adapt=1), slots=B)
    res = enc.encode(y, u, v, keep_recon=True)
    rec = enc.last_recon
    order = list(enc.last_order)
    enc.close()
    _compare(host, res, rec)
    assert order != list(range(F))          # B pictures were placed
    assert enc.stats.get("b_ratio", 0) > 0


@pytest.mark.parametrize("kw", [dict(), dict(ctu64=False), dict(wpp=False), dict(bit_depth=10),
                                dict(bframes=0, refs=3), dict(intra_only=True)])
def test_gpu_hevc_entropy_matches_host_writer(host, kw):
    """The GPU CABAC stage (kernels/hevc_entropy.hip: the host writer's coder run per WPP row
    on the device, substreams packed to pinned memory, headers + entry points on the host)
    gives the same bytes as the host writer on the same decision records, for CTU 64 / 32,
    with and without WPP, Main 10, several references and intra-only -- and they decode."""
    from govideocompressor_amd.models.h264_gpu import synth_clip
    from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams
    bd = kw.pop("bit_depth", 8)
    w, h, F, B = 352, 200, 7, 3
    y, u, v = synth_clip(B, F, w, h, seed=11, bit_depth=bd)
    out = {}
    for ent in ("gpu", "host"):
        enc = GpuHevcEncoder(HevcParams(width=w, height=h, bit_depth=bd, **kw), slots=B, entropy=ent)
        out[ent] = [r.bitstream for r in enc.encode(y, u, v, metrics=False)]
        enc.close()
    assert out["gpu"] == out["host"]
    for bs in out["gpu"]:
        assert len(host.hevc_decode(bs, False)) == F


def test_gpu_hevc_entropy_4k_dense_matches_host_writer():
    """4K at a low QP: 34 CTU rows over the coder's 8 waves (rows round-robin per wave), CTUs
    with more non-zero 4x4 blocks than the per-CTU LDS stage holds (the rest read from the level
    planes), and an I picture larger than the pinned output buffer (read back from the device
    area instead) -- the GPU coder still gives the host writer's bytes."""
    from govideocompressor_amd.models.h264_gpu import synth_clip
    from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams
    y, u, v = synth_clip(1, 3, 3840, 2160, seed=12, kind="noise")
    out = {}
    for ent in ("gpu", "host"):
        enc = GpuHevcEncoder(HevcParams(width=3840, height=2160, crf=None, qp=14, lookahead=False), slots=1, entropy=ent)
        out[ent] = enc.encode(y, u, v, metrics=False)[0].bitstream
        if ent == "gpu":
            assert enc.stats.get("entropy_readback_steps", 0) >= 1, enc.stats
        enc.close()
    assert len(out["gpu"]) > 1_000_000
    assert out["gpu"] == out["host"]
