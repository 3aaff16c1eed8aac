"""T0/T2 on the host library: Exp-Golomb, CAVLC tables and known answers, NAL
emulation prevention, the CPU reference encoder against the independent decoder,
MP4 mux/demux, the Intra4x4 tap table."""
import itertools

import numpy as np
import pytest

from govideocompressor_amd.utils import yuv


def _bits(data, n):
    return "".join(f"{b:08b}" for b in data)[:n]


def test_exp_golomb_known_answers(host):
    data, n = host.exp_golomb([0, 1, 2, 3, 4, 7, 8], False)
    assert _bits(data, n) == "1" "010" "011" "00100" "00101" "0001000" "0001001"
    data, n = host.exp_golomb([0, 1, -1, 2, -2], True)
    assert _bits(data, n) == "1" "010" "011" "00100" "00101"
    vals = list(range(0, 300, 7))
    d, _ = host.exp_golomb(vals, False)
    assert host.read_exp_golomb(d, len(vals), False) == vals
    sv = [-100, -1, 0, 5, 1000]
    d, _ = host.exp_golomb(sv, True)
    assert host.read_exp_golomb(d, len(sv), True) == sv


def _prefix_free(codes):
    codes = [c for c in codes if c]
    for a, b in itertools.permutations(codes, 2):
        if b.startswith(a):
            return False
    return True


def test_coeff_token_tables_prefix_free_and_kraft(host):
    lens, bits = host.table("coeff_token_len"), host.table("coeff_token_bits")
    for t in range(3):   # the fourth table (nC >= 8) is a fixed 6-bit code
        codes = [format(b, f"0{ln}b") for ln, b in zip(lens[t], bits[t]) if ln > 0]
        assert _prefix_free(codes)
        assert sum(2.0 ** -len(c) for c in codes) <= 1.0 + 1e-12
    assert all(ln == 6 for ln in lens[3] if ln > 0)
    cl, cb = host.table("chroma_dc_coeff_token")
    codes = [format(b, f"0{ln}b") for ln, b in zip(cl, cb) if ln > 0]
    assert _prefix_free(codes)


def test_total_zeros_and_run_before_prefix_free(host):
    tl, tb = host.table("total_zeros_len"), host.table("total_zeros_bits")
    for tc in range(15):
        codes = [format(b, f"0{ln}b") for ln, b in zip(tl[tc], tb[tc]) if ln > 0]
        assert len(codes) == 16 - tc and _prefix_free(codes)
    rl, rb = host.table("run_before_len"), host.table("run_before_bits")
    for zl in range(7):
        codes = [format(b, f"0{ln}b") for ln, b in zip(rl[zl], rb[zl]) if ln > 0]
        assert _prefix_free(codes)


def test_cavlc_richardson_example(host):
    # the classic worked example, block 0 3 -1 0 / 0 -1 1 0 / 1 0 0 0 / 0 0 0 0, given in scan order
    coef = [0, 3, 0, 1, -1, -1, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0]
    data, n, tc = host.cavlc_block(coef, 0, 15, 16, 0)
    assert tc == 5
    assert _bits(data, n) == "000010001110010111101101"


def test_cbp_mapping_tables_are_permutations(host):
    assert sorted(host.table("intra_cbp")[0]) == list(range(48))
    assert sorted(host.table("inter_cbp")[0]) == list(range(48))
    assert sorted(host.table("zigzag")[0]) == list(range(16))


def test_nal_emulation_prevention(host):
    nal = host.nal_wrap(bytes([0, 0, 0, 0, 0, 1, 0, 0, 2, 5]), 3, 5)
    assert nal[:5] == b"\x00\x00\x00\x01\x65"
    body = nal[5:]
    assert b"\x00\x00\x00" not in body and b"\x00\x00\x01" not in body and b"\x00\x00\x02" not in body
    many = host.nal_wrap_many(np.frombuffer(b"\x01\x02\x00\x00\x01", dtype=np.uint8), [2, 3], 2, 1)
    assert many[0] == b"\x00\x00\x00\x01\x41\x01\x02"
    assert many[1] == b"\x00\x00\x00\x01\x41\x00\x00\x03\x01"
    parsed = host.parse_nals(nal + many[0])
    assert [p[0] for p in parsed] == [5, 1]


@pytest.mark.parametrize("w,h,qp", [(48, 32, 20), (50, 34, 34), (176, 144, 27)])
def test_cpu_encoder_decoder_roundtrip(host, w, h, qp):
    c = yuv.synth_clip_cpu(5, w, h, seed=w + qp)
    enc = host.CpuEncoder(dict(width=w, height=h, qp=qp, keyint=3))
    es = enc.encode(c.i420(), c.frames, 7)
    pics = host.decode(es)
    assert len(pics) == 5 and [p["idr"] for p in pics] == [1, 0, 0, 1, 0]
    rec = np.asarray(enc.recon()).reshape(5, -1)
    for t, p in enumerate(pics):
        assert np.array_equal(p["i420"], rec[t])
    unf = host.decode(es, skip_deblock=True)
    ru = np.asarray(enc.recon_unfiltered())
    cw, ch = (w + 15) // 16 * 16, (h + 15) // 16 * 16
    fs = cw * ch * 3 // 2
    for t, p in enumerate(unf):
        if p["idr"]:   # P pictures of a skip_deblock decode predict from unfiltered references
            fr = ru[t * fs:(t + 1) * fs]
            assert np.array_equal(p["y_coded"].reshape(-1), fr[: cw * ch])
    st = enc.stats()
    assert all(s["psnr_y"] > 28 for s in st)
    info = host.stream_info(es)
    assert (info["width"], info["height"], info["frames"], info["idr_frames"]) == (w, h, 5, 2)
    assert info["profile_idc"] == 66 and info["entropy"] == "cavlc"


def test_cpu_encoder_no_deblock_recon(host):
    c = yuv.synth_clip_cpu(4, 64, 48, seed=2)
    enc = host.CpuEncoder(dict(width=64, height=48, qp=30, deblock=0))
    es = enc.encode(c.i420(), 4, 0)
    ru = np.asarray(enc.recon_unfiltered()).reshape(4, -1)
    for t, p in enumerate(host.decode(es)):
        assert np.array_equal(p["y_coded"].reshape(-1), ru[t, : 64 * 48])


def test_mp4_roundtrip(host):
    c = yuv.synth_clip_cpu(4, 64, 48, seed=1)
    es = host.CpuEncoder(dict(width=64, height=48, qp=30)).encode(c.i420(), 4, 0)
    mp4 = host.mp4_mux(es, 25.0)
    assert mp4[4:8] == b"ftyp" and b"moov" in mp4 and b"avcC" in mp4
    back = host.mp4_demux(mp4)
    a, b = host.decode(back), host.decode(es)
    assert len(a) == 4 and all(np.array_equal(x["i420"], y["i420"]) for x, y in zip(a, b))
    assert abs(host.stream_info(back)["fps"] - 25.0) < 1e-6 or host.stream_info(back)["fps"] in (0.0, 30.0, 25.0)


def test_concat_requires_start_codes(host):
    with pytest.raises(Exception):
        host.concat([b"\x01\x02\x03\x04\x05"])


def test_i4x4_tap_table(host):
    assert host.selftest_i4_taps(2000, 1) == 0


def test_lowres_costs(host):
    c = yuv.synth_clip_cpu(4, 64, 48, seed=3)
    frames = np.ascontiguousarray(c.i420())  # I420 frames back to back (luma read, chroma skipped)
    intra, inter = host.lowres_costs(frames, 64, 48, 4)
    assert len(intra) == 4 and all(x > 0 for x in intra)
    assert inter[1] <= intra[1] * 1.5


@pytest.mark.parametrize("cqm,coded,seed", [(1, 0xFF, 0), (2, 0xFF, 1), (2, 0b01011001, 2), (3, 0xFF, 3), (3, 0b10010110, 4)])
def test_scaling_matrices_roundtrip(host, cqm, coded, seed):
    """H.264 scaling matrices (7.3.2.1.1.1, 8.5.9): the default matrices (x264 --cqm jvt), custom
    lists in the SPS, and PPS lists over SPS defaults, with lists left out so that fall-back
    rules A and B apply.  The CPU encoder quantises and reconstructs with the weights the
    decoder derives; the decoder's unfiltered output equals that reconstruction on every
    frame, and the weights change the bitstream against flat matrices."""
    rng = np.random.default_rng(seed)
    w, h, n = 96, 64, 4
    c = yuv.synth_clip_cpu(n, w, h, seed=seed)
    base = dict(width=w, height=h, qp=28, keyint=2, deblock=0, t8x8=1, cabac=seed % 2)
    cfg = dict(base, cqm=cqm, cqm_coded=coded, cqm4=rng.integers(4, 64, (6, 16)).astype(np.uint8),
               cqm8=rng.integers(4, 64, (2, 64)).astype(np.uint8))
    enc = host.CpuEncoder(cfg)
    es = enc.encode(c.i420(), n, 0)
    ru = np.asarray(enc.recon_unfiltered())
    cw, ch = (w + 15) // 16 * 16, (h + 15) // 16 * 16
    fs = cw * ch * 3 // 2
    pics = host.decode(es)
    assert len(pics) == n
    for t, p in enumerate(pics):
        fr = ru[t * fs:(t + 1) * fs]
        assert np.array_equal(p["y_coded"].reshape(-1), fr[: cw * ch]), t
        assert np.array_equal(p["u_coded"].reshape(-1), fr[cw * ch: cw * ch + cw * ch // 4]), t
    flat = host.CpuEncoder(base).encode(c.i420(), n, 0)
    assert flat != es
    assert host.stream_info(es)["profile_idc"] == 100
