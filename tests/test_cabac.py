"""CABAC entropy coding and High-profile 8x8 transform (T0/T2 tiers, CPU).

The CABAC writer (csrc/common/h264_cabac.h, shared with the gfx950 slice kernel) and the
independent decoder (csrc/host/h264_decoder.cc) are written separately; these tests pin
them against each other and against the CAVLC path:

* the same decision records coded with CAVLC and with CABAC decode to identical pictures
  (4x4 and 8x8 transforms, Intra4x4/8x8/16x16, all P partitions, per-MB QP deltas);
* the parse-only decoder recovers exactly the records the writer was given;
* encoder streams (CPU reference encoder) round-trip under CABAC.

Reference parity: x264's defaults behind `-vcodec libx264` (server.go:69-70) are CABAC +
High profile; a third-party CABAC stream is not available in this environment, so the
context-initialisation tables are parity-unpinned (see h264_cabac_tables.h).
"""
import numpy as np
import pytest

from govideocompressor_amd.utils import yuv
from govideocompressor_amd.utils.h264_synth import random_stream, unpack_levels

MBF_T8x8 = 2


@pytest.mark.parametrize("w,h,seed,t8", [(64, 48, 1, False), (96, 64, 2, False), (50, 34, 3, False),
                                         (96, 64, 4, True), (176, 144, 5, True), (34, 18, 6, True)])
def test_cabac_and_cavlc_decode_identically(host, w, h, seed, t8):
    a = random_stream(host, w, h, 5, seed=seed, cabac=False, t8x8=t8)
    b = random_stream(host, w, h, 5, seed=seed, cabac=True, t8x8=t8)
    pa, pb = host.decode(a), host.decode(b)
    assert len(pa) == len(pb) == 5
    for x, y in zip(pa, pb):
        assert np.array_equal(x["i420"], y["i420"])
        assert np.array_equal(x["mb_kind"], y["mb_kind"])
        assert np.array_equal(x["mv"], y["mv"])
    assert len(b) < len(a)  # CABAC is the more efficient coder of the same symbols


@pytest.mark.parametrize("t8", [False, True])
def test_cabac_parse_recovers_records(host, t8):
    w, h = 112, 80
    recs = []
    s = random_stream(host, w, h, 4, seed=11, cabac=True, t8x8=t8, records=recs)
    seg = host.parse([s], 1)[0]
    assert seg["error"] is None
    nmb = (w // 16) * (h // 16)
    for t, (hdr, coef) in enumerate(recs):
        got = seg["hdr"][t]
        lev = unpack_levels(seg, t)
        for mb in range(nmb):
            k_in, k_out = int(hdr[mb, 0]), int(got[mb, 0])
            if k_in in (2, 3) and k_out == 3:  # P16x16 / P_Skip hint coded as P_Skip
                continue
            assert k_in == k_out or (k_in == 3 and k_out == 2), (t, mb, k_in, k_out)
            cin = coef[mb].copy()
            if k_in == 1:
                for b in range(16):
                    cin[b * 16] = 0  # I16x16: AC blocks start at scan position 1
            if k_in == 1 or np.any(cin[:256]) or np.any(cin[272:]):
                assert got[mb, 2] == hdr[mb, 2]  # QP (coded through mb_qp_delta)
            if k_in not in (0, 1, 8):
                mv_in = np.frombuffer(hdr[mb, 16:32].tobytes(), np.int16)
                mv_out = np.frombuffer(got[mb, 16:32].tobytes(), np.int16)
                assert np.array_equal(mv_in, mv_out)
            if k_in == 8:
                assert np.array_equal(hdr[mb, 48:64], got[mb, 48:64])  # I8x8 modes
            assert np.array_equal(cin, lev[mb]), (t, mb, k_in)
            luma_coded = np.any(cin[:256] != 0)
            if t8 and luma_coded and k_in not in (0, 1):
                want = (k_in == 8) or bool(hdr[mb, 5] & MBF_T8x8)
                assert bool(got[mb, 5] & MBF_T8x8) == want


def test_cabac_cpu_encoder_roundtrip(host):
    c = yuv.synth_clip_cpu(5, 96, 64, seed=9)
    enc = host.CpuEncoder(dict(width=96, height=64, qp=28, cabac=1, keyint=5))
    es = enc.encode(c.i420(), 5, 0)
    pics = host.decode(es)
    assert len(pics) == 5
    rec = enc.recon().reshape(5, -1)
    for t, p in enumerate(pics):
        assert np.array_equal(p["i420"], rec[t])
    cav = host.CpuEncoder(dict(width=96, height=64, qp=28, cabac=0, keyint=5)).encode(c.i420(), 5, 0)
    assert len(es) < len(cav)


def test_cabac_parameter_sets_profiles(host):
    def sps_profile(ps):
        i = ps.index(b"\x00\x00\x00\x01\x67")
        return ps[i + 5]
    assert sps_profile(host.parameter_sets(dict(width=64, height=64))) == 66
    assert sps_profile(host.parameter_sets(dict(width=64, height=64, cabac=1))) == 77
    assert sps_profile(host.parameter_sets(dict(width=64, height=64, cabac=1, t8x8=1))) == 100


def test_cabac_large_levels_and_mvds(host):
    """Escape paths: coeff_abs_level_minus1 >= 14 (UEG0 suffix) and |mvd| >= 9 (UEG3)."""
    w, h = 64, 64
    cfg = dict(width=w, height=h, qp=20, cabac=1)
    nmb = 16
    out = [host.parameter_sets(cfg)]
    hdr = np.zeros((nmb, 64), np.uint8)
    hdr[:, 8:16] = 0xFF
    coef = np.zeros((nmb, 408), np.int16)
    rng = np.random.default_rng(3)
    for mb in range(nmb):
        hdr[mb, 0] = 1  # I16x16 DC pred
        hdr[mb, 3] = 2
        hdr[mb, 2] = 20
        coef[mb, 256:272] = rng.integers(-300, 300, 16)
        coef[mb, 272:280] = rng.integers(-40, 40, 8)
    out.append(host.write_slice(cfg, dict(idr=1, qp=20, frame_num=0), hdr, coef)[0])
    hdr2 = np.zeros((nmb, 64), np.uint8)
    hdr2[:, 8:16] = 0xFF
    coef2 = np.zeros((nmb, 408), np.int16)
    for mb in range(nmb):
        hdr2[mb, 0] = 2  # P16x16
        hdr2[mb, 2] = 20
        hdr2[mb, 8:12] = 0
        mv = rng.integers(-400, 400, 2)
        hdr2[mb, 16:32] = np.frombuffer(np.tile(mv.astype(np.int16), 4).tobytes(), np.uint8)
        coef2[mb, 0:16] = rng.integers(-100, 100, 16)
    out.append(host.write_slice(cfg, dict(idr=0, qp=20, frame_num=1), hdr2, coef2)[0])
    s = b"".join(out)
    seg = host.parse([s], 1)[0]
    assert seg["error"] is None
    lev = unpack_levels(seg, 1)
    assert np.array_equal(lev[:, 0:16], coef2[:, 0:16])
    got_mv = np.frombuffer(seg["hdr"][1][:, 16:20].tobytes(), np.int16).reshape(nmb, 2)
    want_mv = np.frombuffer(hdr2[:, 16:20].tobytes(), np.int16).reshape(nmb, 2)
    assert np.array_equal(got_mv, want_mv)
    assert len(host.decode(s)) == 2


@pytest.mark.parametrize("t8,seed", [(False, 21), (True, 22)])
def test_cabac_symbol_decomposition_is_exact(host, t8, seed):
    """The GPU's decomposition (each MB binarised on its own into 16-bit symbols, any order;
    then the symbols arithmetic-coded in MB order, bypass bins batched) yields exactly the
    serial writer's bytes."""
    w, h = 96, 80
    recs = []
    random_stream(host, w, h, 4, seed=seed, cabac=True, t8x8=t8, records=recs)
    cfg = dict(width=w, height=h, qp=28, cabac=1, t8x8=int(t8))
    for t, (hdr, coef) in enumerate(recs):
        fp = dict(idr=int(t == 0), qp=27 + t, frame_num=t)
        a, b, nsyms = host.cabac_slice_data_two_ways(cfg, fp, hdr, coef)
        assert a == b and nsyms > 0
