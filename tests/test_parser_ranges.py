"""Exp-Golomb range hardening of the H.264 / HEVC parameter-set and slice-header parsers.

A ue(v) code with 32 leading zeros carries values up to 2^32 - 1 (2^33 - 2 with a full
suffix).  Narrowed to ``int`` these wrap to negative numbers, and ``+ 1`` turns 2^32 - 1
into 0, so checks that only reject large values used to pass them (round-4 review):
``num_tile_columns_minus1`` -> 0 columns -> ``cw[-1]`` heap write, ``delta_idx_minus1`` ->
``sets[idx + 1]``, ``collocated_ref_idx`` -> ``refs[-1]``, ``luma_log2_weight_denom`` ->
a negative shift.  Every such read now goes through ``BitReader::get_ue_max`` /
``get_se_range`` (csrc/host/bitstream.h), which compare the raw code with the element's
legal range before any narrowing.

The streams come from the independent writer in tests/hevc_kat.py (which records where
each Exp-Golomb code sits) and a small H.264 parameter-set writer below; every code of
every NAL is replaced by wrap-inducing values and the decoders must reject the stream with
an exception (under tools/asan_tests.sh: with no sanitizer report)."""
import numpy as np
import pytest

from hevc_kat import Bits, KatStream, nal

_OK = (ValueError, RuntimeError, IndexError, OverflowError, MemoryError)
# 2^32 - 1 -> int -1 (and "+ 1" -> 0); 2^31 -> INT_MIN; 2^33 - 2: the largest 32-leading-zero code
_WRAPS = [(1 << 32) - 1, 1 << 31, (1 << 33) - 2]


def _content(w, h, seed):
    r = np.random.default_rng(seed)
    return r.integers(0, 256, (h, w)), r.integers(0, 256, (h // 2, w // 2)), r.integers(0, 256, (h // 2, w // 2))


def _kat_streams():
    a = KatStream(32, 32, weighted=True)
    a.idr_pcm(*_content(32, 32, 1))
    a.p_picture(1, [0], [{"mvd": (3, -2)}] + [{"skip": True}] * 3,
                wp={"denom": 5, "w": 40, "o": -7, "cdenom_delta": 1, "cw": [(70, 3), (50, -20)]})
    b = KatStream(32, 32, sps_st_rps=1)
    b.idr_pcm(*_content(32, 32, 2))
    b.p_picture(1, [0], [{"skip": True}] * 4)
    b.p_picture(2, [1, 0], [{"skip": True}] * 4, tmvp=True, nref=2, inter_rps=True)
    return a, b


def _hevc_decode(host, data):
    return host.hevc_decode_full(data, True, False)


def test_kat_streams_decode_unmodified(host):
    for s in _kat_streams():
        pics = _hevc_decode(host, s.bytes())
        assert len(pics) == len([u for u in s.units if u[0] in (1, 19)])


@pytest.mark.parametrize("value", _WRAPS)
def test_every_hevc_exp_golomb_site_rejects_wrapping_codes(host, value):
    """All ue(v) / se(v) sites of VPS / SPS / PPS / slice headers, including
    delta_idx_minus1, collocated_ref_idx and luma_log2_weight_denom."""
    n = 0
    for s in _kat_streams():
        for unit, site in s.ue_sites():
            data = s.with_ue(unit, site, value)
            try:
                _hevc_decode(host, data)
            except _OK:
                n += 1
    assert n > 60  # nearly every site must fail cleanly; a few (VPS, VUI-like skips) are ignored


def _kat_with_site(s, unit_type, k, value):
    """Replace the k-th Exp-Golomb code of the last unit of ``unit_type``."""
    unit = max(i for i, (t, _) in enumerate(s.units) if t == unit_type)
    return s.with_ue(unit, k, value)


def _expect(host, data, what):
    with pytest.raises(_OK) as e:
        _hevc_decode(host, data)
    assert what in str(e.value), str(e.value)


def test_hevc_delta_idx_minus1_wrap(host):
    _, b = _kat_streams()
    # slice header of the third picture: slice_pic_parameter_set_id, slice_type, delta_idx_minus1, ...
    _expect(host, _kat_with_site(b, 1, 2, (1 << 32) - 1), "delta_idx_minus1")


def test_hevc_collocated_ref_idx_wrap(host):
    _, b = _kat_streams()
    # ..., abs_delta_rps_minus1 (3), num_ref_idx_l0_active_minus1 (4), collocated_ref_idx (5)
    _expect(host, _kat_with_site(b, 1, 5, (1 << 32) - 1), "collocated_ref_idx")


def test_hevc_log2_weight_denom_wrap(host):
    a, _ = _kat_streams()
    # P slice header: pps id, slice_type, num_negative, num_positive, delta_poc_s0, denom (5)
    _expect(host, _kat_with_site(a, 1, 5, (1 << 32) - 1), "luma_log2_weight_denom")


def _hevc_pps(tile_cols_minus1: int, tile_rows_minus1: int, widths: list[int]) -> bytes:
    """The KatStream PPS with tiles on (non-uniform spacing)."""
    b = Bits()
    b.ue(0)
    b.ue(0)
    b.u(0, 7)          # dependent slices, output flag, extra bits, sign hiding, cabac_init_present
    b.ue(0)
    b.ue(0)
    b.se(0)
    b.u(0, 3)          # constrained intra, transform skip, cu_qp_delta
    b.se(0)
    b.se(0)
    b.u(0, 4)          # slice chroma offsets, weighted, weighted bipred, transquant bypass
    b.u(1, 1)          # tiles_enabled_flag
    b.u(0, 1)          # WPP
    b.ue(tile_cols_minus1)
    b.ue(tile_rows_minus1)
    b.u(0, 1)          # uniform_spacing_flag 0
    for wd in widths:
        b.ue(wd)
    b.u(1, 1)          # loop_filter_across_tiles
    b.u(0, 1)
    b.u(0, 1)          # deblocking control
    b.u(0, 1)
    b.u(0, 1)
    b.ue(0)
    b.u(0, 2)
    b.trailing()
    return nal(34, b.bytes())


def test_hevc_tile_columns_wrap_rejected(host):
    """num_tile_columns_minus1 = 2^32 - 1 used to become 0 columns and write cw[-1]."""
    a = KatStream(32, 32)
    a.idr_pcm(*_content(32, 32, 3))
    data = a.bytes()
    idr = data.index(b"\x00\x00\x00\x01\x26")
    bad = data[:idr] + _hevc_pps((1 << 32) - 1, 0, []) + data[idr:]
    _expect(host, bad, "num_tile_columns_minus1")


# ----------------------------------------------------------------------------- H.264
def _h264_nal(ref_idc: int, ntype: int, rbsp: bytes) -> bytes:
    out = bytearray(b"\x00\x00\x00\x01")
    out.append((ref_idc << 5) | ntype)
    zeros = 0
    for x in rbsp:
        if zeros >= 2 and x <= 3:
            out.append(3)
            zeros = 0
        out.append(x)
        zeros = zeros + 1 if x == 0 else 0
    return bytes(out)


def _h264_units():
    """Baseline SPS / PPS / IDR slice header of a 32x32 picture, the I slice coded as two
    I_PCM macroblocks... kept to the header: the range checks fire before any MB data."""
    sps = Bits()
    sps.u(66, 8)
    sps.u(0xC0, 8)
    sps.u(30, 8)
    sps.ue(0)      # sps id
    sps.ue(0)      # log2_max_frame_num_minus4
    sps.ue(0)      # poc type 0
    sps.ue(0)      # log2_max_poc_lsb_minus4
    sps.ue(1)      # max_num_ref_frames
    sps.u(0, 1)
    sps.ue(1)      # width 2 MBs
    sps.ue(1)      # height 2 MBs
    sps.u(1, 1)    # frame_mbs_only
    sps.u(1, 1)
    sps.u(0, 1)    # cropping
    sps.u(0, 1)    # vui
    sps.trailing()
    pps = Bits()
    pps.ue(0)
    pps.ue(0)
    pps.u(0, 2)
    pps.ue(0)      # slice groups
    pps.ue(0)
    pps.ue(0)
    pps.u(0, 3)
    pps.se(0)
    pps.se(0)
    pps.se(0)
    pps.u(1, 1)    # deblocking control present
    pps.u(0, 2)
    pps.trailing()
    sl = Bits()
    sl.ue(0)       # first_mb
    sl.ue(7)       # I
    sl.ue(0)       # pps id
    sl.u(0, 4)     # frame_num
    sl.ue(0)       # idr_pic_id
    sl.u(0, 4)     # poc lsb
    sl.u(0, 2)     # no_output_of_prior_pics, long_term_reference
    sl.se(0)       # slice_qp_delta
    sl.ue(1)       # disable_deblocking_filter_idc
    # mb_type I_PCM (25) for both... four MBs, each PCM
    for _ in range(4):
        sl.ue(25)
        sl.align_zero()
        sl.u(0, 8 * 384)
    sl.trailing()
    return [(3, 7, sps), (3, 8, pps), (3, 5, sl)]


def _h264_bytes(units, unit=None, site=None, value=None):
    out = bytearray()
    for k, (ri, t, b) in enumerate(units):
        out += _h264_nal(ri, t, (b.with_ue(site, value) if k == unit else b).bytes())
    return bytes(out)


def test_h264_units_decode_unmodified(host):
    frames = host.decode(_h264_bytes(_h264_units()))
    assert len(frames) == 1


@pytest.mark.parametrize("value", _WRAPS)
def test_every_h264_header_exp_golomb_site_rejects_wrapping_codes(host, value):
    units = _h264_units()
    for unit, (_, _, b) in enumerate(units):
        for site in range(len(b.ue_sites)):
            data = _h264_bytes(units, unit, site, value)
            for fn in (host.decode, host.stream_info, lambda d: host.parse([d], 1)):
                try:
                    fn(data)
                except _OK:
                    pass


def test_h264_pps_id_wrap_rejected(host):
    """pic_parameter_set_id in a slice header indexed the PPS table unchecked."""
    units = _h264_units()
    with pytest.raises(_OK) as e:
        host.decode(_h264_bytes(units, 2, 2, (1 << 32) - 1))
    assert "pic_parameter_set_id" in str(e.value)
