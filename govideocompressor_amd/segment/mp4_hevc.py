"""HEVC (``hvc1`` + ``hvcC``) MP4 mux / demux for encoded pieces.

The reference stores every piece as ``<idx>.mp4`` whatever ``-vcodec`` the operator
passes (client.go:54, 101-130 -- ``-c:v libx265`` pieces included), and merges them
with ``ffmpeg -f concat -c copy`` (server.go:349-361).  The native muxer in
``csrc/host/annexb.cc`` writes ``avc1`` tracks; this module is its HEVC sibling
(ISO/IEC 14496-15 §8.3: ``HEVCDecoderConfigurationRecord`` with the VPS/SPS/PPS
arrays, 4-byte NAL length prefixes in ``mdat``).  Container-only work on host
bytes, so it is plain Python: a piece is a few MB and this runs once per piece.

B pictures (the encoder's default GOP codes one B between anchors, x265 --bframes) are
stored in decode order, so the track carries composition offsets (``ctts``) and an edit
list from the pictures' PicOrderCnt (8.3.1, parsed here from the slice headers) like the
``avc1`` track of segment/mp4.py.
"""
from __future__ import annotations

import struct

_VPS, _SPS, _PPS, _AUD = 32, 33, 34, 35
# NAL types that belong to the picture they follow: end of sequence / bitstream, filler
# data, suffix SEI (Table 7-1)
_SUFFIX = (36, 37, 38, 40)


def is_hevc_annexb(data: bytes) -> bool:
    """True when the first NAL of an Annex-B stream carries an HEVC VPS/SPS/AUD/slice header
    (H.264 NAL headers are one byte with forbidden_zero_bit=0 and type 7/9 at the front)."""
    nals = split_nals(data[:256])
    if not nals:
        return False
    h = nals[0]
    # forbidden_zero_bit = 0, nuh_layer_id = 0, nuh_temporal_id_plus1 >= 1
    return (len(h) >= 2 and h[0] & 0x81 == 0 and h[1] >> 3 == 0 and (h[1] & 0x7) >= 1
            and (h[0] >> 1) & 0x3F in (_VPS, _SPS, _PPS, _AUD))


def split_nals(data: bytes) -> list[bytes]:
    """Annex-B -> NAL payloads (start codes and trailing zero bytes stripped)."""
    out, n, i, start = [], len(data), 0, -1
    while i + 2 < n:
        if data[i] == 0 and data[i + 1] == 0 and data[i + 2] == 1:
            if start >= 0:
                out.append(data[start:i].rstrip(b"\x00"))
            start = i + 3
            i += 3
        else:
            i += 1
    if start >= 0 and start < n:
        out.append(data[start:].rstrip(b"\x00"))
    return [x for x in out if x]


def _rbsp(nal: bytes) -> bytes:
    return nal.replace(b"\x00\x00\x03", b"\x00\x00")


class _Bits:
    def __init__(self, b: bytes):
        self.b, self.p = b, 0

    def u(self, n: int) -> int:
        v = 0
        for _ in range(n):
            v = (v << 1) | ((self.b[self.p >> 3] >> (7 - (self.p & 7))) & 1)
            self.p += 1
        return v

    def ue(self) -> int:
        z = 0
        while self.u(1) == 0:
            z += 1
        return (1 << z) - 1 + self.u(z)


def parse_sps(sps_nal: bytes) -> dict:
    """Fields of an HEVC SPS the ``hvcC`` record and the track header need."""
    r = _rbsp(sps_nal)
    br = _Bits(r[2:])
    br.u(4)
    max_sub = br.u(3)
    nesting = br.u(1)
    ptl = r[3:15]  # general_profile_space .. general_level_idc (12 bytes, byte aligned)
    br.p += 96
    sub_prof, sub_lvl = [], []
    for _ in range(max_sub):
        sub_prof.append(br.u(1))
        sub_lvl.append(br.u(1))
    if max_sub > 0:
        br.p += 2 * (8 - max_sub)
    for i in range(max_sub):
        br.p += 88 * sub_prof[i] + 8 * sub_lvl[i]
    sps_id = br.ue()
    chroma = br.ue()
    if chroma == 3:
        br.u(1)
    w, h = br.ue(), br.ue()
    sw, sh = (2, 2) if chroma == 1 else ((2, 1) if chroma == 2 else (1, 1))
    if br.u(1):
        left, right, top, bottom = br.ue(), br.ue(), br.ue(), br.ue()
        w -= sw * (left + right)
        h -= sh * (top + bottom)
    bdl, bdc = br.ue(), br.ue()
    log2_poc = br.ue() + 4
    return dict(ptl=ptl, max_sub_layers=max_sub + 1, temporal_nesting=nesting, chroma_format_idc=chroma,
                width=w, height=h, bit_depth_luma=bdl + 8, bit_depth_chroma=bdc + 8, sps_id=sps_id,
                log2_max_poc_lsb=log2_poc)


def display_order(stream: bytes) -> list[int]:
    """Display index of every picture of an Annex-B HEVC stream, in decode order: PicOrderCnt
    (8.3.1: slice_pic_order_cnt_lsb plus the MSB carried from the previous TemporalId-0
    reference picture) ranked within each coded video sequence (an IDR / BLA, or a CRA that
    starts the stream), sequences following each other."""
    sps_lsb: dict[int, int] = {}
    pps: dict[int, tuple[int, int, int]] = {}   # id -> (sps id, output_flag_present, extra bits)
    pocs: list[tuple[int, int]] = []            # (cvs ordinal, POC) per picture, decode order
    cvs, prev_lsb, prev_msb, first = -1, 0, 0, True
    for nal in split_nals(stream):
        t = (nal[0] >> 1) & 0x3F
        if t == _SPS:
            info = parse_sps(nal)
            sps_lsb[info["sps_id"]] = info["log2_max_poc_lsb"]
            continue
        if t == _PPS:
            br = _Bits(_rbsp(nal)[2:])
            pid, sid = br.ue(), br.ue()
            br.u(1)
            pps[pid] = (sid, br.u(1), br.u(3))
            continue
        if t >= 32 or len(nal) < 3 or not nal[2] & 0x80:
            continue  # non-VCL, or not the first slice segment of a picture
        br = _Bits(_rbsp(nal)[2:])
        br.u(1)
        if 16 <= t <= 23:
            br.u(1)
        sid, out_flag, extra = pps[br.ue()]
        br.u(extra)
        br.ue()   # slice_type
        if out_flag:
            br.u(1)
        log2 = sps_lsb[sid]
        irap_reset = t in (16, 17, 18, 19, 20) or (t == 21 and first)
        if t in (19, 20):       # IDR: PicOrderCnt 0
            lsb = 0
        else:
            lsb = br.u(log2)
        if irap_reset:
            msb = 0
            cvs += 1
        else:
            half = 1 << (log2 - 1)
            if lsb < prev_lsb and prev_lsb - lsb >= half:
                msb = prev_msb + (1 << log2)
            elif lsb > prev_lsb and lsb - prev_lsb > half:
                msb = prev_msb - (1 << log2)
            else:
                msb = prev_msb
        first = False
        tid = (nal[1] & 7) - 1
        if tid == 0 and not (t <= 14 and t % 2 == 0) and t not in (6, 7, 8, 9):  # not SLNR / RADL / RASL
            prev_lsb, prev_msb = lsb, msb
        pocs.append((cvs, msb + lsb))
    ranks = sorted(range(len(pocs)), key=lambda i: pocs[i])
    out = [0] * len(pocs)
    for r, i in enumerate(ranks):
        out[i] = r
    return out


def _box(kind: bytes, *payload: bytes) -> bytes:
    body = b"".join(payload)
    return struct.pack(">I", 8 + len(body)) + kind + body


def _full(kind: bytes, version: int, flags: int, *payload: bytes) -> bytes:
    return _box(kind, struct.pack(">I", (version << 24) | flags), *payload)


_MATRIX = struct.pack(">9I", 0x10000, 0, 0, 0, 0x10000, 0, 0, 0, 0x40000000)


def hvcc_record(vps: list[bytes], sps: list[bytes], pps: list[bytes]) -> bytes:
    s = parse_sps(sps[0])
    rec = bytes([1]) + s["ptl"][:11] + bytes([s["ptl"][11]])
    rec += struct.pack(">HBBBBH", 0xF000, 0xFC, 0xFC | s["chroma_format_idc"], 0xF8 | (s["bit_depth_luma"] - 8),
                       0xF8 | (s["bit_depth_chroma"] - 8), 0)
    rec += bytes([(s["max_sub_layers"] << 3) | (s["temporal_nesting"] << 2) | 3])
    arrays = [(t, xs) for t, xs in ((_VPS, vps), (_SPS, sps), (_PPS, pps)) if xs]
    rec += bytes([len(arrays)])
    for t, xs in arrays:
        rec += bytes([0x80 | t]) + struct.pack(">H", len(xs))
        for x in xs:
            rec += struct.pack(">H", len(x)) + x
    return rec


def hevc_track(stream: bytes, fps: float | None = 30.0):
    """Annex-B HEVC -> one ``hvc1`` :class:`~.mp4.Track` (parameter sets in ``hvcC``)."""
    from . import mp4
    vps, sps, pps = [], [], []
    samples: list[bytearray] = []
    sync: list[int] = []
    pending = bytearray()
    for nal in split_nals(stream):
        t = (nal[0] >> 1) & 0x3F
        if t in (_VPS, _SPS, _PPS):
            lst = {_VPS: vps, _SPS: sps, _PPS: pps}[t]
            if nal not in lst:
                lst.append(nal)
            continue
        if t == _AUD:
            continue
        rec = struct.pack(">I", len(nal)) + nal
        if t < 32:  # VCL
            if len(nal) > 2 and nal[2] & 0x80:  # first_slice_segment_in_pic_flag
                samples.append(bytearray(pending))
                if 16 <= t <= 21:
                    sync.append(len(samples))
                pending = bytearray()
            elif not samples:
                raise ValueError("hevc mp4 mux: a slice segment precedes the first picture start")
            samples[-1] += rec
        elif t in _SUFFIX and samples:
            samples[-1] += rec  # suffix SEI / EOS / EOB / filler: the current picture's
        else:
            pending += rec  # prefix SEI etc. belong to the next picture
    if not samples or not sps or not pps:
        raise ValueError("hevc mp4 mux: stream has no pictures or no SPS/PPS")
    if pending:
        samples[-1] += pending  # trailing non-VCL NALs stay with the last picture
    info = parse_sps(sps[0])
    w, h = info["width"], info["height"]
    fps = fps if fps and fps > 0 else 30.0
    timescale, delta = int(round(fps * 1000)), 1000
    entry = mp4._visual_entry(b"hvc1", w, h, _box(b"hvcC", hvcc_record(vps, sps, pps)))
    marks = set(sync)
    disp = display_order(stream)
    if len(disp) != len(samples):
        raise ValueError("hevc mp4 mux: picture count and slice headers disagree")
    cts, media_time = mp4.reorder_offsets(disp, delta)
    return mp4.Track(b"vide", timescale, entry, [bytes(x) for x in samples], [delta] * len(samples),
                     cts if media_time else None, [(i + 1) in marks for i in range(len(samples))], w, h, media_time)


def mux(stream: bytes, fps: float = 30.0) -> bytes:
    """Annex-B HEVC -> MP4 bytes (one ``hvc1`` track; P-only GOPs need no ``ctts``)."""
    from . import mp4
    return mp4.write([hevc_track(stream, fps)])


def _children(b: bytes, start: int, end: int):
    i = start
    while i + 8 <= end:
        size, kind = struct.unpack(">I4s", b[i:i + 8])
        hdr = 8
        if size == 1:
            size, hdr = struct.unpack(">Q", b[i + 8:i + 16])[0], 16
        elif size == 0:
            size = end - i
        yield kind, i + hdr, i + size
        i += size


def _find(b: bytes, start: int, end: int, path: list[bytes]):
    for kind, s, e in _children(b, start, end):
        if kind == path[0]:
            return (s, e) if len(path) == 1 else _find(b, s, e, path[1:])
    raise ValueError(f"mp4: box {b'/'.join(path).decode()} not found")


def is_hevc_mp4(data: bytes) -> bool:
    from . import mp4
    try:
        return mp4.video_track(mp4.read(data)).codec in (b"hvc1", b"hev1")
    except (ValueError, struct.error, IndexError):
        return False


def track_fps(data: bytes) -> float | None:
    """Frame rate of an MP4's video track: timescale / its (median) sample duration."""
    from . import mp4
    try:
        return mp4.track_fps(mp4.video_track(mp4.read(data))) or None
    except (ValueError, struct.error, IndexError):
        return None


def demux(data: bytes) -> bytes:
    """``hvc1`` MP4 -> Annex-B (parameter sets from ``hvcC`` first, then every sample)."""
    from . import mp4
    t = mp4.video_track(mp4.read(data))
    if t.codec not in (b"hvc1", b"hev1"):
        raise ValueError("mp4: not an HEVC track")
    return mp4.video_to_annexb(t)
