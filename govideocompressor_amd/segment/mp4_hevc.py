"""HEVC (``hvc1`` + ``hvcC``) MP4 mux / demux for encoded pieces.

The reference stores every piece as ``<idx>.mp4`` whatever ``-vcodec`` the operator
passes (client.go:54, 101-130 -- ``-c:v libx265`` pieces included), and merges them
with ``ffmpeg -f concat -c copy`` (server.go:349-361).  The native muxer in
``csrc/host/annexb.cc`` writes ``avc1`` tracks; this module is its HEVC sibling
(ISO/IEC 14496-15 §8.3: ``HEVCDecoderConfigurationRecord`` with the VPS/SPS/PPS
arrays, 4-byte NAL length prefixes in ``mdat``).  Container-only work on host
bytes, so it is plain Python: a piece is a few MB and this runs once per piece.

The encoder's HEVC streams are IDR + P in output order (no reordering), so decode
time == composition time and no ``ctts`` box is needed.
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
    br.ue()
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
    return dict(ptl=ptl, max_sub_layers=max_sub + 1, temporal_nesting=nesting, chroma_format_idc=chroma,
                width=w, height=h, bit_depth_luma=bdl + 8, bit_depth_chroma=bdc + 8)


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


def mux(stream: bytes, fps: float = 30.0) -> bytes:
    """Annex-B HEVC -> MP4 bytes (one ``hvc1`` track, one chunk, ``mdat`` after ``moov``)."""
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
    n = len(samples)
    media_dur, movie_dur = n * delta, int(round(n * 1000.0 / fps))
    v1 = media_dur > 0xFFFFFFFF or movie_dur > 0xFFFFFFFF  # 64-bit durations (version 1 boxes)
    mdat_body = b"".join(bytes(s) for s in samples)

    ftyp = _box(b"ftyp", b"isom", struct.pack(">I", 512), b"isomiso2hvc1mp41")
    entry = _box(b"hvc1", bytes(6), struct.pack(">H", 1), bytes(16), struct.pack(">HHII", w, h, 0x480000, 0x480000),
                 struct.pack(">IH", 0, 1), bytes(32), struct.pack(">Hh", 0x18, -1),
                 _box(b"hvcC", hvcc_record(vps, sps, pps)))

    def moov(offset: int) -> bytes:
        wide = offset + len(mdat_body) + 16 > 0xFFFFFFFF
        stco = (_full(b"co64", 0, 0, struct.pack(">IQ", 1, offset)) if wide
                else _full(b"stco", 0, 0, struct.pack(">II", 1, offset)))
        stbl = _box(b"stbl",
                    _full(b"stsd", 0, 0, struct.pack(">I", 1), entry),
                    _full(b"stts", 0, 0, struct.pack(">III", 1, n, delta)),
                    _full(b"stss", 0, 0, struct.pack(">I", len(sync)), *(struct.pack(">I", s) for s in sync)),
                    _full(b"stsc", 0, 0, struct.pack(">IIII", 1, 1, n, 1)),
                    _full(b"stsz", 0, 0, struct.pack(">II", 0, n), *(struct.pack(">I", len(s)) for s in samples)),
                    stco)
        minf = _box(b"minf", _full(b"vmhd", 0, 1, bytes(8)),
                    _box(b"dinf", _full(b"dref", 0, 0, struct.pack(">I", 1), _full(b"url ", 0, 1))), stbl)
        if v1:
            mdhd = _full(b"mdhd", 1, 0, struct.pack(">QQIQHH", 0, 0, timescale, media_dur, 0x55C4, 0))
            tkhd = _full(b"tkhd", 1, 3, struct.pack(">QQIIQ", 0, 0, 1, 0, movie_dur), bytes(8),
                         struct.pack(">hhhH", 0, 0, 0, 0), _MATRIX, struct.pack(">II", w << 16, h << 16))
            mvhd = _full(b"mvhd", 1, 0, struct.pack(">QQIQ", 0, 0, 1000, movie_dur), struct.pack(">IH", 0x10000, 0x100),
                         bytes(10), _MATRIX, bytes(24), struct.pack(">I", 2))
        else:
            mdhd = _full(b"mdhd", 0, 0, struct.pack(">IIIIHH", 0, 0, timescale, media_dur, 0x55C4, 0))
            tkhd = _full(b"tkhd", 0, 3, struct.pack(">IIIII", 0, 0, 1, 0, movie_dur), bytes(8),
                         struct.pack(">hhhH", 0, 0, 0, 0), _MATRIX, struct.pack(">II", w << 16, h << 16))
            mvhd = _full(b"mvhd", 0, 0, struct.pack(">IIII", 0, 0, 1000, movie_dur), struct.pack(">IH", 0x10000, 0x100),
                         bytes(10), _MATRIX, bytes(24), struct.pack(">I", 2))
        mdia = _box(b"mdia", mdhd,
                    _full(b"hdlr", 0, 0, struct.pack(">I", 0), b"vide", bytes(12), b"VideoHandler\x00"), minf)
        return _box(b"moov", mvhd, _box(b"trak", tkhd, mdia))

    size = len(moov(0))
    wide = len(ftyp) + size + 16 + len(mdat_body) > 0xFFFFFFFF
    hdr = struct.pack(">I", 1) + b"mdat" + struct.pack(">Q", 16 + len(mdat_body)) if wide else \
        struct.pack(">I", 8 + len(mdat_body)) + b"mdat"
    m = moov(len(ftyp) + size + len(hdr))
    if len(m) != size:  # stco -> co64 switch changed the size; recompute once
        m = moov(len(ftyp) + len(m) + len(hdr))
    return ftyp + m + hdr + mdat_body


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
    try:
        s, e = _find(data, 0, len(data), [b"moov", b"trak", b"mdia", b"minf", b"stbl", b"stsd"])
    except ValueError:
        return False
    return data[s + 12:s + 16] in (b"hvc1", b"hev1")


def track_fps(data: bytes) -> float | None:
    """Frame rate of an MP4's (first) track: mdhd timescale / the first stts delta."""
    try:
        ms, me = _find(data, 0, len(data), [b"moov", b"trak", b"mdia", b"mdhd"])
        ver = data[ms]
        timescale = struct.unpack(">I", data[ms + (20 if ver == 1 else 12):ms + (24 if ver == 1 else 16)])[0]
        ts, te = _find(data, 0, len(data), [b"moov", b"trak", b"mdia", b"minf", b"stbl", b"stts"])
        n = struct.unpack(">I", data[ts + 4:ts + 8])[0]
        if n < 1 or timescale <= 0:
            return None
        delta = struct.unpack(">I", data[ts + 12:ts + 16])[0]
        return timescale / delta if delta > 0 else None
    except (ValueError, struct.error, IndexError):
        return None


def demux(data: bytes) -> bytes:
    """``hvc1`` MP4 -> Annex-B (parameter sets from ``hvcC`` first, then every sample)."""
    s, e = _find(data, 0, len(data), [b"moov", b"trak", b"mdia", b"minf", b"stbl"])
    stbl = {k: (a, b_) for k, a, b_ in _children(data, s, e)}
    ss, _ = stbl[b"stsd"]
    ent = ss + 8
    _, esz_kind = struct.unpack(">I4s", data[ent:ent + 8])
    if esz_kind not in (b"hvc1", b"hev1"):
        raise ValueError("mp4: not an HEVC track")
    esz = struct.unpack(">I", data[ent:ent + 4])[0]
    hs, he = _find(data, ent + 8 + 78, ent + esz, [b"hvcC"])
    rec = data[hs:he]
    nls = (rec[21] & 3) + 1
    out = bytearray()
    p = 23
    for _ in range(rec[22]):
        cnt = struct.unpack(">H", rec[p + 1:p + 3])[0]
        p += 3
        for _ in range(cnt):
            ln = struct.unpack(">H", rec[p:p + 2])[0]
            out += b"\x00\x00\x00\x01" + rec[p + 2:p + 2 + ln]
            p += 2 + ln
    zs, _ = stbl[b"stsz"]
    fixed, n = struct.unpack(">II", data[zs + 4:zs + 12])
    sizes = [fixed] * n if fixed else list(struct.unpack(f">{n}I", data[zs + 12:zs + 12 + 4 * n]))
    if b"co64" in stbl:
        cs, _ = stbl[b"co64"]
        nc = struct.unpack(">I", data[cs + 4:cs + 8])[0]
        offs = list(struct.unpack(f">{nc}Q", data[cs + 8:cs + 8 + 8 * nc]))
    else:
        cs, _ = stbl[b"stco"]
        nc = struct.unpack(">I", data[cs + 4:cs + 8])[0]
        offs = list(struct.unpack(f">{nc}I", data[cs + 8:cs + 8 + 4 * nc]))
    sc, _ = stbl[b"stsc"]
    ne = struct.unpack(">I", data[sc + 4:sc + 8])[0]
    runs = [struct.unpack(">III", data[sc + 8 + 12 * i:sc + 20 + 12 * i]) for i in range(ne)]
    k = 0
    for ci, off in enumerate(offs):
        per = [r[1] for r in runs if r[0] <= ci + 1][-1]
        for _ in range(per):
            if k >= n:
                break
            q, end = off, off + sizes[k]
            while q < end:
                ln = int.from_bytes(data[q:q + nls], "big")
                out += b"\x00\x00\x00\x01" + data[q + nls:q + nls + ln]
                q += nls + ln
            off = end
            k += 1
    return bytes(out)
