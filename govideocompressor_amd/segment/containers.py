"""MPEG-TS and Matroska/WebM demuxers: the other containers the reference's splitter reads.

The reference probes and splits whatever ``ffmpeg -i`` opens (server.go:199-201, 241):
besides MP4 that is typically MPEG-TS (broadcast, HLS, camera ``.m2ts``) and Matroska.
Here both are demuxed natively into

* the video elementary stream as Annex-B (H.264 ``0x1B`` / ``V_MPEG4/ISO/AVC``, HEVC
  ``0x24`` / ``V_MPEGH/ISO/HEVC``; Matroska's length-prefixed NAL units are rewritten with
  start codes and the CodecPrivate parameter sets in front), which the native splitter then
  cuts at keyframes;
* the presentation time of every video access unit (decode order), so pieces cut the
  audio at the same instants;
* AAC audio as an ISO-BMFF ``mp4a`` track (ADTS frames in TS, ``A_AAC`` in Matroska), which
  the pieces carry like the MP4 path's ``-acodec copy``.  Other audio codecs are dropped
  (listed in ``Demuxed.dropped``) -- the pieces are written as MP4.

Both parsers bound every length field by its parent, so truncated or corrupt files raise
``ValueError`` instead of reading past the data.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

from . import mp4

AAC_RATES = (96000, 88200, 64000, 48000, 44100, 32000, 24000, 22050, 16000, 12000, 11025, 8000, 7350)


@dataclass
class Demuxed:
    codec: str                                   # "h264" | "hevc"
    annexb: bytes
    pts: list[float] = field(default_factory=list)   # seconds per access unit (decode order), from 0
    audio: list[mp4.Track] = field(default_factory=list)
    dropped: list[str] = field(default_factory=list)
    width: int = 0
    height: int = 0


# ------------------------------------------------------------------------------- AAC
def _esds(asc: bytes, avg_bitrate: int = 0) -> bytes:
    """ES_Descriptor with a DecoderConfigDescriptor (AAC, objectTypeIndication 0x40)."""
    def desc(tag: int, body: bytes) -> bytes:
        n = len(body)
        return bytes([tag, 0x80 | ((n >> 21) & 0x7F), 0x80 | ((n >> 14) & 0x7F), 0x80 | ((n >> 7) & 0x7F), n & 0x7F]) + body
    dsi = desc(0x05, asc)
    dcd = desc(0x04, bytes([0x40, 0x15]) + (0).to_bytes(3, "big") + struct.pack(">II", avg_bitrate, avg_bitrate) + dsi)
    sl = desc(0x06, b"\x02")
    return mp4._full(b"esds", 0, 0, desc(0x03, struct.pack(">HB", 1, 0) + dcd + sl))


def aac_track(asc: bytes, rate: int, channels: int, frames: list[bytes], pts0: float = 0.0) -> mp4.Track:
    """Raw AAC frames (1024 samples each) -> an ``mp4a`` track.  ``pts0``: the first frame's
    time relative to the video's first picture, in seconds.  Negative: the frames before the
    picture are dropped; positive: the track starts that much later (an empty edit, mp4.Track
    negative ``media_time``), so the audio stays in sync."""
    entry = mp4._box(b"mp4a", bytes(6), struct.pack(">H", 1), bytes(8), struct.pack(">HHHH", channels, 16, 0, 0),
                     struct.pack(">I", rate << 16), _esds(asc))
    skip = int(round(-pts0 * rate / 1024.0)) if pts0 < 0 else 0
    frames = frames[skip:]
    delay = int(round(pts0 * rate)) if pts0 > 0.5 / rate else 0
    return mp4.Track(b"soun", rate, entry, list(frames), [1024] * len(frames), media_time=-delay)


def asc_of(profile: int, rate_idx: int, channels: int) -> bytes:
    """AudioSpecificConfig: audioObjectType (5 bits), samplingFrequencyIndex, channelConfiguration."""
    v = ((profile + 1) << 11) | (rate_idx << 7) | (channels << 3)
    return struct.pack(">H", v)


def adts_frames(data: bytes) -> tuple[bytes, int, int, list[bytes]]:
    """ADTS stream -> (AudioSpecificConfig, sample rate, channels, raw frames)."""
    out, i, cfg = [], 0, None
    n = len(data)
    while i + 7 <= n:
        if data[i] != 0xFF or (data[i + 1] & 0xF6) != 0xF0:
            i += 1  # resynchronise
            continue
        prot_absent = data[i + 1] & 1
        profile = data[i + 2] >> 6
        sfi = (data[i + 2] >> 2) & 15
        ch = ((data[i + 2] & 1) << 2) | (data[i + 3] >> 6)
        flen = ((data[i + 3] & 3) << 11) | (data[i + 4] << 3) | (data[i + 5] >> 5)
        hl = 7 if prot_absent else 9
        if flen < hl or i + flen > n or sfi >= len(AAC_RATES):
            break
        if cfg is None:
            cfg = (profile, sfi, ch)
        out.append(bytes(data[i + hl:i + flen]))
        i += flen
    if cfg is None:
        raise ValueError("ADTS: no AAC frame found")
    profile, sfi, ch = cfg
    return asc_of(profile, sfi, ch), AAC_RATES[sfi], ch, out


# ------------------------------------------------------------------------------- MPEG-TS
TS_VIDEO = {0x1B: "h264", 0x24: "hevc"}
TS_AAC = 0x0F


def is_ts(head: bytes) -> bool:
    return len(head) >= 189 and head[0] == 0x47 and head[188] == 0x47


def _pes_payload(pes: bytes) -> tuple[bytes, int | None]:
    """PES packet -> (payload, 33-bit PTS in 90 kHz ticks or None)."""
    if len(pes) < 9 or pes[:3] != b"\x00\x00\x01":
        raise ValueError("TS: PES without a start code prefix")
    sid = pes[3]
    if sid in (0xBC, 0xBE, 0xBF, 0xF0, 0xF1, 0xF2, 0xF8, 0xFF):  # no optional header
        return pes[6:], None
    flags, hlen = pes[7], pes[8]
    if 9 + hlen > len(pes):
        raise ValueError("TS: PES header overruns the packet")
    pts = None
    if flags & 0x80 and hlen >= 5:
        b = pes[9:14]
        pts = ((b[0] >> 1) & 7) << 30 | b[1] << 22 | (b[2] >> 1) << 15 | b[3] << 7 | b[4] >> 1
    return pes[9 + hlen:], pts


PTS_WRAP = 1 << 33


def unwrap_pts(ticks: list[int | None], anchor: int | None = None) -> list[int | None]:
    """33-bit PTS values (one stream, decode order) made continuous across the wrap: each
    value is moved by a multiple of 2^33 to the one nearest the previous value (the first
    one: nearest ``anchor``, e.g. the video's first PTS, so streams stay comparable)."""
    out: list[int | None] = []
    prev = anchor
    for v in ticks:
        if v is None:
            out.append(None)
            continue
        if prev is not None:
            v += PTS_WRAP * round((prev - v) / PTS_WRAP)
        out.append(v)
        prev = v
    return out


def access_units(payload: bytes, codec: str) -> int:
    """Pictures starting in a PES payload: H.264 slices with first_mb_in_slice 0 (the ue(v)
    code '1'), HEVC VCL NAL units with first_slice_segment_in_pic_flag."""
    n, i, end = 0, 0, len(payload)
    while True:
        i = payload.find(b"\x00\x00\x01", i)
        if i < 0 or i + 5 > end:
            return n
        h = payload[i + 3]
        if codec == "h264":
            if (h & 0x1F) in (1, 5) and payload[i + 4] & 0x80:
                n += 1
        elif ((h >> 1) & 0x3F) < 32 and payload[i + 5] & 0x80:
            n += 1
        i += 3


def per_picture_pts(pes: list[tuple[bytes, int | None]], codec: str, display: list[int] | None = None) -> list[float]:
    """One presentation time (seconds, unwrapped 90 kHz ticks / 90000) per picture, decode
    order: a PES's PTS belongs to the first picture starting in it (ISO 13818-1 2.4.3.7);
    pictures without one (later pictures of a multi-picture PES, PES packets without a PTS)
    are placed at the stream's frame interval from the nearest picture with a PTS in DISPLAY
    order -- ``display``: each picture's display index (decode order, from the POCs; None:
    no reordering), since with B pictures the previous picture in decode order is usually a
    later anchor."""
    ticks = unwrap_pts([t for _, t in pes])
    per: list[float | None] = []
    for (pl, _), t in zip(pes, ticks):
        k = access_units(pl, codec)
        if k == 0:
            continue  # parameter sets / SEI / a continuation of the previous picture
        per.append(None if t is None else t / 90000.0)
        per += [None] * (k - 1)
    # frame interval: the median of (time step / picture-count step) between known times
    # (sorted by time: B-picture reordering makes decode-order steps negative)
    known = sorted((x, i) for i, x in enumerate(per) if x is not None)
    steps = [(b - a) / abs(j - i) for (a, i), (b, j) in zip(known, known[1:]) if b > a and j != i]
    dt = sorted(steps)[len(steps) // 2] if steps else 1.0 / 30
    if display is None or len(display) != len(per):
        display = list(range(len(per)))
    known_d = sorted((display[i], x) for i, x in enumerate(per) if x is not None)
    out = []
    for i, x in enumerate(per):
        if x is None:
            d = display[i]
            before = [(kd, kx) for kd, kx in known_d if kd < d]
            after = [(kd, kx) for kd, kx in known_d if kd > d]
            if before:
                x = before[-1][1] + (d - before[-1][0]) * dt
            elif after:
                x = after[0][1] - (after[0][0] - d) * dt
            else:
                x = d * dt
        out.append(x)
    return out


def _display_order(stream: bytes, codec: str) -> list[int] | None:
    """Display index per picture (decode order) from the stream's POCs; None if unparsable."""
    try:
        if codec == "h264":
            from ..ops import native
            return list(native.host().h264_samples(stream)["display"])
        from .mp4_hevc import display_order
        return display_order(stream)
    except Exception:  # noqa: BLE001 -- a damaged stream still demuxes, with decode-order fill
        return None


def ts_demux(data: bytes) -> Demuxed:
    try:
        return _ts_demux(data)
    except (IndexError, struct.error) as e:
        raise ValueError(f"TS: malformed stream ({e})") from None


def _ts_demux(data: bytes) -> Demuxed:
    n = len(data)
    if n < 188 or data[0] != 0x47:
        raise ValueError("TS: not an MPEG transport stream (no 0x47 sync byte)")
    pmt_pids: set[int] = set()
    streams: dict[int, int] = {}            # pid -> stream_type
    buf: dict[int, bytearray] = {}          # pid -> PES being assembled
    pes: dict[int, list[tuple[bytes, float | None]]] = {}
    sections: dict[int, bytearray] = {}

    def flush(pid: int):
        b = buf.pop(pid, None)
        if b:
            pes.setdefault(pid, []).append(_pes_payload(bytes(b)))

    def psi(pid: int, payload: bytes, pusi: bool):
        if pusi:
            if not payload:
                return
            payload = payload[1 + payload[0]:]  # pointer_field
            sections[pid] = bytearray(payload)
        elif pid in sections:
            sections[pid] += payload
        else:
            return
        sec = sections[pid]
        if len(sec) < 3:
            return
        slen = ((sec[1] & 0x0F) << 8) | sec[2]
        if len(sec) < 3 + slen:
            return
        body = bytes(sec[:3 + slen])
        del sections[pid]
        if body[0] == 0x00:  # PAT
            for k in range(8, 3 + slen - 4, 4):
                prog = (body[k] << 8) | body[k + 1]
                p = ((body[k + 2] & 0x1F) << 8) | body[k + 3]
                if prog != 0:
                    pmt_pids.add(p)
        elif body[0] == 0x02:  # PMT
            pil = ((body[10] & 0x0F) << 8) | body[11]
            k = 12 + pil
            while k + 5 <= 3 + slen - 4:
                st, ep = body[k], ((body[k + 1] & 0x1F) << 8) | body[k + 2]
                eil = ((body[k + 3] & 0x0F) << 8) | body[k + 4]
                streams.setdefault(ep, st)
                k += 5 + eil

    for off in range(0, n - n % 188, 188):
        pkt = data[off:off + 188]
        if pkt[0] != 0x47:
            raise ValueError(f"TS: lost sync at byte {off}")
        pusi = bool(pkt[1] & 0x40)
        pid = ((pkt[1] & 0x1F) << 8) | pkt[2]
        afc = (pkt[3] >> 4) & 3
        p = 4
        if afc & 2:
            p += 1 + pkt[4]
        if not afc & 1 or p > 188:
            continue
        payload = pkt[p:]
        if pid == 0 or pid in pmt_pids:
            psi(pid, payload, pusi)
            continue
        if pid not in streams:
            continue
        if pusi:
            flush(pid)
            buf[pid] = bytearray(payload)
        elif pid in buf:
            buf[pid] += payload
    for pid in list(buf):
        flush(pid)

    vpids = [p for p, st in streams.items() if st in TS_VIDEO]
    if not vpids:
        raise ValueError("TS: no H.264 / HEVC video stream")
    vp = sorted(vpids)[0]
    vpes = pes.get(vp, [])
    codec = TS_VIDEO[streams[vp]]
    out = Demuxed(codec, b"".join(pl for pl, _ in vpes))
    first_tick = next((t for _, t in vpes if t is not None), None)
    pics = per_picture_pts(vpes, codec, _display_order(out.annexb, codec))
    t0 = min(pics) if pics else 0.0
    out.pts = [t - t0 for t in pics]
    for pid, st in sorted(streams.items()):
        if pid == vp or st in TS_VIDEO:
            continue
        if st != TS_AAC:
            out.dropped.append(f"TS stream type {st:#04x} (pid {pid})")
            continue
        apes = pes.get(pid, [])
        if not apes:
            continue
        asc, rate, ch, frames = adts_frames(b"".join(pl for pl, _ in apes))
        at = unwrap_pts([next((t for _, t in apes if t is not None), None)], first_tick)[0]
        apts = at / 90000.0 if at is not None else t0
        out.audio.append(aac_track(asc, rate, ch, frames, apts - t0))
    return out


# ------------------------------------------------------------------------------- Matroska
EBML_ID = 0x1A45DFA3
MKV_SEGMENT, MKV_INFO, MKV_TRACKS, MKV_CLUSTER = 0x18538067, 0x1549A966, 0x1654AE6B, 0x1F43B675
MKV_VIDEO = {"V_MPEG4/ISO/AVC": "h264", "V_MPEGH/ISO/HEVC": "hevc"}


def is_mkv(head: bytes) -> bool:
    return head[:4] == b"\x1a\x45\xdf\xa3"


def _vint(b: bytes, i: int, end: int, keep_marker: bool) -> tuple[int, int]:
    if i >= end:
        raise ValueError("MKV: element header past its parent")
    first = b[i]
    if first == 0:
        raise ValueError("MKV: invalid variable-length integer")
    ln = 1
    while not first & (0x80 >> (ln - 1)):
        ln += 1
    if i + ln > end:
        raise ValueError("MKV: variable-length integer past its parent")
    v = first if keep_marker else first & (0xFF >> ln)
    for k in range(1, ln):
        v = (v << 8) | b[i + k]
    if not keep_marker and v == (1 << (7 * ln)) - 1:
        v = -1  # unknown size
    return v, i + ln


def _elements(b: bytes, start: int, end: int):
    """(id, data start, data end) of the EBML elements in [start, end); an unknown size
    extends to the end of the parent."""
    i = start
    while i < end:
        eid, j = _vint(b, i, end, True)
        size, k = _vint(b, j, end, False)
        e = end if size < 0 else k + size
        if e > end:
            raise ValueError(f"MKV: element {eid:#x} overruns its parent")
        yield eid, k, e
        i = e


def _uint(b: bytes, s: int, e: int) -> int:
    return int.from_bytes(b[s:e], "big") if e > s else 0


def _float(b: bytes, s: int, e: int) -> float:
    if e - s == 4:
        return struct.unpack(">f", b[s:e])[0]
    if e - s == 8:
        return struct.unpack(">d", b[s:e])[0]
    return 0.0


def _laced(b: bytes, s: int, e: int, lacing: int) -> list[bytes]:
    """Frames of a (Simple)Block payload starting at the lacing header."""
    if lacing == 0:
        return [bytes(b[s:e])]
    if s >= e:
        raise ValueError("MKV: empty laced block")
    count = b[s] + 1
    i = s + 1
    sizes: list[int] = []
    if lacing == 1:  # Xiph
        for _ in range(count - 1):
            v = 0
            while True:
                if i >= e:
                    raise ValueError("MKV: Xiph lacing past the block")
                v += b[i]
                i += 1
                if b[i - 1] != 255:
                    break
            sizes.append(v)
    elif lacing == 3:  # EBML
        v, i = _vint(b, i, e, False)
        sizes.append(v)
        for _ in range(count - 2):
            raw, j = _vint(b, i, e, False)
            ln = j - i
            sizes.append(sizes[-1] + raw - ((1 << (7 * ln - 1)) - 1))
            i = j
    elif lacing == 2:  # fixed
        total = e - i
        if total % count:
            raise ValueError("MKV: fixed lacing does not divide the block")
        sizes = [total // count] * (count - 1)
    rest = e - i - sum(sizes)
    if rest < 0 or any(x < 0 for x in sizes):
        raise ValueError("MKV: lace sizes exceed the block")
    sizes.append(rest)
    out = []
    for z in sizes:
        out.append(bytes(b[i:i + z]))
        i += z
    return out


def _nal_config(codec: str, priv: bytes) -> tuple[int, bytes]:
    """(NAL length size, Annex-B parameter sets) from avcC / hvcC CodecPrivate."""
    sc = b"\x00\x00\x00\x01"
    out = bytearray()
    if codec == "h264":
        if len(priv) < 7:
            raise ValueError("MKV: short avcC")
        nls = (priv[4] & 3) + 1
        p = 5
        for mask in (0x1F, 0xFF):
            cnt = priv[p] & mask
            p += 1
            for _ in range(cnt):
                ln = struct.unpack(">H", priv[p:p + 2])[0]
                out += sc + priv[p + 2:p + 2 + ln]
                p += 2 + ln
    else:
        if len(priv) < 23:
            raise ValueError("MKV: short hvcC")
        nls = (priv[21] & 3) + 1
        p = 23
        for _ in range(priv[22]):
            cnt = struct.unpack(">H", priv[p + 1:p + 3])[0]
            p += 3
            for _ in range(cnt):
                ln = struct.unpack(">H", priv[p:p + 2])[0]
                out += sc + priv[p + 2:p + 2 + ln]
                p += 2 + ln
    if p > len(priv):
        raise ValueError("MKV: codec configuration record overruns CodecPrivate")
    return nls, bytes(out)


def mkv_demux(data: bytes) -> Demuxed:
    try:
        return _mkv_demux(data)
    except (IndexError, struct.error, UnicodeDecodeError) as e:
        raise ValueError(f"MKV: malformed stream ({e})") from None


def _mkv_demux(data: bytes) -> Demuxed:
    b = data
    n = len(b)
    if not is_mkv(b[:4]):
        raise ValueError("MKV: no EBML header")
    seg = None
    for eid, s, e in _elements(b, 0, n):
        if eid == MKV_SEGMENT:
            seg = (s, e)
            break
    if seg is None:
        raise ValueError("MKV: no Segment")
    scale = 1_000_000  # TimestampScale, ns
    tracks: dict[int, dict] = {}
    blocks: dict[int, list[tuple[float, bytes]]] = {}

    def block(tn_data: tuple[int, int], cluster_tc: int):
        s, e = tn_data
        tn, i = _vint(b, s, e, False)
        if i + 3 > e:
            raise ValueError("MKV: short block header")
        rel = struct.unpack(">h", b[i:i + 2])[0]
        flags = b[i + 2]
        t = (cluster_tc + rel) * scale / 1e9
        for fr in _laced(b, i + 3, e, (flags >> 1) & 3):
            blocks.setdefault(tn, []).append((t, fr))

    for eid, s, e in _elements(b, *seg):
        if eid == MKV_INFO:
            for cid, cs, ce in _elements(b, s, e):
                if cid == 0x2AD7B1:
                    scale = _uint(b, cs, ce) or scale
        elif eid == MKV_TRACKS:
            for tid, ts_, te in _elements(b, s, e):
                if tid != 0xAE:
                    continue
                t = {"number": 0, "type": 0, "codec": "", "priv": b"", "w": 0, "h": 0, "rate": 0.0, "ch": 1}
                for cid, cs, ce in _elements(b, ts_, te):
                    if cid == 0xD7:
                        t["number"] = _uint(b, cs, ce)
                    elif cid == 0x83:
                        t["type"] = _uint(b, cs, ce)
                    elif cid == 0x86:
                        t["codec"] = bytes(b[cs:ce]).rstrip(b"\0").decode("ascii", "replace")
                    elif cid == 0x63A2:
                        t["priv"] = bytes(b[cs:ce])
                    elif cid == 0xE0:
                        for vid, vs, ve in _elements(b, cs, ce):
                            if vid == 0xB0:
                                t["w"] = _uint(b, vs, ve)
                            elif vid == 0xBA:
                                t["h"] = _uint(b, vs, ve)
                    elif cid == 0xE1:
                        for aid, as_, ae in _elements(b, cs, ce):
                            if aid == 0xB5:
                                t["rate"] = _float(b, as_, ae)
                            elif aid == 0x9F:
                                t["ch"] = _uint(b, as_, ae)
                tracks[t["number"]] = t
        elif eid == MKV_CLUSTER:
            tc = 0
            for cid, cs, ce in _elements(b, s, e):
                if cid == 0xE7:
                    tc = _uint(b, cs, ce)
                elif cid == 0xA3:  # SimpleBlock
                    block((cs, ce), tc)
                elif cid == 0xA0:  # BlockGroup
                    for gid, gs, ge in _elements(b, cs, ce):
                        if gid == 0xA1:
                            block((gs, ge), tc)
    vids = [t for t in tracks.values() if t["type"] == 1 and t["codec"] in MKV_VIDEO]
    if not vids:
        raise ValueError("MKV: no H.264 / HEVC video track")
    v = vids[0]
    codec = MKV_VIDEO[v["codec"]]
    nls, ps = _nal_config(codec, v["priv"])
    out_v = bytearray(ps)
    sc = b"\x00\x00\x00\x01"
    frames = blocks.get(v["number"], [])
    for _, fr in frames:
        q = 0
        while q < len(fr):
            ln = int.from_bytes(fr[q:q + nls], "big")
            if ln <= 0 or q + nls + ln > len(fr):
                raise ValueError("MKV: NAL length field overruns its frame")
            out_v += sc + fr[q + nls:q + nls + ln]
            q += nls + ln
    t0 = min((t for t, _ in frames), default=0.0)
    out = Demuxed(codec, bytes(out_v), [t - t0 for t, _ in frames], width=v["w"], height=v["h"])
    for t in tracks.values():
        if t is v or t["type"] != 2:
            if t is not v and t["type"] == 1:
                out.dropped.append(f"MKV video track {t['number']} ({t['codec']})")
            continue
        if t["codec"] != "A_AAC" or len(t["priv"]) < 2:
            out.dropped.append(f"MKV audio track {t['number']} ({t['codec']})")
            continue
        af = blocks.get(t["number"], [])
        if not af:
            continue
        asc = t["priv"]
        sfi = ((asc[0] & 7) << 1) | (asc[1] >> 7)
        rate = int(t["rate"]) or (AAC_RATES[sfi] if sfi < len(AAC_RATES) else 48000)
        ch = t["ch"] or ((asc[1] >> 3) & 15)
        out.audio.append(aac_track(asc, rate, ch, [fr for _, fr in af], af[0][0] - t0))
    return out


def demux(path_or_data, kind: str) -> Demuxed:
    data = path_or_data
    if isinstance(path_or_data, str):
        with open(path_or_data, "rb") as f:
            data = f.read()
    if kind == "ts":
        return ts_demux(data)
    if kind == "mkv":
        return mkv_demux(data)
    raise ValueError(f"no demuxer for {kind}")
