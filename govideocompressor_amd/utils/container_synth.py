"""Minimal MPEG-TS and Matroska writers for tests (no ffmpeg in the image): an Annex-B H.264
or HEVC stream (+ raw AAC frames) -> ``.ts`` (PAT/PMT with CRC-32, one PES per access unit
with PTS/DTS, ADTS audio) or ``.mkv`` (EBML, avcC / hvcC CodecPrivate, clusters of
SimpleBlocks in decode order stamped with presentation times, EBML- or Xiph-laced audio).

They feed ``segment/containers.py``'s demuxers in tests/test_containers.py."""
from __future__ import annotations

import struct

from ..segment import mp4
from ..segment.containers import AAC_RATES, asc_of


def video_track(stream: bytes, fps: float):
    from ..segment import mp4_hevc
    if mp4_hevc.is_hevc_annexb(stream):
        return mp4_hevc.hevc_track(stream, fps), "hevc"
    return mp4.h264_track(stream, fps), "h264"


def _to_annexb(sample: bytes) -> bytes:
    out, q = bytearray(), 0
    while q < len(sample):
        ln = int.from_bytes(sample[q:q + 4], "big")
        out += b"\x00\x00\x00\x01" + sample[q + 4:q + 4 + ln]
        q += 4 + ln
    return bytes(out)


def _params(track) -> bytes:
    t = mp4.Track(track.handler, track.timescale, track.sample_entry)
    return mp4.video_to_annexb(t)


# ------------------------------------------------------------------------------- MPEG-TS
def crc32_mpeg(data: bytes) -> int:
    crc = 0xFFFFFFFF
    for byte in data:
        crc ^= byte << 24
        for _ in range(8):
            crc = ((crc << 1) ^ 0x04C11DB7) & 0xFFFFFFFF if crc & 0x80000000 else (crc << 1) & 0xFFFFFFFF
    return crc


def _ts_time(prefix: int, v: int) -> bytes:
    return bytes([(prefix << 4) | (((v >> 30) & 7) << 1) | 1, (v >> 22) & 0xFF, (((v >> 15) & 0x7F) << 1) | 1,
                  (v >> 7) & 0xFF, ((v & 0x7F) << 1) | 1])


def _pes(stream_id: int, payload: bytes, pts: int | None, dts: int | None, bounded: bool) -> bytes:
    if pts is None:  # a PES without timestamps
        opt = bytes([0x80, 0x00, 0])
    else:
        hdr = _ts_time(3 if dts is not None else 2, pts) + (_ts_time(1, dts) if dts is not None else b"")
        opt = bytes([0x80, 0xC0 if dts is not None else 0x80, len(hdr)]) + hdr
    n = len(opt) + len(payload)
    return b"\x00\x00\x01" + bytes([stream_id]) + struct.pack(">H", n if bounded and n < 65536 else 0) + opt + payload


class _TsWriter:
    def __init__(self):
        self.cc: dict[int, int] = {}
        self.out = bytearray()

    def packets(self, pid: int, payload: bytes, psi: bool = False):
        first = True
        i = 0
        while first or i < len(payload):
            cc = self.cc.get(pid, 0)
            self.cc[pid] = (cc + 1) & 15
            chunk = payload[i:i + 184]
            hdr = bytes([0x47, (0x40 if first else 0) | (pid >> 8), pid & 0xFF])
            if len(chunk) < 184:
                if psi:
                    pkt = hdr + bytes([0x10 | cc]) + chunk + b"\xff" * (184 - len(chunk))
                else:  # adaptation-field stuffing
                    af = 183 - len(chunk)
                    stuffing = bytes([af]) + ((b"\x00" + b"\xff" * (af - 1)) if af > 0 else b"")
                    pkt = hdr + bytes([0x30 | cc]) + stuffing + chunk
            else:
                pkt = hdr + bytes([0x10 | cc]) + chunk
            assert len(pkt) == 188
            self.out += pkt
            i += len(chunk)
            first = False

    def section(self, pid: int, body: bytes):
        sec = body + struct.pack(">I", crc32_mpeg(body))
        self.packets(pid, b"\x00" + sec, psi=True)


def write_ts(stream: bytes, fps: float = 25.0, audio: list[bytes] | None = None, rate: int = 48000,
             channels: int = 2, base_s: float = 1.0, audio_delay_s: float = 0.0, pes_pictures: int = 1,
             no_pts: tuple = ()) -> bytes:
    """Annex-B video (+ raw AAC frames, 1024 samples each) -> an MPEG transport stream.

    ``base_s``: the first PTS (values past 2^33 ticks wrap, as a long capture's do);
    ``audio_delay_s``: the audio starts that much after the first picture;
    ``pes_pictures``: pictures per video PES (only the first carries the PTS);
    ``no_pts``: picture indexes whose PES is written without a PTS."""
    track, codec = video_track(stream, fps)
    w = _TsWriter()
    vpid, apid, pmt = 0x100, 0x101, 0x1000
    pat = bytes([0x00, 0xB0, 13, 0x00, 0x01, 0xC1, 0x00, 0x00, 0x00, 0x01, 0xE0 | (pmt >> 8), pmt & 0xFF])
    es = bytes([0x1B if codec == "h264" else 0x24, 0xE0 | (vpid >> 8), vpid & 0xFF, 0xF0, 0x00])
    if audio:
        es += bytes([0x0F, 0xE0 | (apid >> 8), apid & 0xFF, 0xF0, 0x00])
    body = bytes([0x00, 0x01, 0xC1, 0x00, 0x00, 0xE0 | (vpid >> 8), vpid & 0xFF, 0xF0, 0x00]) + es
    pmt_sec = bytes([0x02, 0xB0 | ((len(body) + 4) >> 8), (len(body) + 4) & 0xFF]) + body
    w.section(0, pat)
    w.section(pmt, pmt_sec)
    pts = track.pts_seconds()
    delay = track.media_time / track.timescale
    params = _params(track)
    base = int(base_s * 90000)
    aframes = list(audio or [])
    sfi = AAC_RATES.index(rate)
    ai = 0
    for k, s in enumerate(track.samples):
        if k % pes_pictures == 0:
            au = b"".join((params if j == 0 else b"") + _to_annexb(track.samples[j])
                          for j in range(k, min(k + pes_pictures, len(track.samples))))
            p90 = base + int(round((pts[k] + delay) * 90000))
            d90 = base + int(round(k / fps * 90000))
            if k in no_pts:
                p90 = d90 = None
            w.packets(vpid, _pes(0xE0, au, p90, d90 if d90 != p90 else None, bounded=False))
        # audio up to this picture's decode time, 4 frames per PES
        last = k + 1 == len(track.samples)
        while ai < len(aframes) and (last or ai * 1024 / rate <= (k + 1) / fps):
            chunk = aframes[ai:ai + 4]
            adts = b""
            for fr in chunk:
                flen = len(fr) + 7
                adts += bytes([0xFF, 0xF1, (1 << 6) | (sfi << 2) | (channels >> 2), ((channels & 3) << 6) | (flen >> 11),
                               (flen >> 3) & 0xFF, ((flen & 7) << 5) | 0x1F, 0xFC]) + fr
            a90 = base + int(round((delay + audio_delay_s + ai * 1024 / rate) * 90000))
            w.packets(apid, _pes(0xC0, adts, a90, None, bounded=True))
            ai += len(chunk)
    return bytes(w.out)


# ------------------------------------------------------------------------------- Matroska
def _ebml_id(eid: int) -> bytes:
    n = (eid.bit_length() + 7) // 8
    return eid.to_bytes(n, "big")


def _ebml_size(n: int) -> bytes:
    for ln in range(1, 9):
        if n < (1 << (7 * ln)) - 1:
            return (n | (1 << (7 * ln))).to_bytes(ln, "big")
    raise ValueError("EBML size too large")


def el(eid: int, payload: bytes) -> bytes:
    return _ebml_id(eid) + _ebml_size(len(payload)) + payload


def el_uint(eid: int, v: int) -> bytes:
    return el(eid, v.to_bytes(max(1, (v.bit_length() + 7) // 8), "big"))


def write_mkv(stream: bytes, fps: float = 25.0, audio: list[bytes] | None = None, rate: int = 48000,
              channels: int = 2, lacing: str = "ebml") -> bytes:
    """Annex-B video (+ raw AAC frames) -> Matroska; video blocks in decode order stamped
    with presentation times (ms), audio laced 4 frames per block (``ebml`` / ``xiph``)."""
    track, codec = video_track(stream, fps)
    kind = b"avcC" if codec == "h264" else b"hvcC"
    priv = mp4._config_box(track.sample_entry, kind)
    head = el(0x1A45DFA3, el_uint(0x4286, 1) + el_uint(0x42F7, 1) + el_uint(0x42F2, 4) + el_uint(0x42F3, 8) +
              el(0x4282, b"matroska") + el_uint(0x4287, 4) + el_uint(0x4285, 2))
    info = el(0x1549A966, el_uint(0x2AD7B1, 1_000_000) + el(0x4D80, b"mivc-test") + el(0x5741, b"mivc-test"))
    vtrack = el(0xAE, el_uint(0xD7, 1) + el_uint(0x73C5, 1) + el_uint(0x83, 1) +
                el(0x86, b"V_MPEG4/ISO/AVC" if codec == "h264" else b"V_MPEGH/ISO/HEVC") + el(0x63A2, priv) +
                el(0xE0, el_uint(0xB0, track.width) + el_uint(0xBA, track.height)))
    tracks = vtrack
    if audio:
        asc = asc_of(1, AAC_RATES.index(rate), channels)
        tracks += el(0xAE, el_uint(0xD7, 2) + el_uint(0x73C5, 2) + el_uint(0x83, 2) + el(0x86, b"A_AAC") +
                     el(0x63A2, asc) + el(0xE1, el(0xB5, struct.pack(">d", float(rate))) + el_uint(0x9F, channels)))
    pts = track.pts_seconds()
    delay = track.media_time / track.timescale
    clusters = b""
    sync = track.sync or [True] * len(track.samples)
    aframes = list(audio or [])
    ai = 0
    k = 0
    while k < len(track.samples):
        # one cluster per keyframe run
        j = k + 1
        while j < len(track.samples) and not sync[j]:
            j += 1
        ctc = int(round((pts[k] + delay) * 1000))
        body = el_uint(0xE7, ctc)
        for i in range(k, j):
            ms = int(round((pts[i] + delay) * 1000)) - ctc
            body += el(0xA3, b"\x81" + struct.pack(">hB", ms, 0x80 if sync[i] else 0) + track.samples[i])
        t_end = (j / fps) + delay
        while ai < len(aframes) and (j == len(track.samples) or ai * 1024 / rate < t_end):
            chunk = aframes[ai:ai + 4]
            ms = int(round((delay + ai * 1024 / rate) * 1000)) - ctc
            if len(chunk) == 1:
                blk = b"\x82" + struct.pack(">hB", ms, 0x80) + chunk[0]
            elif lacing == "xiph":
                lace = b""
                for fr in chunk[:-1]:
                    n = len(fr)
                    lace += b"\xff" * (n // 255) + bytes([n % 255])
                blk = b"\x82" + struct.pack(">hB", ms, 0x80 | 0x02) + bytes([len(chunk) - 1]) + lace + b"".join(chunk)
            else:
                lace = _ebml_size(len(chunk[0]))
                for a, b in zip(chunk[:-2], chunk[1:-1]):
                    d = len(b) - len(a)
                    ln = 1
                    while not (-(1 << (7 * ln - 1)) + 1 <= d <= (1 << (7 * ln - 1)) - 1):
                        ln += 1
                    lace += (d + (1 << (7 * ln - 1)) - 1 | (1 << (7 * ln))).to_bytes(ln, "big")
                blk = b"\x82" + struct.pack(">hB", ms, 0x80 | 0x06) + bytes([len(chunk) - 1]) + lace + b"".join(chunk)
            body += el(0xA3, blk)
            ai += len(chunk)
        clusters += el(0x1F43B675, body)
        k = j
    seg = el(0x18538067, info + el(0x1654AE6B, tracks) + clusters)
    return head + seg
