"""ISO-BMFF (MP4) reader / writer for every track kind: the container layer of split,
worker output and merge.

The reference's pieces are ``.mp4`` files cut with ``ffmpeg -f segment -c copy
-acodec copy -map 0:0 -map 0:1`` (server.go:199-201): video AND audio travel together,
the worker's ffmpeg writes an ``.mp4`` (client.go:115) and ``concat.sh`` stream-copies
every track into the result (server.go:357).  This module gives the same data flow
without ffmpeg:

* :func:`read` -- every ``trak`` of a file: sample bytes (``stco``/``co64`` +
  ``stsc`` + ``stsz``), decode durations (``stts``), composition offsets (``ctts`` v0/v1),
  sync samples (``stss``), the first edit's ``media_time`` (``elst``), timescale, handler
  and the raw sample entry (``stsd``), so any codec passes through untouched;
* :func:`write` -- tracks back into one file: ``mdat`` chunks of <= 0.5 s interleaved by
  time, ``co64`` when offsets pass 4 GiB, version-1 ``mvhd``/``tkhd``/``mdhd`` for
  64-bit durations, ``ctts`` + an edit list for reordered (B-picture) video;
* :func:`h264_track` / :func:`video_to_annexb` -- H.264 Annex-B <-> ``avc1`` samples
  with ``avcC``, composition offsets from picture order counts (``_host.h264_samples``);
* :func:`cut` / :func:`concat` -- an audio track's samples for one piece's time range,
  and the pieces' tracks appended back to back (same sample entry required).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

VIDEO_CODECS = (b"avc1", b"avc3", b"hvc1", b"hev1")


@dataclass
class Track:
    handler: bytes                      # b"vide", b"soun", ...
    timescale: int
    sample_entry: bytes                 # one complete sample entry box (goes into stsd)
    samples: list[bytes] = field(default_factory=list)
    durations: list[int] = field(default_factory=list)   # decode-time deltas
    cts: list[int] | None = None        # composition offsets (None: all zero)
    sync: list[bool] | None = None      # None: every sample is a sync sample
    width: int = 0
    height: int = 0
    # the media edit's media_time (media timescale): samples before it are hidden (B-picture
    # reordering delay, AAC priming); 0 = the media plays from its start
    media_time: int = 0
    language: int = 0x55C4              # 'und'
    # start delay (media timescale): an empty edit of this length plays before the media edit
    # (audio beginning after the video).  Independent of media_time, so a late AAC track keeps
    # its priming skip.  A negative media_time given to the constructor means a delay (older
    # callers' convention) and is moved here.
    delay: int = 0

    def __post_init__(self):
        if self.media_time < 0:
            self.delay += -self.media_time
            self.media_time = 0

    @property
    def codec(self) -> bytes:
        return self.sample_entry[4:8]

    @property
    def duration(self) -> int:
        return int(sum(self.durations))

    def dts(self) -> list[int]:
        out, t = [], 0
        for d in self.durations:
            out.append(t)
            t += d
        return out

    def pts_seconds(self) -> list[float]:
        """Presentation time of every sample (decode order), edit list applied."""
        c = self.cts or [0] * len(self.samples)
        return [(d + o - self.media_time + self.delay) / self.timescale for d, o in zip(self.dts(), c)]


# ------------------------------------------------------------------------------- boxes
def _box(kind: bytes, *payload: bytes) -> bytes:
    body = b"".join(payload)
    if 8 + len(body) > 0xFFFFFFFF:
        return struct.pack(">I", 1) + kind + struct.pack(">Q", 16 + len(body)) + body
    return struct.pack(">I", 8 + len(body)) + kind + body


def _full(kind: bytes, version: int, flags: int, *payload: bytes) -> bytes:
    return _box(kind, struct.pack(">I", (version << 24) | flags), *payload)


_MATRIX = struct.pack(">9I", 0x10000, 0, 0, 0, 0x10000, 0, 0, 0, 0x40000000)


def children(b: bytes, start: int, end: int):
    i = start
    while i + 8 <= end:
        size, kind = struct.unpack(">I4s", b[i:i + 8])
        hdr = 8
        if size == 1:
            size, hdr = struct.unpack(">Q", b[i + 8:i + 16])[0], 16
        elif size == 0:
            size = end - i
        if size < hdr or i + size > end:
            raise ValueError(f"mp4: box {kind!r} at {i} overruns its parent")
        yield kind, i + hdr, i + size
        i += size


def _child(b: bytes, s: int, e: int, kind: bytes):
    for k, a, z in children(b, s, e):
        if k == kind:
            return a, z
    return None


def _need(b: bytes, s: int, e: int, kind: bytes):
    r = _child(b, s, e, kind)
    if r is None:
        raise ValueError(f"mp4: missing {kind.decode()} box")
    return r


def is_mp4(data: bytes) -> bool:
    return len(data) >= 8 and data[4:8] in (b"ftyp", b"moov", b"mdat", b"free", b"skip", b"wide")


# ------------------------------------------------------------------------------- read
def _read_trak(data: bytes, s: int, e: int, movie_ts: int = 1000) -> Track:
    tk = _need(data, s, e, b"tkhd")
    ver = data[tk[0]]
    wh = data[tk[1] - 8:tk[1]]
    width, height = struct.unpack(">II", wh)
    md = _need(data, s, e, b"mdia")
    mh = _need(data, md[0], md[1], b"mdhd")
    if data[mh[0]] == 1:
        timescale = struct.unpack(">I", data[mh[0] + 20:mh[0] + 24])[0]
        lang = struct.unpack(">H", data[mh[0] + 32:mh[0] + 34])[0]
    else:
        timescale = struct.unpack(">I", data[mh[0] + 12:mh[0] + 16])[0]
        lang = struct.unpack(">H", data[mh[0] + 20:mh[0] + 22])[0]
    hd = _need(data, md[0], md[1], b"hdlr")
    handler = data[hd[0] + 8:hd[0] + 12]
    mi = _need(data, md[0], md[1], b"minf")
    st = _need(data, mi[0], mi[1], b"stbl")
    box = {k: (a, z) for k, a, z in children(data, st[0], st[1])}
    sd = box[b"stsd"]
    if struct.unpack(">I", data[sd[0] + 4:sd[0] + 8])[0] < 1:
        raise ValueError("mp4: empty stsd")
    esz = struct.unpack(">I", data[sd[0] + 8:sd[0] + 12])[0]
    entry = data[sd[0] + 8:sd[0] + 8 + esz]
    # sizes
    if b"stsz" in box:
        a = box[b"stsz"][0]
        fixed, n = struct.unpack(">II", data[a + 4:a + 12])
        sizes = [fixed] * n if fixed else list(struct.unpack(f">{n}I", data[a + 12:a + 12 + 4 * n]))
    elif b"stz2" in box:
        a = box[b"stz2"][0]
        fs, n = data[a + 7], struct.unpack(">I", data[a + 8:a + 12])[0]
        if fs == 16:
            sizes = list(struct.unpack(f">{n}H", data[a + 12:a + 12 + 2 * n]))
        elif fs == 8:
            sizes = list(data[a + 12:a + 12 + n])
        else:
            raw = data[a + 12:a + 12 + (n + 1) // 2]
            sizes = [(raw[i // 2] >> (4 * (1 - i % 2))) & 15 for i in range(n)]
    else:
        raise ValueError("mp4: no sample sizes")
    n = len(sizes)
    # chunk offsets
    if b"co64" in box:
        a = box[b"co64"][0]
        nc = struct.unpack(">I", data[a + 4:a + 8])[0]
        offs = list(struct.unpack(f">{nc}Q", data[a + 8:a + 8 + 8 * nc]))
    else:
        a = box[b"stco"][0]
        nc = struct.unpack(">I", data[a + 4:a + 8])[0]
        offs = list(struct.unpack(f">{nc}I", data[a + 8:a + 8 + 4 * nc]))
    a = box[b"stsc"][0]
    ne = struct.unpack(">I", data[a + 4:a + 8])[0]
    runs = [struct.unpack(">III", data[a + 8 + 12 * i:a + 20 + 12 * i]) for i in range(ne)]
    samples, k, ri, per = [], 0, 0, 0
    for ci, off in enumerate(offs):
        while ri < len(runs) and runs[ri][0] <= ci + 1:
            per = runs[ri][1]
            ri += 1
        for _ in range(per):
            if k >= n:
                break
            if off + sizes[k] > len(data):
                raise ValueError("mp4: sample data past the end of the file")
            samples.append(data[off:off + sizes[k]])
            off += sizes[k]
            k += 1
    if k != n:
        raise ValueError(f"mp4: chunk table covers {k} of {n} samples")
    # timing
    a = box[b"stts"][0]
    ne = struct.unpack(">I", data[a + 4:a + 8])[0]
    durs: list[int] = []
    for i in range(ne):
        c, d = struct.unpack(">II", data[a + 8 + 8 * i:a + 16 + 8 * i])
        durs += [d] * c
    durs = (durs + [durs[-1] if durs else 1] * n)[:n]
    cts = None
    if b"ctts" in box:
        a = box[b"ctts"][0]
        v = data[a]
        ne = struct.unpack(">I", data[a + 4:a + 8])[0]
        cts = []
        for i in range(ne):
            c, o = struct.unpack(">Ii" if v == 1 else ">II", data[a + 8 + 8 * i:a + 16 + 8 * i])
            cts += [o] * c
        cts = (cts + [0] * n)[:n]
    sync = None
    if b"stss" in box:
        a = box[b"stss"][0]
        ne = struct.unpack(">I", data[a + 4:a + 8])[0]
        marks = set(struct.unpack(f">{ne}I", data[a + 8:a + 8 + 4 * ne]))
        sync = [(i + 1) in marks for i in range(n)]
    media_time = delay = 0
    ed = _child(data, s, e, b"edts")
    if ed is not None:
        el = _child(data, ed[0], ed[1], b"elst")
        if el is not None:
            v = data[el[0]]
            ne = struct.unpack(">I", data[el[0] + 4:el[0] + 8])[0]
            p = el[0] + 8
            empty = 0  # leading empty edits (media_time -1): a start delay, movie timescale
            for _ in range(ne):
                if v == 1:
                    sd, mt = struct.unpack(">Qq", data[p:p + 16])
                    p += 20
                else:
                    sd, mt = struct.unpack(">Ii", data[p:p + 8])
                    p += 12
                if mt < 0:
                    empty += sd
                    continue
                media_time = mt
                delay = (empty * timescale + movie_ts // 2) // max(movie_ts, 1)
                break
    del ver
    return Track(handler, timescale, entry, samples, durs, cts, sync, width >> 16, height >> 16, media_time, lang, delay)


def read(data: bytes) -> list[Track]:
    """Every track of an MP4 file (bytes).  Malformed input raises ValueError."""
    try:
        mv = _child(data, 0, len(data), b"moov")
        if mv is None:
            raise ValueError("mp4: no moov box")
        mts = 1000
        mh = _child(data, mv[0], mv[1], b"mvhd")
        if mh is not None:
            mts = struct.unpack(">I", data[mh[0] + (20 if data[mh[0]] == 1 else 12):][:4])[0] or 1000
        return [_read_trak(data, a, z, mts) for k, a, z in children(data, mv[0], mv[1]) if k == b"trak"]
    except (KeyError, struct.error, IndexError, OverflowError, MemoryError) as e:
        raise ValueError(f"mp4: malformed file ({type(e).__name__}: {e})") from None


def video_track(tracks: list[Track]) -> Track:
    for t in tracks:
        if t.handler == b"vide" and t.codec in VIDEO_CODECS:
            return t
    raise ValueError("mp4: no H.264/HEVC video track (avc1/avc3/hvc1/hev1)")


def audio_tracks(tracks: list[Track]) -> list[Track]:
    return [t for t in tracks if t.handler == b"soun"]


# ------------------------------------------------------------------------------- write
def _runs(values):
    out = []
    for v in values:
        if out and out[-1][1] == v:
            out[-1][0] += 1
        else:
            out.append([1, v])
    return out


def _trak(t: Track, track_id: int, chunks: list[tuple[int, int]], offs: list[int], movie_ts: int, wide: bool) -> bytes:
    n = len(t.samples)
    media_dur = t.duration
    edit_dur = media_dur - t.media_time
    movie_dur = ((edit_dur + t.delay) * movie_ts + t.timescale - 1) // t.timescale
    v1 = media_dur > 0xFFFFFFFF or movie_dur > 0xFFFFFFFF
    stts = _full(b"stts", 0, 0, struct.pack(">I", len(r := _runs(t.durations))), *(struct.pack(">II", c, d) for c, d in r))
    parts = [_full(b"stsd", 0, 0, struct.pack(">I", 1), t.sample_entry), stts]
    if t.cts is not None and any(t.cts):
        neg = min(t.cts) < 0
        r = _runs(t.cts)
        parts.append(_full(b"ctts", 1 if neg else 0, 0, struct.pack(">I", len(r)),
                           *(struct.pack(">Ii" if neg else ">II", c, o) for c, o in r)))
    if t.sync is not None and not all(t.sync):
        ss = [i + 1 for i, s in enumerate(t.sync) if s]
        parts.append(_full(b"stss", 0, 0, struct.pack(">I", len(ss)), *(struct.pack(">I", x) for x in ss)))
    spc = [c for _, c in chunks]
    stsc_rows, prev = [], None
    for i, c in enumerate(spc):
        if c != prev:
            stsc_rows.append((i + 1, c, 1))
            prev = c
    parts.append(_full(b"stsc", 0, 0, struct.pack(">I", len(stsc_rows)), *(struct.pack(">III", *r) for r in stsc_rows)))
    sizes = [len(s) for s in t.samples]
    if n and all(x == sizes[0] for x in sizes):
        parts.append(_full(b"stsz", 0, 0, struct.pack(">II", sizes[0], n)))
    else:
        parts.append(_full(b"stsz", 0, 0, struct.pack(">II", 0, n), struct.pack(f">{n}I", *sizes) if n else b""))
    if wide:
        parts.append(_full(b"co64", 0, 0, struct.pack(">I", len(offs)), struct.pack(f">{len(offs)}Q", *offs)))
    else:
        parts.append(_full(b"stco", 0, 0, struct.pack(">I", len(offs)), struct.pack(f">{len(offs)}I", *offs)))
    stbl = _box(b"stbl", *parts)
    if t.handler == b"vide":
        mhd = _full(b"vmhd", 0, 1, bytes(8))
        name = b"VideoHandler\x00"
    elif t.handler == b"soun":
        mhd = _full(b"smhd", 0, 0, bytes(4))
        name = b"SoundHandler\x00"
    else:
        mhd = _full(b"nmhd", 0, 0)
        name = b"DataHandler\x00"
    minf = _box(b"minf", mhd, _box(b"dinf", _full(b"dref", 0, 0, struct.pack(">I", 1), _full(b"url ", 0, 1))), stbl)
    if v1:
        mdhd = _full(b"mdhd", 1, 0, struct.pack(">QQIQHH", 0, 0, t.timescale, media_dur, t.language, 0))
    else:
        mdhd = _full(b"mdhd", 0, 0, struct.pack(">IIIIHH", 0, 0, t.timescale, media_dur, t.language, 0))
    mdia = _box(b"mdia", mdhd, _full(b"hdlr", 0, 0, bytes(4), t.handler, bytes(12), name), minf)
    vol = 0x0100 if t.handler == b"soun" else 0
    if v1:
        tkhd = _full(b"tkhd", 1, 3, struct.pack(">QQIIQ", 0, 0, track_id, 0, movie_dur), bytes(8),
                     struct.pack(">hhhH", 0, 0, vol, 0), _MATRIX, struct.pack(">II", t.width << 16, t.height << 16))
    else:
        tkhd = _full(b"tkhd", 0, 3, struct.pack(">IIIII", 0, 0, track_id, 0, movie_dur), bytes(8),
                     struct.pack(">hhhH", 0, 0, vol, 0), _MATRIX, struct.pack(">II", t.width << 16, t.height << 16))
    boxes = [tkhd]
    if t.delay > 0:  # start delay: an empty edit, then the media from media_time
        delay = (t.delay * movie_ts + t.timescale // 2) // t.timescale
        media_movie = (edit_dur * movie_ts + t.timescale - 1) // t.timescale
        fmt = ">IQqhhQqhh" if v1 else ">IIihhIihh"
        el = _full(b"elst", 1 if v1 else 0, 0, struct.pack(fmt, 2, delay, -1, 1, 0, media_movie, t.media_time, 1, 0))
        boxes.append(_box(b"edts", el))
    elif t.media_time > 0:
        if v1:
            el = _full(b"elst", 1, 0, struct.pack(">IQqhh", 1, movie_dur, t.media_time, 1, 0))
        else:
            el = _full(b"elst", 0, 0, struct.pack(">IIihh", 1, movie_dur, t.media_time, 1, 0))
        boxes.append(_box(b"edts", el))
    return _box(b"trak", *boxes, mdia)


def write(tracks: list[Track], brand: bytes = b"isom", chunk_seconds: float = 0.5) -> bytes:
    """Tracks -> MP4 bytes (``ftyp``, ``mdat`` of time-interleaved chunks, ``moov``)."""
    if not tracks:
        raise ValueError("mp4: nothing to write")
    movie_ts = 1000
    # chunks: (track, first sample, count) cut every chunk_seconds of decode time
    chunk_list = []
    per_track: list[list[tuple[int, int]]] = []
    for ti, t in enumerate(tracks):
        if len(t.durations) != len(t.samples):
            raise ValueError("mp4: one duration per sample")
        cs, start, t0, acc = [], 0, 0, 0
        limit = max(1, int(chunk_seconds * t.timescale))
        for i, d in enumerate(t.durations):
            acc += d
            if acc - t0 >= limit or i == len(t.durations) - 1:
                cs.append((start, i + 1 - start))
                chunk_list.append((t0 / t.timescale, ti, len(cs) - 1))
                start, t0 = i + 1, acc
        per_track.append(cs)
    chunk_list.sort()
    total = sum(len(s) for t in tracks for s in t.samples)
    ftyp = _box(b"ftyp", brand, struct.pack(">I", 512), b"isomiso2avc1mp41")
    big = total + 16 > 0xFFFFFFFF
    mdat_hdr = (struct.pack(">I", 1) + b"mdat" + struct.pack(">Q", 16 + total)) if big else \
        struct.pack(">I", 8 + total) + b"mdat"
    base = len(ftyp) + len(mdat_hdr)
    wide = base + total > 0xFFFFFFFF
    offs = [[0] * len(cs) for cs in per_track]
    body = bytearray()
    for _, ti, ci in chunk_list:
        offs[ti][ci] = base + len(body)
        s0, cnt = per_track[ti][ci]
        for s in tracks[ti].samples[s0:s0 + cnt]:
            body += s
    moov_dur = max((t.duration - t.media_time + t.delay) * movie_ts // t.timescale for t in tracks)
    v1 = moov_dur > 0xFFFFFFFF
    if v1:
        mvhd = _full(b"mvhd", 1, 0, struct.pack(">QQIQ", 0, 0, movie_ts, moov_dur), struct.pack(">IH", 0x10000, 0x100),
                     bytes(10), _MATRIX, bytes(24), struct.pack(">I", len(tracks) + 1))
    else:
        mvhd = _full(b"mvhd", 0, 0, struct.pack(">IIII", 0, 0, movie_ts, moov_dur), struct.pack(">IH", 0x10000, 0x100),
                     bytes(10), _MATRIX, bytes(24), struct.pack(">I", len(tracks) + 1))
    traks = [_trak(t, i + 1, [(s, c) for s, c in per_track[i]], offs[i], movie_ts, wide) for i, t in enumerate(tracks)]
    return ftyp + mdat_hdr + bytes(body) + _box(b"moov", mvhd, *traks)


# ------------------------------------------------------------------------------- H.264
def avcc_record(sps: bytes, pps: bytes) -> bytes:
    return (bytes([1, sps[1], sps[2], sps[3], 0xFF, 0xE1]) + struct.pack(">H", len(sps)) + sps +
            bytes([1]) + struct.pack(">H", len(pps)) + pps)


def _visual_entry(fourcc: bytes, w: int, h: int, config: bytes) -> bytes:
    return _box(fourcc, bytes(6), struct.pack(">H", 1), bytes(16), struct.pack(">HHII", w, h, 0x480000, 0x480000),
                struct.pack(">IH", 0, 1), bytes(32), struct.pack(">Hh", 0x18, -1), config)


def reorder_offsets(display: list[int], delta: int) -> tuple[list[int], int]:
    """Composition offsets (non-negative, ctts v0) and the edit-list media_time for
    samples whose display index is ``display[i]`` (decode order i)."""
    delay = max([i - d for i, d in enumerate(display)] + [0])
    return [(d - i + delay) * delta for i, d in enumerate(display)], delay * delta


def h264_track(stream: bytes, fps: float | None = None) -> Track:
    """Annex-B H.264 -> an ``avc1`` video track (B pictures get ctts + an edit list)."""
    from ..ops import native
    hs = native.host().h264_samples(stream)
    fps = fps if fps and fps > 0 else (hs["fps"] or 30.0)
    timescale, delta = int(round(fps * 1000)), 1000
    data, samples, p = hs["data"], [], 0
    for s in hs["sizes"]:
        samples.append(data[p:p + s])
        p += s
    cts, media_time = reorder_offsets(list(hs["display"]), delta)
    entry = _visual_entry(b"avc1", hs["width"], hs["height"], _box(b"avcC", avcc_record(hs["sps"], hs["pps"])))
    return Track(b"vide", timescale, entry, samples, [delta] * len(samples), cts if media_time else None,
                 [bool(x) for x in hs["sync"]], hs["width"], hs["height"], media_time)


def _config_box(entry: bytes, kind: bytes) -> bytes:
    r = _child(entry, 8 + 78, len(entry), kind)
    if r is None:
        raise ValueError(f"mp4: sample entry has no {kind.decode()}")
    return entry[r[0]:r[1]]


def video_to_annexb(t: Track) -> bytes:
    """A video track's samples as an Annex-B stream, parameter sets first."""
    out = bytearray()
    sc = b"\x00\x00\x00\x01"
    if t.codec in (b"avc1", b"avc3"):
        rec = _config_box(t.sample_entry, b"avcC")
        nls = (rec[4] & 3) + 1
        p = 5
        for cnt_mask in (0x1F, 0xFF):
            cnt = rec[p] & cnt_mask
            p += 1
            for _ in range(cnt):
                ln = struct.unpack(">H", rec[p:p + 2])[0]
                out += sc + rec[p + 2:p + 2 + ln]
                p += 2 + ln
    elif t.codec in (b"hvc1", b"hev1"):
        rec = _config_box(t.sample_entry, b"hvcC")
        nls = (rec[21] & 3) + 1
        p = 23
        for _ in range(rec[22]):
            cnt = struct.unpack(">H", rec[p + 1:p + 3])[0]
            p += 3
            for _ in range(cnt):
                ln = struct.unpack(">H", rec[p:p + 2])[0]
                out += sc + rec[p + 2:p + 2 + ln]
                p += 2 + ln
    else:
        raise ValueError(f"mp4: {t.codec!r} is not an H.264/HEVC track")
    for s in t.samples:
        q = 0
        while q < len(s):
            ln = int.from_bytes(s[q:q + nls], "big")
            if ln <= 0 or q + nls + ln > len(s):
                raise ValueError("mp4: NAL length field overruns its sample")
            out += sc + s[q + nls:q + nls + ln]
            q += nls + ln
    return bytes(out)


def track_fps(t: Track) -> float:
    if not t.durations:
        return 0.0
    d = sorted(t.durations)[len(t.durations) // 2]
    return t.timescale / d if d else 0.0


# ------------------------------------------------------------------------------- audio
def cut(t: Track, t0: float, t1: float | None) -> Track:
    """Samples of ``t`` whose presentation time lies in [t0, t1) seconds.

    The first piece (t0 = 0) also keeps the samples before time 0 -- the encoder-delay
    (priming) frames an AAC track's edit list hides -- together with the track's
    ``media_time``, so the piece, and the merge that starts with it, play the same samples
    from the same instant as the input."""
    pts = t.pts_seconds()
    # samples the media edit hides (dts + cts < media_time: AAC priming) travel with the track's
    # first presented sample, whichever piece that lands in (a late-starting track included)
    c = t.cts or [0] * len(t.samples)
    hidden = [d + o < t.media_time for d, o in zip(t.dts(), c)]
    eff = [t.delay / t.timescale if h else x for x, h in zip(pts, hidden)]
    first = t0 <= 1e-9
    keep = [i for i, x in enumerate(eff) if (first or x >= t0 - 1e-9) and (t1 is None or x < t1 - 1e-9)]
    mt = t.media_time if any(hidden[i] for i in keep) else 0
    delay = t.delay if first else 0
    if not first and keep and t.durations:
        # a track that starts inside this piece (audio beginning after the video): keep the
        # gap as a start delay instead of playing the samples from the piece's first instant
        gap = eff[keep[0]] - t0
        if gap * t.timescale > 2 * max(t.durations):
            delay = int(round(gap * t.timescale))
    return Track(t.handler, t.timescale, t.sample_entry, [t.samples[i] for i in keep], [t.durations[i] for i in keep],
                 [t.cts[i] for i in keep] if t.cts else None, [t.sync[i] for i in keep] if t.sync else None,
                 t.width, t.height, mt, t.language, delay)


def concat(parts: list[Track], starts: list[float] | None = None) -> Track:
    """Tracks appended in order (a merge's audio); every part needs the same sample entry.
    The first part's edit (its priming samples' ``media_time``) is the result's.  ``starts``
    (seconds, one per part): where each part begins in the result -- when the first part
    with samples is not the first part, or starts with a delay, the result starts late by
    that much (audio beginning after the video)."""
    if starts is not None and len(starts) != len(parts):
        raise ValueError("mp4: one start time per part")
    lead = next((i for i, p in enumerate(parts) if p.samples), None)
    parts = [p for p in parts if p.samples]
    if not parts:
        raise ValueError("mp4: no samples to concatenate")
    first = parts[0]
    if starts is not None and starts[lead] > 0:
        # the part's own delay plus where it begins; its media_time (a priming skip) stays
        first = Track(first.handler, first.timescale, first.sample_entry, first.samples, first.durations, first.cts,
                      first.sync, first.width, first.height, first.media_time, first.language,
                      first.delay + int(round(starts[lead] * first.timescale)))
        parts[0] = first
    for p in parts[1:]:
        if p.sample_entry != first.sample_entry or p.timescale != first.timescale:
            raise ValueError("mp4: pieces carry different audio formats; cannot stream-copy them into one track")
    out = Track(first.handler, first.timescale, first.sample_entry, [], [], None, None, first.width, first.height,
                first.media_time, first.language, first.delay)
    any_cts = any(p.cts for p in parts)
    any_sync = any(p.sync is not None for p in parts)
    cts, sync = [], []
    for p in parts:
        out.samples += p.samples
        out.durations += p.durations
        cts += p.cts if p.cts else [0] * len(p.samples)
        sync += p.sync if p.sync is not None else [True] * len(p.samples)
    out.cts = cts if any_cts else None
    out.sync = sync if any_sync else None
    return out


# ------------------------------------------------------------------------------- helpers
def annexb_from_mp4(data: bytes) -> bytes:
    """The video track (H.264 or HEVC, whichever trak holds it) as Annex-B."""
    return video_to_annexb(video_track(read(data)))


def mux_video(stream: bytes, fps: float | None = None, codec: str | None = None,
              extra: list[Track] | tuple = ()) -> bytes:
    """Annex-B video (+ pass-through tracks, e.g. the piece's audio) -> MP4 bytes."""
    from . import mp4_hevc
    hevc = mp4_hevc.is_hevc_annexb(stream) if codec is None else codec == "hevc"
    v = mp4_hevc.hevc_track(stream, fps) if hevc else h264_track(stream, fps)
    return write([v, *extra])


def file_audio(data: bytes) -> list[Track]:
    """Audio tracks of an MP4 (empty for Annex-B / Y4M data or files without audio)."""
    if not is_mp4(data):
        return []
    try:
        return audio_tracks(read(data))
    except (ValueError, struct.error, IndexError):
        return []
