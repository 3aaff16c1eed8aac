"""Generic MP4 layer (segment/mp4.py): multi-track read/write, ctts from picture order
counts, audio passthrough through split -> worker -> merge (the reference's
``-acodec copy -map 0:0 -map 0:1`` pieces, server.go:199-200, and ``concat -c copy``,
server.go:357).  The audio is a synthetic ``mp4a`` track (opaque samples: the
container layer never decodes audio)."""
import struct

import numpy as np
import pytest

from govideocompressor_amd.segment import mp4
from govideocompressor_amd.utils import yuv


def _audio_track(seconds: float, rate: int = 48000, frame: int = 1024, seed: int = 0) -> mp4.Track:
    rng = np.random.default_rng(seed)
    n = int(np.ceil(seconds * rate / frame))
    esds = mp4._full(b"esds", 0, 0, bytes([3, 25, 0, 1, 0, 4, 17, 0x40, 0x15]) + bytes(12) +
                     bytes([5, 2, 0x11, 0x90, 6, 1, 2]))
    entry = mp4._box(b"mp4a", bytes(6), struct.pack(">H", 1), bytes(8), struct.pack(">HHHHI", 2, 16, 0, 0, rate << 16),
                     esds)
    samples = [rng.integers(0, 256, int(rng.integers(100, 400)), dtype=np.uint8).tobytes() for _ in range(n)]
    return mp4.Track(b"soun", rate, entry, samples, [frame] * n)


def _h264_stream(host, frames=24, w=96, h=64, keyint=6):
    c = yuv.synth_clip_cpu(frames, w, h, seed=3)
    return host.CpuEncoder(dict(width=w, height=h, qp=28, keyint=keyint)).encode(c.i420(), frames, 0), c


def test_write_read_roundtrip_multi_track(host):
    es, _ = _h264_stream(host)
    a = _audio_track(1.0)
    v = mp4.h264_track(es, 24.0)
    data = mp4.write([a, v])  # audio first: readers must find the video trak anyway
    tr = mp4.read(data)
    assert [t.handler for t in tr] == [b"soun", b"vide"]
    assert tr[0].samples == a.samples and tr[0].durations == a.durations and tr[0].sample_entry == a.sample_entry
    assert tr[1].samples == v.samples and tr[1].sync == v.sync
    assert mp4.annexb_from_mp4(data) and len(host.decode(mp4.annexb_from_mp4(data))) == 24
    assert abs(mp4.track_fps(tr[1]) - 24.0) < 1e-6


def test_ctts_from_poc_b_pictures(host):
    from tests.test_h264_bframes import _b_stream
    s, _ = _b_stream(host, 64, 48, 1)
    v = mp4.h264_track(s, 30.0)
    assert v.media_time > 0 and v.cts is not None
    pts = v.pts_seconds()  # coding order I0 P2 B1 -> display 0, 2, 1
    assert np.argsort(pts).tolist() == [0, 2, 1]
    assert abs(min(pts)) < 1e-9
    back = mp4.read(mp4.write([v]))[0]
    assert back.cts == v.cts and back.media_time == v.media_time
    pics = host.decode(mp4.annexb_from_mp4(mp4.write([v])))
    assert [p["poc"] for p in pics] == [0, 2, 4]


def test_cut_and_concat_audio():
    a = _audio_track(2.0, seed=5)
    parts = [mp4.cut(a, 0.0, 0.5), mp4.cut(a, 0.5, 1.25), mp4.cut(a, 1.25, None)]
    assert sum(len(p.samples) for p in parts) == len(a.samples)
    back = mp4.concat(parts)
    assert back.samples == a.samples and back.durations == a.durations
    other = _audio_track(0.2, rate=44100)
    with pytest.raises(ValueError):
        mp4.concat([a, other])


def test_audio_priming_edit_survives_cut_and_concat():
    """An AAC track whose edit list hides one priming frame (media_time 1024): the first piece
    keeps the priming frame and the edit, later pieces start at their own time, and the
    concatenation plays exactly the input's samples with the input's edit."""
    a = _audio_track(1.5, seed=11)
    a.media_time = 1024
    assert a.pts_seconds()[0] < 0
    parts = [mp4.cut(a, 0.0, 0.5), mp4.cut(a, 0.5, 1.0), mp4.cut(a, 1.0, None)]
    assert parts[0].media_time == 1024 and parts[0].samples[0] == a.samples[0]
    assert parts[1].media_time == 0 and parts[2].media_time == 0
    back = mp4.concat(parts)
    assert back.samples == a.samples and back.media_time == 1024
    rt = mp4.read(mp4.write([back]))[0]
    assert rt.media_time == 1024 and rt.samples == a.samples


def test_late_audio_with_priming_keeps_both_edits():
    """Audio that starts 0.4 s after the video AND hides one AAC priming frame: the empty
    edit (delay) and the media edit (media_time 1024) are both kept through write / read,
    cut and concat with the pieces' start times (round-4 review: the concat dropped the
    positive media_time, so the priming frame played and the audio landed 1024 samples
    early)."""
    a = _audio_track(1.5, seed=13)
    a.media_time, a.delay = 1024, int(0.4 * a.timescale)
    t_first = a.pts_seconds()[1]          # the first presented frame: 0.4 s
    assert abs(t_first - 0.4) < 1e-9
    rt = mp4.read(mp4.write([a]))[0]
    assert rt.media_time == 1024 and abs(rt.delay - a.delay) <= 1 and rt.samples == a.samples
    bounds = [0.0, 0.25, 0.75, None]
    parts = [mp4.cut(a, bounds[i], bounds[i + 1]) for i in range(3)]
    assert not parts[0].samples
    assert parts[1].media_time == 1024 and parts[1].samples[0] == a.samples[0]
    assert abs(parts[1].pts_seconds()[1] - (0.4 - 0.25)) < 1e-3
    back = mp4.concat(parts, starts=[0.0, 0.25, 0.75])
    assert back.samples == a.samples and back.media_time == 1024
    assert abs(back.pts_seconds()[1] - 0.4) < 1e-3
    rt = mp4.read(mp4.write([back]))[0]
    assert rt.media_time == 1024 and abs(rt.pts_seconds()[1] - 0.4) < 1e-3


def test_split_worker_merge_keeps_audio(tmp_path, host):
    """server s (mp4 with audio) -> every piece carries its audio span -> worker transcode
    with -acodec copy -> merge: the output audio == the input audio, sample for sample."""
    from govideocompressor_amd.backends import PieceJob, get_backend
    from govideocompressor_amd.segment.merge import merge_files
    from govideocompressor_amd.segment.split import split
    es, clip = _h264_stream(host, frames=36, keyint=12)
    a = _audio_track(36 / 30.0 + 0.05, seed=9)
    a.media_time = 1024  # AAC encoder delay hidden by the edit list: kept through split and merge
    src = tmp_path / "movie.mp4"
    src.write_bytes(mp4.write([a, mp4.h264_track(es, 30.0)]))
    d, n = split(str(src), frames=12, out_root=str(tmp_path), log=lambda *_: None)
    assert n == 3
    pieces = [tmp_path / d / f"{i}.mp4" for i in range(n)]
    got = [mp4.audio_tracks(mp4.read(p.read_bytes())) for p in pieces]
    assert all(len(g) == 1 and g[0].samples for g in got)
    assert sum(len(g[0].samples) for g in got) == len(a.samples)
    be = get_backend("cpu")
    jobs = [PieceJob(str(i), str(p), str(tmp_path / f"o{i}.mp4")) for i, p in enumerate(pieces)]
    res = be.run(jobs, "-vcodec libx264 -crf 26 -acodec copy")
    be.close()
    assert all(r.ok for r in res), [r.reason for r in res]
    out = tmp_path / "merged.mp4"
    merge_files([j.out_path for j in jobs], str(out))
    tr = mp4.read(out.read_bytes())
    aud = mp4.audio_tracks(tr)
    assert len(aud) == 1 and aud[0].samples == a.samples and aud[0].sample_entry == a.sample_entry
    assert aud[0].media_time == 1024
    pics = host.decode(mp4.annexb_from_mp4(out.read_bytes()))
    assert len(pics) == 36
    # -an drops it
    res = get_backend("cpu").run([PieceJob("0", str(pieces[0]), str(tmp_path / "na.mp4"))], "-vcodec libx264 -an")
    assert res[0].ok and not mp4.audio_tracks(mp4.read((tmp_path / "na.mp4").read_bytes()))


def test_malformed_mp4_raises_valueerror():
    es = b"\x00\x00\x00\x18ftypisom\x00\x00\x02\x00isomiso2" + b"\x00\x00\x00\x10moov\x00\x00\x00\x08trak"
    with pytest.raises(ValueError):
        mp4.read(es)
    assert mp4.read(b"\x00\x00\x00\x08moov") == []
    with pytest.raises(ValueError):
        mp4.annexb_from_mp4(b"\x00\x00\x00\x08moov")
