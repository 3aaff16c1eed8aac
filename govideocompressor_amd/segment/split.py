"""``server s``: cut a clip into independent pieces ``<dir>/<i>.<ext>``.

Reference (server.go:47-63, 193-204): ``dir = "12" + path`` with ``\\`` -> ``.``,
then ``ffmpeg -f segment -segment_time T -c copy -reset_timestamps 1`` writes
``dir/%d.mp4``; the piece count is ``fileCount(dir)``.

Here:

* compressed input (``.264`` / ``.265`` / ``.mp4`` with an H.264 or HEVC track): the
  native C++ splitter cuts at the first IDR access unit (HEVC: IDR / BLA / CRA without
  RASL pictures) at or after each ``T``-second boundary and re-emits the
  parameter sets at the head of every piece (the ``-reset_timestamps`` analogue);
  pieces keep the input's container (``.mp4`` via the native muxer, or ``.264``).
  No re-encode -- a stream copy, like ``-c copy``.
* raw input (``.yuv`` / ``.y4m``): frame-range pieces written as self-describing
  ``.y4m`` files (streamed, never the whole clip in memory).

Fixed defects: D16 (a path with ``/`` produced ``12dir/file`` -- the directory is
now ``12<basename>`` under ``out_root``), D3 (video-only input works), D1/D2 (no
division by zero / regex panic: see plan.py / probe.py).  A ``plan.json``
manifest records geometry and frame ranges for merge and resume.
"""
from __future__ import annotations

import json
import os
import re

from ..utils import yuv
from . import plan as P
from .probe import MediaInfo, annexb_of, probe, reference_seconds, split_stream, stream_frames

PIECE_RE = re.compile(r"^([+-]?[0-9]+)\.(mp4|264|h264|265|hevc|y4m)$")
CONTAINERS = ("mp4", "ts", "mkv")  # inputs whose pieces are written as MP4 (with their audio)
RAW_DEFAULT_SECONDS = 2.0


def split_dir_name(path: str) -> str:
    """The reference's ``"12" + path`` (``\\`` -> ``.``), applied to the file name only."""
    return "12" + os.path.basename(path.replace("\\", "."))


def piece_files(d: str) -> dict[str, str]:
    """idx token -> file name for every piece in a split directory."""
    out: dict[str, str] = {}
    if not os.path.isdir(d):
        return out
    for name in os.listdir(d):
        m = PIECE_RE.match(name)
        if m and os.path.isfile(os.path.join(d, name)):
            out.setdefault(m.group(1), name)
    return out


def file_count(d: str) -> int:
    """``fileCount``: recursive count of regular files (server.go:206-223), kept for parity;
    the coordinator itself enumerates actual piece names (fixes D8)."""
    n = 0
    for _, _, files in os.walk(d):
        n += len(files)
    return n


def split(path: str, size_mb: int = 10, seconds: float | None = None, frames: int | None = None,
          out_root: str = ".", width: int = 0, height: int = 0, fps: float = 30.0, bit_depth: int = 8,
          log=print) -> tuple[str, int]:
    """Returns (directory, number of pieces)."""
    info: MediaInfo = probe(path, width, height, fps, bit_depth)
    d = os.path.join(out_root, split_dir_name(path))
    os.makedirs(d, exist_ok=True)
    compressed = info.kind in ("h264", "hevc", *CONTAINERS)
    if frames:
        seg_frames = int(frames)
        seg_s = seg_frames / info.fps
    elif seconds:
        seg_s = float(seconds)
        seg_frames = P.frames_for_seconds(seg_s, info.fps)
    elif compressed:
        seg_s = P.reference_segment_seconds(size_mb, reference_seconds(info), info.bytes)
        seg_frames = P.frames_for_seconds(seg_s, info.fps)
    else:
        seg_s = RAW_DEFAULT_SECONDS
        seg_frames = P.frames_for_seconds(seg_s, info.fps)
    log(f"segment[{int(seg_s)}]s")
    log("split video....wait")
    ranges = []
    if compressed:
        from ..ops import native
        from . import mp4
        h = native.host()
        audio, pts = [], []
        if info.kind == "mp4":
            pieces = split_stream(annexb_of(path, info.kind), seg_frames)
            # -acodec copy -map 0:0 -map 0:1 (server.go:199-200): each piece carries the audio
            # samples of its own time span, cut at the video piece boundaries
            with open(path, "rb") as f:
                tracks = mp4.read(f.read())
            audio = mp4.audio_tracks(tracks)
            pts = mp4.video_track(tracks).pts_seconds()
        elif info.kind in ("ts", "mkv"):
            from .containers import demux
            dm = demux(path, info.kind)
            pieces = split_stream(dm.annexb, seg_frames)
            audio, pts = dm.audio, dm.pts
            for what in dm.dropped:
                log(f"note: {what} is not carried into the pieces")
        else:
            pieces = split_stream(annexb_of(path, info.kind), seg_frames)
        frames = [stream_frames(pc) for pc in pieces]
        starts = [sum(frames[:i]) for i in range(len(pieces))]
        for i, pc in enumerate(pieces):
            if info.kind in CONTAINERS:
                t0 = pts[starts[i]] if starts[i] < len(pts) else None
                t1 = pts[starts[i + 1]] if i + 1 < len(pieces) and starts[i + 1] < len(pts) else None
                extra = [mp4.cut(a, 0.0 if i == 0 else t0, t1) for a in audio] if t0 is not None else []
                name, data = f"{i}.mp4", mp4.mux_video(pc, info.fps, info.codec, [a for a in extra if a.samples])
            else:
                name, data = f"{i}.{'265' if info.codec == 'hevc' else '264'}", pc
            with open(os.path.join(d, name), "wb") as f:
                f.write(data)
            ranges.append({"idx": str(i), "file": name, "frames": frames[i]})
    else:
        pl = P.fixed_plan(info.frames, seg_frames)
        for i, (s, c, _) in enumerate(pl.tolist()):
            if info.kind == "y4m":
                clip = yuv.read_y4m(path, s, c)
            else:
                clip = yuv.read_yuv(path, info.width, info.height, info.fps, info.bit_depth, s, c)
            name = f"{i}.y4m"
            yuv.write_y4m(os.path.join(d, name), clip)
            ranges.append({"idx": str(i), "file": name, "start": s, "frames": c})
    manifest = {"source": os.path.abspath(path), "info": info.as_dict(), "segment_seconds": seg_s,
                "segment_frames": seg_frames, "pieces": ranges}
    with open(os.path.join(d, "plan.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    log(f"[{d}] [{len(ranges)}]")
    return d, len(ranges)
