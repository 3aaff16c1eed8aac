"""Backend-neutral piece handling: load a piece as frames, write the encoded result.

A *piece* is what the reference's worker downloads (``<idx>.mp4``, client.go:92-94)
and what ``convert`` turns into ``c<idx>.mp4`` (client.go:101-130).  A backend
receives a batch of :class:`PieceJob` and returns one :class:`PieceResult` each;
the GPU backend encodes the whole batch in one batched launch sequence.
"""
from __future__ import annotations

import json
import os
import time
from dataclasses import dataclass, field

import numpy as np

from ..jobs.ffargs import EncoderConfig
from ..segment.probe import annexb_of, kind_of
from ..utils import yuv


class BackendError(RuntimeError):
    """A piece-level failure whose message is sent back as ``fail;<idx>;<reason>``."""


@dataclass
class PieceJob:
    idx: str
    in_path: str
    out_path: str
    log_path: str | None = None


@dataclass
class PieceResult:
    idx: str
    ok: bool
    reason: str = ""
    stats: dict = field(default_factory=dict)


def load_clip(path: str) -> yuv.Clip:
    """Decode a piece to planar frames (raw pieces are read directly)."""
    kind = kind_of(path)
    if kind == "y4m":
        return yuv.read_y4m(path)
    if kind == "yuv":
        raise BackendError("raw .yuv pieces carry no geometry; split them to .y4m")
    try:
        return decode_stream_cpu(annexb_of(path, kind))
    except (RuntimeError, ValueError) as e:
        raise BackendError(f"{os.path.basename(path)}: {e}") from None


def decode_stream_cpu(stream: bytes, fps: float | None = None) -> yuv.Clip:
    """CPU decode of an Annex-B H.264 or HEVC stream (the independent decoders of
    csrc/host: h264_decoder.cc, hevc_dec.cc) into an 8-bit display-order clip."""
    from ..ops import native
    from ..segment.probe import codec_of
    h = native.host()
    if codec_of(stream) == "hevc":
        info = h.hevc_stream_info(stream)
        pics = sorted((p for p in h.hevc_decode_full(stream, True, False) if p["display"] >= 0),
                      key=lambda p: p["display"])
        if not pics:
            raise BackendError("no decodable pictures")
        p0 = pics[0]
        x0, y0, w, hh = p0["crop_x"], p0["crop_y"], p0["width"], p0["height"]
        sh = p0["bit_depth"] - 8
        ys = np.stack([(p["y"][y0:y0 + hh, x0:x0 + w] >> sh) for p in pics]).astype(np.uint8)
        us = np.stack([(p["u"][y0 // 2:(y0 + hh) // 2, x0 // 2:(x0 + w) // 2] >> sh) for p in pics]).astype(np.uint8)
        vs = np.stack([(p["v"][y0 // 2:(y0 + hh) // 2, x0 // 2:(x0 + w) // 2] >> sh) for p in pics]).astype(np.uint8)
        return yuv.Clip(ys, us, vs, fps or info["fps"] or 30.0)
    info = h.stream_info(stream)
    pics = h.decode(stream)
    if not pics:
        raise BackendError("no decodable pictures")
    w, hh = pics[0]["width"], pics[0]["height"]
    buf = np.concatenate([p["i420"] for p in pics])
    return yuv.Clip.from_i420(buf, w, hh, fps or info["fps"] or 30.0)


def output_size(cfg: EncoderConfig, clip: yuv.Clip) -> tuple[int, int]:
    if cfg.size:
        return cfg.size
    return clip.width, clip.height


def write_output(job: PieceJob, stream: bytes, fps: float, codec: str | None = None, audio: str = "copy") -> int:
    """Write an Annex-B stream as ``.mp4`` (``avc1`` with ctts for B pictures, ``hvc1`` for
    HEVC) or raw by extension.  ``codec`` ("h264" / "hevc", from the job's EncoderConfig)
    picks the sample entry; without it the stream's first NAL header decides.  With
    ``audio="copy"`` the input piece's audio tracks are stream-copied into the output
    (the reference's pieces keep their audio: server.go:199-200)."""
    from ..segment import mp4
    if not job.out_path.lower().endswith(".mp4"):
        data = stream
    else:
        extra = []
        if audio == "copy" and job.in_path.lower().endswith((".mp4", ".m4v", ".mov")):
            with open(job.in_path, "rb") as f:
                extra = mp4.file_audio(f.read())
        data = mp4.mux_video(stream, fps, codec, extra)
    tmp = job.out_path + ".part"
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, job.out_path)
    return len(data)


def write_log(job: PieceJob, stats: dict) -> None:
    """The per-piece log that replaces ffmpeg's stderr dump (``c<idx>.mp4.log``, client.go:120-127);
    written with truncation (fixes D12)."""
    if job.log_path:
        with open(job.log_path, "w") as f:
            json.dump(stats, f, indent=1, default=float)
            f.write("\n")


def unit_plan(n_frames: int, keyint: int | None) -> list[tuple[int, int]]:
    """Closed-GOP units of a piece: (start, count) with count <= keyint."""
    g = keyint if keyint and keyint > 0 else n_frames
    return [(s, min(g, n_frames - s)) for s in range(0, n_frames, g)]


def idr_id(piece_idx: str, unit: int) -> int:
    """idr_pic_id for unit ``unit`` of piece ``piece_idx``: consecutive IDR pictures differ
    inside a piece (alternating parity) and across the boundary of consecutive pieces
    (even base per piece), as 7.4.3 requires once the pieces are concatenated."""
    try:
        base = 2 * int(piece_idx)
    except ValueError:
        base = 0
    return (base + (unit & 1)) & 0xFFFF


class Timer:
    def __init__(self):
        self.t = {}

    def add(self, k: str, dt: float):
        self.t[k] = self.t.get(k, 0.0) + dt

    def span(self, k: str):
        tm = self

        class _S:
            def __enter__(self):
                self.t0 = time.perf_counter()

            def __exit__(self, *a):
                tm.add(k, time.perf_counter() - self.t0)
        return _S()
