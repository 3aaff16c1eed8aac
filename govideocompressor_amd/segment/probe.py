"""Container / stream probe (the reference's ``GetSumTime``, server.go:239-265).

The reference runs ``ffmpeg -i <file>``, regex-matches ``Duration: HH:MM:SS``
from stderr and returns ``h*3600 + m*60 + s + 1`` -- fractional seconds are
dropped and one second is added (server.go:262).  When the regex does not match
it panics on an empty slice (defect D2).  Here the duration comes from the
stream itself:

* raw ``.yuv``  -- geometry/fps/bit depth given by the caller, frames = size / frame bytes
* ``.y4m``      -- header (W, H, F, C)
* ``.264/.h264`` Annex-B -- SPS (geometry, VUI timing) + access-unit count (C++ probe)
* ``.265/.hevc`` Annex-B -- HEVC SPS (geometry, bit depth, VUI timing) + picture count
  (csrc/host/hevc_dec_ps.cc)
* ``.mp4``      -- demuxed by the native ISO-BMFF reader (``avc1`` or ``hvc1``/``hev1``
  track), then as Annex-B
* ``.ts`` / ``.m2ts`` (MPEG-TS) and ``.mkv`` / ``.webm`` (Matroska) -- demuxed by
  ``segment/containers.py`` (H.264 / HEVC video, AAC audio), then as Annex-B

and :func:`reference_seconds` reproduces the reference's integer arithmetic.
"""
from __future__ import annotations

import os
import struct
from dataclasses import asdict, dataclass

from ..utils import yuv


class ProbeError(ValueError):
    pass


@dataclass
class MediaInfo:
    path: str
    kind: str           # yuv | y4m | h264 | hevc | mp4 | ts | mkv
    width: int
    height: int
    fps: float
    frames: int
    bit_depth: int = 8
    bytes: int = 0
    idr_frames: int = 0
    entropy: str = ""   # cavlc | cabac for compressed inputs
    profile_idc: int = 0
    codec: str = "raw"  # raw | h264 | hevc (the compressed stream's codec)

    @property
    def duration_s(self) -> float:
        return self.frames / self.fps if self.fps > 0 else 0.0

    def as_dict(self) -> dict:
        d = asdict(self)
        d["duration_s"] = self.duration_s
        return d


def kind_of(path: str) -> str:
    ext = os.path.splitext(path)[1].lower()
    if ext in (".yuv", ".i420", ".raw"):
        return "yuv"
    if ext == ".y4m":
        return "y4m"
    if ext in (".264", ".h264", ".avc", ".bin"):
        return "h264"
    if ext in (".265", ".h265", ".hevc"):
        return "hevc"
    if ext in (".mp4", ".m4v", ".mov"):
        return "mp4"
    if ext in (".ts", ".m2ts", ".mts", ".m2t"):
        return "ts"
    if ext in (".mkv", ".webm", ".mk3d"):
        return "mkv"
    # sniff
    with open(path, "rb") as f:
        head = f.read(189)
    from .containers import is_mkv, is_ts
    if is_ts(head):
        return "ts"
    if is_mkv(head):
        return "mkv"
    if head.startswith(b"YUV4MPEG2"):
        return "y4m"
    if head[:4] in (b"\x00\x00\x00\x01",) or head[:3] == b"\x00\x00\x01":
        from .mp4_hevc import is_hevc_annexb
        return "hevc" if is_hevc_annexb(head) else "h264"
    if head[4:8] == b"ftyp":
        return "mp4"
    raise ProbeError(f"cannot tell the container of {path}; use .yuv/.y4m/.264/.265/.mp4/.ts/.mkv")


def codec_of(stream: bytes) -> str:
    """Codec of an Annex-B stream from its first NAL header: "hevc" or "h264"."""
    from .mp4_hevc import is_hevc_annexb
    return "hevc" if is_hevc_annexb(stream) else "h264"



def annexb_of(path: str, kind: str | None = None) -> bytes:
    from ..ops import native
    kind = kind or kind_of(path)
    with open(path, "rb") as f:
        data = f.read()
    if kind == "mp4":
        from . import mp4
        try:
            return mp4.annexb_from_mp4(data)  # the video trak, wherever it sits among the tracks
        except ValueError as e:
            raise ProbeError(f"{path}: {e}") from None
    if kind in ("h264", "hevc"):
        return data
    if kind in ("ts", "mkv"):
        from .containers import demux
        try:
            return demux(data, kind).annexb
        except (ValueError, IndexError, struct.error) as e:
            raise ProbeError(f"{path}: {e}") from None
    raise ProbeError(f"{path} is not a compressed stream")


def probe(path: str, width: int = 0, height: int = 0, fps: float = 30.0, bit_depth: int = 8) -> MediaInfo:
    if not os.path.isfile(path):
        raise ProbeError(f"no such file: {path}")
    size = os.path.getsize(path)
    kind = kind_of(path)
    if kind == "yuv":
        if width <= 0 or height <= 0:
            raise ProbeError("raw .yuv input needs its geometry (--size WxH)")
        fb = yuv.frame_bytes(width, height, bit_depth)
        return MediaInfo(path, kind, width, height, fps, size // fb, bit_depth, size)
    if kind == "y4m":
        with open(path, "rb") as f:
            hd = yuv.parse_y4m_header(f.read(256))
        return MediaInfo(path, kind, hd.width, hd.height, hd.fps, hd.frames_in(size), hd.bit_depth, size)
    from ..ops import native
    stream = annexb_of(path, kind)
    if codec_of(stream) == "hevc":
        try:
            hi = native.host().hevc_stream_info(stream)
        except RuntimeError as e:
            raise ProbeError(f"{path}: {e}") from None
        if hi["width"] <= 0:
            raise ProbeError(f"{path}: no HEVC sequence parameter set found")
        return MediaInfo(path, kind, hi["width"], hi["height"], hi["fps"] or fps, hi["frames"], hi["bit_depth"], size,
                         hi["irap_frames"], "cabac", 0, "hevc")
    info = native.host().stream_info(stream)
    if info["width"] <= 0:
        raise ProbeError(f"{path}: no H.264 sequence parameter set found")
    return MediaInfo(path, kind, info["width"], info["height"], info["fps"] or fps, info["frames"], 8, size,
                     info["idr_frames"], info["entropy"], info["profile_idc"], "h264")


def split_stream(stream: bytes, min_frames: int) -> list[bytes]:
    """Keyframe-aligned pieces of an Annex-B stream (H.264: at IDR access units; HEVC: at
    IDR / BLA / CRA-without-RASL access units), parameter sets re-emitted per piece."""
    from ..ops import native
    h = native.host()
    if codec_of(stream) == "hevc":
        return h.hevc_split_pieces(stream, min_frames)
    return h.split_pieces(stream, min_frames)


def stream_frames(stream: bytes) -> int:
    from ..ops import native
    h = native.host()
    if codec_of(stream) == "hevc":
        return h.hevc_stream_info(stream)["frames"]
    return h.stream_info(stream)["frames"]


def reference_seconds(info: MediaInfo) -> int:
    """``GetSumTime``: whole seconds of the Duration line, plus one (server.go:250-262)."""
    return int(info.duration_s) + 1
