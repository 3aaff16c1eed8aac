"""Raw video I/O: planar I420 (8-bit) / I420P10 (16-bit LE) files and YUV4MPEG2.

The reference never touches raw frames (ffmpeg does, client.go:115); here raw
YUV is a first-class input (BASELINE.json: "synthetic raw-YUV input") and the
splitter's piece format for raw sources is Y4M, which is self-describing, so a
worker needs no side channel to know a piece's geometry.
"""
from __future__ import annotations

import io
import os
from dataclasses import dataclass

import numpy as np


@dataclass
class Clip:
    """F frames of planar 4:2:0 video held as numpy arrays [F,H,W], [F,H/2,W/2] x2."""
    y: np.ndarray
    u: np.ndarray
    v: np.ndarray
    fps: float = 30.0

    @property
    def frames(self) -> int:
        return int(self.y.shape[0])

    @property
    def width(self) -> int:
        return int(self.y.shape[2])

    @property
    def height(self) -> int:
        return int(self.y.shape[1])

    @property
    def bit_depth(self) -> int:
        return 8 if self.y.dtype == np.uint8 else 10

    def slice(self, start: int, count: int) -> "Clip":
        return Clip(self.y[start:start + count], self.u[start:start + count], self.v[start:start + count], self.fps)

    def i420(self) -> np.ndarray:
        """Tightly packed frames (Y then U then V per frame), the CPU encoder's layout."""
        f = self.frames
        return np.concatenate([self.y.reshape(f, -1), self.u.reshape(f, -1), self.v.reshape(f, -1)], axis=1).reshape(-1)

    @staticmethod
    def from_i420(buf: np.ndarray | bytes, width: int, height: int, fps: float = 30.0, bit_depth: int = 8) -> "Clip":
        dt = np.uint8 if bit_depth == 8 else np.dtype("<u2")
        a = np.frombuffer(buf, dtype=dt) if isinstance(buf, (bytes, bytearray, memoryview)) else buf.view(dt)
        ys, cs = width * height, (width // 2) * (height // 2)
        fsz = ys + 2 * cs
        if a.size % fsz:
            raise ValueError(f"raw size {a.size} is not a multiple of the frame size {fsz}")
        f = a.size // fsz
        a = a.reshape(f, fsz)
        return Clip(a[:, :ys].reshape(f, height, width), a[:, ys:ys + cs].reshape(f, height // 2, width // 2),
                    a[:, ys + cs:].reshape(f, height // 2, width // 2), fps)


def to_8bit(x, bit_depth: int = 10):
    """High-bit-depth samples -> 8 bits with rounding (``(x + 2^(s-1)) >> s``, clipped), the
    conversion swscale applies for yuv420p10 -> yuv420p.  A plain ``x >> 2`` truncates and
    darkens the picture by half a level on average.  Works on numpy arrays and torch tensors."""
    s = int(bit_depth) - 8
    if s <= 0:
        return x
    try:
        import torch
        if isinstance(x, torch.Tensor):
            return ((x.to(torch.int32) + (1 << (s - 1))) >> s).clamp_(0, 255).to(torch.uint8)
    except ImportError:  # pragma: no cover
        pass
    a = np.asarray(x).astype(np.int32)
    return np.clip((a + (1 << (s - 1))) >> s, 0, 255).astype(np.uint8)


def rescale_bits(x, from_bd: int, to_bd: int = 10):
    """Samples of ``from_bd`` bits -> ``to_bd`` bits (both > 8, int16 planes): a left shift when
    widening, a rounded right shift (clipped) when narrowing -- e.g. 12-bit High 10-family input
    feeding the Main 10 encoder.  Works on numpy arrays and torch tensors."""
    s = int(from_bd) - int(to_bd)
    if s == 0:
        return x
    hi = (1 << int(to_bd)) - 1
    try:
        import torch
        if isinstance(x, torch.Tensor):
            if s < 0:
                return (x.to(torch.int32) << -s).to(torch.int16)
            return ((x.to(torch.int32) + (1 << (s - 1))) >> s).clamp_(0, hi).to(torch.int16)
    except ImportError:  # pragma: no cover
        pass
    a = np.asarray(x).astype(np.int32)
    if s < 0:
        return (a << -s).astype(np.int16)
    return np.clip((a + (1 << (s - 1))) >> s, 0, hi).astype(np.int16)


def frame_bytes(width: int, height: int, bit_depth: int = 8) -> int:
    return (width * height + 2 * (width // 2) * (height // 2)) * (1 if bit_depth == 8 else 2)


# --------------------------------------------------------------------------- Y4M
def _fps_from(tok: str) -> float:
    n, _, d = tok.partition(":")
    return float(n) / float(d or 1)


def _fps_to(fps: float) -> str:
    for den in (1, 1001):
        num = fps * den
        if abs(num - round(num)) < 1e-6:
            return f"{int(round(num))}:{den}"
    return f"{int(round(fps * 1000))}:1000"


@dataclass
class Y4mHeader:
    width: int
    height: int
    fps: float
    bit_depth: int
    header_len: int
    frame_len: int  # including the 'FRAME\n' marker

    def frames_in(self, nbytes: int) -> int:
        return max(0, (nbytes - self.header_len) // self.frame_len)


def parse_y4m_header(head: bytes) -> Y4mHeader:
    if not head.startswith(b"YUV4MPEG2"):
        raise ValueError("not a YUV4MPEG2 stream")
    nl = head.find(b"\n")
    if nl < 0:
        raise ValueError("truncated Y4M header")
    w = h = 0
    fps, depth = 30.0, 8
    for tok in head[:nl].decode().split()[1:]:
        k, val = tok[0], tok[1:]
        if k == "W":
            w = int(val)
        elif k == "H":
            h = int(val)
        elif k == "F":
            fps = _fps_from(val)
        elif k == "C":
            if not val.startswith("420"):
                raise ValueError(f"unsupported Y4M colour space C{val} (4:2:0 only)")
            if val.startswith("420p10"):
                depth = 10
    if w <= 0 or h <= 0:
        raise ValueError("Y4M header without W/H")
    return Y4mHeader(w, h, fps, depth, nl + 1, 6 + frame_bytes(w, h, depth))


def read_y4m(path_or_bytes, start: int = 0, count: int | None = None) -> Clip:
    data = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else None
    if data is None:
        with open(path_or_bytes, "rb") as f:
            hd = parse_y4m_header(f.read(256))
            total = hd.frames_in(os.fstat(f.fileno()).st_size)
            count = total - start if count is None else min(count, total - start)
            f.seek(hd.header_len + start * hd.frame_len)
            body = f.read(count * hd.frame_len)
    else:
        hd = parse_y4m_header(bytes(data[:256]))
        total = hd.frames_in(len(data))
        count = total - start if count is None else min(count, total - start)
        body = bytes(data[hd.header_len + start * hd.frame_len: hd.header_len + (start + count) * hd.frame_len])
    a = np.frombuffer(body, dtype=np.uint8).reshape(count, hd.frame_len)
    if count and not np.all(a[:, :6] == np.frombuffer(b"FRAME\n", dtype=np.uint8)):
        raise ValueError("Y4M frame marker missing (frame parameters are not supported)")
    raw = np.ascontiguousarray(a[:, 6:]).reshape(-1)
    return Clip.from_i420(raw, hd.width, hd.height, hd.fps, hd.bit_depth)


def y4m_bytes(clip: Clip) -> bytes:
    cs = "420p10" if clip.bit_depth == 10 else "420jpeg"
    out = io.BytesIO()
    out.write(f"YUV4MPEG2 W{clip.width} H{clip.height} F{_fps_to(clip.fps)} Ip A1:1 C{cs}\n".encode())
    for i in range(clip.frames):
        out.write(b"FRAME\n")
        for p in (clip.y, clip.u, clip.v):
            out.write(np.ascontiguousarray(p[i]).tobytes())
    return out.getvalue()


def write_y4m(path: str, clip: Clip) -> None:
    with open(path, "wb") as f:
        f.write(y4m_bytes(clip))


def read_yuv(path: str, width: int, height: int, fps: float = 30.0, bit_depth: int = 8,
             start: int = 0, count: int | None = None) -> Clip:
    fb = frame_bytes(width, height, bit_depth)
    total = os.path.getsize(path) // fb
    count = total - start if count is None else min(count, total - start)
    with open(path, "rb") as f:
        f.seek(start * fb)
        buf = f.read(count * fb)
    return Clip.from_i420(buf, width, height, fps, bit_depth)


def write_yuv(path: str, clip: Clip) -> None:
    with open(path, "wb") as f:
        f.write(clip.i420().tobytes())


def synth_clip_cpu(frames: int, width: int, height: int, seed: int = 0, fps: float = 30.0) -> Clip:
    """Deterministic moving-texture clip on the CPU (tests / no-GPU inputs).

    Not bit-identical to the gfx950 synth kernel; it only has to give the encoder
    realistic motion (a panning low-frequency texture plus a moving square)."""
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, size=(height // 8 + 4, width // 8 + 4)).astype(np.float32)
    big = np.kron(base, np.ones((8, 8), dtype=np.float32))
    k = np.array([1, 4, 6, 4, 1], dtype=np.float32) / 16.0
    for ax in (0, 1):
        big = np.apply_along_axis(lambda r: np.convolve(r, k, mode="same"), ax, big)
    y = np.empty((frames, height, width), dtype=np.uint8)
    u = np.empty((frames, height // 2, width // 2), dtype=np.uint8)
    v = np.empty_like(u)
    for t in range(frames):
        dx, dy = (t * 2) % 24, (t // 2) % 16
        fr = big[dy:dy + height, dx:dx + width].copy()
        sx, sy = (8 + 3 * t) % max(1, width - 16), (8 + 2 * t) % max(1, height - 16)
        fr[sy:sy + 16, sx:sx + 16] = 235.0
        fr += rng.normal(0.0, 1.0, size=fr.shape)
        y[t] = np.clip(fr, 16, 235).astype(np.uint8)
        cu = fr[::2, ::2] * 0.25 + 96.0
        u[t] = np.clip(cu, 16, 240).astype(np.uint8)
        v[t] = np.clip(255.0 - cu, 16, 240).astype(np.uint8)
    return Clip(y, u, v, fps)
