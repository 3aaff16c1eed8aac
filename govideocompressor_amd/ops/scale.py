"""Bicubic picture resampling (``-s WxH``) on gfx950 + its numpy golden model.

The reference's operators scale with ffmpeg's ``-s 1280x720`` (server.go:87-90), i.e.
swscale's default SWS_BICUBIC: the Mitchell-Netravali cubic with B = 0, C = 0.6, support
widened by the downscale ratio (``taps = 4 * ceil(in / out)``), coefficients normalised
per output sample and quantised to 14 bits.  :func:`taps` builds those tables once per
geometry (host); ``csrc/kernels/scale.hip`` runs the separable LDS-tiled filter; and
:func:`scale_plane_ref` is the same integer arithmetic in numpy (the bit-exact oracle of
``tests/test_gpu_scale.py``).  Exact parity with swscale's own rounding is unpinned (no
ffmpeg in this image); the filter family and support match.

Also: :func:`rgb_to_i420` (packed RGB24 -> I420, BT.601 limited range) on the GPU.
"""
from __future__ import annotations

import math

import numpy as np

COEF_BITS = 14
B_PARAM, C_PARAM = 0.0, 0.6


def cubic(x: np.ndarray, B: float = B_PARAM, C: float = C_PARAM) -> np.ndarray:
    x = np.abs(x)
    w = np.zeros_like(x)
    a = x < 1
    b = (x >= 1) & (x < 2)
    w[a] = ((12 - 9 * B - 6 * C) * x[a] ** 3 + (-18 + 12 * B + 6 * C) * x[a] ** 2 + (6 - 2 * B)) / 6
    w[b] = ((-B - 6 * C) * x[b] ** 3 + (6 * B + 30 * C) * x[b] ** 2 + (-12 * B - 48 * C) * x[b] + (8 * B + 24 * C)) / 6
    return w


def taps(n_in: int, n_out: int) -> tuple[np.ndarray, np.ndarray]:
    """(first input index [n_out] int32, coefficients [n_out, T] int16 summing to 2^14)."""
    s = max(1.0, n_in / n_out)
    T = 4 * int(math.ceil(s))
    centre = (np.arange(n_out) + 0.5) * n_in / n_out - 0.5
    first = np.floor(centre).astype(np.int64) - T // 2 + 1
    pos = first[:, None] + np.arange(T)[None, :]
    w = cubic((pos - centre[:, None]) / s)
    w /= w.sum(axis=1, keepdims=True)
    q = np.round(w * (1 << COEF_BITS)).astype(np.int64)
    fix = (1 << COEF_BITS) - q.sum(axis=1)
    q[np.arange(n_out), np.argmax(w, axis=1)] += fix  # exact unit gain
    return first.astype(np.int32), q.astype(np.int16)


def scale_plane_ref(p: np.ndarray, ow: int, oh: int, bd: int = 8) -> np.ndarray:
    """Golden model: [N, h, w] (uint8 / uint16) -> [N, oh, ow], the kernel's integer math."""
    N, h, w = p.shape
    fx, cx = taps(w, ow)
    fy, cy = taps(h, oh)
    xs = np.clip(fx[:, None] + np.arange(cx.shape[1])[None, :], 0, w - 1)
    ys = np.clip(fy[:, None] + np.arange(cy.shape[1])[None, :], 0, h - 1)
    q = p.astype(np.int64)
    sh = bd - 1
    hor = (np.einsum("nyxk,xk->nyx", q[:, :, xs], cx.astype(np.int64)) + (1 << (sh - 1))) >> sh  # [N, h, ow]
    sv = 29 - bd
    ver = np.einsum("nyxk,yk->nyx", hor[:, ys, :].transpose(0, 1, 3, 2), cy.astype(np.int64))  # [N, oh, ow]
    out = np.clip((ver + (1 << (sv - 1))) >> sv, 0, (1 << bd) - 1)
    return out.astype(p.dtype)


class GpuScaler:
    """Device tables per geometry + launches of ``scale.hip``."""

    def __init__(self, device):
        import torch

        from . import native
        self.torch = torch
        self.dev = torch.device(device)
        self.hip = native.hip()
        self._tabs: dict[tuple[int, int], tuple] = {}

    def _tab(self, n_in: int, n_out: int):
        k = (n_in, n_out)
        if k not in self._tabs:
            f, c = taps(n_in, n_out)
            T = self.torch
            self._tabs[k] = (T.from_numpy(f).to(self.dev), T.from_numpy(np.ascontiguousarray(c)).to(self.dev), c.shape[1])
        return self._tabs[k]

    def plane(self, src, ow: int, oh: int, bd: int = 8, out=None, W: int | None = None, H: int | None = None):
        """src: [N, h, w] uint8 (bd 8) or int16 holding 10-bit samples -> [N, H, W] (default
        [N, oh, ow]; columns / rows past ow / oh replicate the edge)."""
        T = self.torch
        N, h, w = src.shape
        W, H = W or ow, H or oh
        if out is None:
            out = T.empty((N, H, W), dtype=src.dtype, device=self.dev)
        fx, cx, tx = self._tab(w, ow)
        fy, cy, ty = self._tab(h, oh)
        tw, th = 64, 32
        while True:
            in_cols = int(math.ceil(tw * w / ow)) + tx + 2
            in_rows = int(math.ceil(th * h / oh)) + ty + 2
            lds = ((in_rows * in_cols + 1) // 2) * 4 + in_rows * tw * 4
            if lds <= 48 * 1024 or (tw <= 8 and th <= 8):
                break
            if tw >= th:
                tw //= 2
            else:
                th //= 2
        rc = self.hip.scale(src.data_ptr(), w, h, src.stride(0), src.stride(1), out.data_ptr(), ow, oh, W, H,
                            out.stride(0), out.stride(1), N, fx.data_ptr(), cx.data_ptr(), tx, fy.data_ptr(),
                            cy.data_ptr(), ty, tw, th, in_cols, in_rows, bd, T.cuda.current_stream(self.dev).cuda_stream)
        if rc != 0:
            raise RuntimeError("scale: filter footprint does not fit LDS (downscale ratio too large)")
        return out

    def clip(self, y, u, v, ow: int, oh: int, bd: int = 8):
        """[B, F, h, w] planes (+ half-size chroma) -> scaled [B, F, oh, ow] planes."""
        B, F = y.shape[0], y.shape[1]
        flat = lambda t: t.reshape(B * F, t.shape[2], t.shape[3])  # noqa: E731
        ys = self.plane(flat(y), ow, oh, bd).reshape(B, F, oh, ow)
        us = self.plane(flat(u), ow // 2, oh // 2, bd).reshape(B, F, oh // 2, ow // 2)
        vs = self.plane(flat(v), ow // 2, oh // 2, bd).reshape(B, F, oh // 2, ow // 2)
        return ys, us, vs


def rgb_to_i420(rgb):
    """[N, h, w, 3] uint8 RGB24 on the device -> (y, u, v) I420 planes (BT.601 limited)."""
    import torch

    from . import native
    N, h, w, _ = rgb.shape
    if w % 2 or h % 2:
        raise ValueError("RGB frames need even width and height")
    rgb = rgb.contiguous()
    y = torch.empty((N, h, w), dtype=torch.uint8, device=rgb.device)
    u = torch.empty((N, h // 2, w // 2), dtype=torch.uint8, device=rgb.device)
    v = torch.empty_like(u)
    native.hip().rgb_to_i420(rgb.data_ptr(), w, h, N, y.data_ptr(), u.data_ptr(), v.data_ptr(),
                             torch.cuda.current_stream(rgb.device).cuda_stream)
    return y, u, v


def rgb_to_i420_ref(rgb: np.ndarray):
    """numpy model of the RGB -> I420 kernel (float BT.601, 2x2 chroma average)."""
    f = rgb.astype(np.float32)
    r, g, b = f[..., 0], f[..., 1], f[..., 2]
    y = 16.0 + 0.257 * r + 0.504 * g + 0.098 * b
    cu = 128.0 - 0.148 * r - 0.291 * g + 0.439 * b
    cv = 128.0 + 0.439 * r - 0.368 * g - 0.071 * b
    N, h, w = y.shape
    pool = lambda c: c.reshape(N, h // 2, 2, w // 2, 2).sum(axis=(2, 4)) * 0.25  # noqa: E731
    q = lambda c: np.clip(np.floor(c + 0.5), 0, 255).astype(np.uint8)  # noqa: E731
    return q(y), q(pool(cu)), q(pool(cv))
