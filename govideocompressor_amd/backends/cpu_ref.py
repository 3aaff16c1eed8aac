"""CPU reference backend: the native C++ :class:`CpuEncoder` (csrc/host/cpu_encoder.cc).

Stands in for the reference's CPU ``ffmpeg -vcodec libx264`` (client.go:115) when
no GPU is present (config 1 plumbing, CPU-only tests of the job API).  Same
bitstream syntax and QP policy as the GPU encoder (I-frame QP = P QP - 3).
Pieces are encoded in parallel threads (the C++ encoder releases the GIL).
"""
from __future__ import annotations

import concurrent.futures as cf
import math
import os
import time

import numpy as np

from ..jobs.ffargs import EncoderConfig
from ..utils import yuv
from .common import BackendError, PieceJob, PieceResult, idr_id, load_clip, output_size, unit_plan, write_log, write_output


def resize_clip(clip: yuv.Clip, ow: int, oh: int) -> yuv.Clip:
    """Bicubic resample (swscale's default filter family), the GPU scaler's numpy model."""
    if (ow, oh) == (clip.width, clip.height):
        return clip
    from ..ops.scale import scale_plane_ref
    return yuv.Clip(scale_plane_ref(clip.y, ow, oh), scale_plane_ref(clip.u, ow // 2, oh // 2),
                    scale_plane_ref(clip.v, ow // 2, oh // 2), clip.fps)


class CpuBackend:
    name = "cpu"

    def __init__(self, threads: int | None = None):
        from ..ops import native
        self.host = native.host()
        self.pool = cf.ThreadPoolExecutor(max_workers=threads or min(8, os.cpu_count() or 2))

    def encode_clip(self, key: str, clip: yuv.Clip, cfg: EncoderConfig) -> tuple[bytes, dict]:
        t0 = time.perf_counter()
        ow, oh = output_size(cfg, clip)
        clip = resize_clip(clip, ow, oh)
        fps = cfg.fps or clip.fps
        qp = cfg.qp if cfg.qp is not None else int(round(cfg.crf if cfg.crf is not None else 23))

        def run(q: int):
            hcfg = dict(width=ow, height=oh, fps=fps, qp=max(0, min(51, q)), keyint=1 << 30,
                        level_idc=int(cfg.level or 0), deblock=int(cfg.opts.get("deblock", True)))
            parts, psnr = [], []
            for u, (s, c) in enumerate(unit_plan(clip.frames, cfg.keyint)):
                enc = self.host.CpuEncoder(hcfg)
                parts.append(enc.encode(clip.slice(s, c).i420(), c, idr_id(key, u)))
                psnr += [st["psnr_y"] for st in enc.stats()]
            return self.host.concat(parts), psnr

        stream, psnr = run(qp)
        if cfg.bitrate:  # ABR on the fixed-QP reference encoder: integer-QP secant search
            target = cfg.bitrate * clip.frames / fps
            tried = {qp: (stream, psnr)}
            for _ in range(4):
                bits = 8 * len(stream)
                nq = max(0, min(51, qp + int(round(6.0 * math.log2(max(bits, 1) / target)))))
                if nq in tried:
                    break
                qp = nq
                stream, psnr = run(qp)
                tried[qp] = (stream, psnr)
            qp = min(tried, key=lambda q: abs(8 * len(tried[q][0]) - target))
            stream, psnr = tried[qp]
        st = {"backend": "cpu", "idx": key, "frames": clip.frames, "width": ow, "height": oh, "fps": fps,
              "stream_bytes": len(stream), "psnr_y": float(np.mean(psnr)) if psnr else 0.0,
              "config": cfg.as_dict(), "seconds": time.perf_counter() - t0}
        return stream, st

    def encode_clips(self, items: list[tuple[str, yuv.Clip]], cfg: EncoderConfig) -> dict[str, tuple[bytes, dict]]:
        self._check(cfg)
        res = self.pool.map(lambda kc: self.encode_clip(kc[0], kc[1], cfg), items)
        return {k: r for (k, _), r in zip(items, res)}

    @staticmethod
    def _check(cfg: EncoderConfig):
        if cfg.codec != "h264":
            raise BackendError(f"codec {cfg.codec} is not available in the cpu backend")
        if cfg.bit_depth != 8:
            raise BackendError("10-bit output is not supported by the cpu backend")
        # the reference encoder is Constrained Baseline at a fixed QP: knobs it honours are
        # the Baseline profile itself, -level and deblocking; anything else is refused
        extra = {k: v for k, v in cfg.opts.items() if (k, v) not in (("cabac", False), ("bframes", 0)) and k != "deblock"}
        if extra:
            raise BackendError(f"the cpu reference backend (Constrained Baseline, fixed QP) cannot honour {extra}")

    def _one(self, j: PieceJob, cfg: EncoderConfig) -> PieceResult:
        try:
            clip = load_clip(j.in_path)
        except Exception as e:  # noqa: BLE001
            return PieceResult(j.idx, False, f"load: {e}")
        stream, st = self.encode_clip(j.idx, clip, cfg)
        st["bytes"] = write_output(j, stream, st["fps"], cfg.codec, cfg.audio)
        write_log(j, st)
        return PieceResult(j.idx, True, stats=st)

    def transcode(self, jobs: list[PieceJob], cfg: EncoderConfig) -> list[PieceResult]:
        try:
            self._check(cfg)
        except BackendError as e:
            return [PieceResult(j.idx, False, str(e)) for j in jobs]
        return list(self.pool.map(lambda j: self._one(j, cfg), jobs))

    def close(self):
        self.pool.shutdown(wait=False)
