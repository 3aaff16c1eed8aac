"""Encode backends used by the worker (backends/{gpu,ffmpeg_subprocess,cpu_ref}).

``get_backend("auto")`` picks the gfx950 encoder when a GPU is visible, else the
C++ reference encoder.  Every backend exposes ``run(jobs, args)`` taking the raw
ffmpeg-style argument string from the wire protocol.
"""
from __future__ import annotations

from ..jobs import ffargs
from .common import BackendError, PieceJob, PieceResult, load_clip


class _Adapter:
    def __init__(self, impl, raw_args: bool = False):
        self.impl = impl
        self.name = impl.name
        self.raw_args = raw_args

    def run(self, jobs: list[PieceJob], args: str) -> list[PieceResult]:
        if self.raw_args:
            return self.impl.transcode_args(jobs, args)
        try:
            cfg = ffargs.parse(args)
        except ffargs.FfArgsError as e:
            return [PieceResult(j.idx, False, str(e)) for j in jobs]
        return self.impl.transcode(jobs, cfg)

    def close(self):
        self.impl.close()


def get_backend(name: str = "auto", **kw) -> _Adapter:
    if name == "auto":
        import torch
        name = "gpu" if torch.cuda.is_available() else "cpu"
    if name == "gpu":
        from .gpu import GpuBackend
        return _Adapter(GpuBackend(**kw))
    if name == "cpu":
        from .cpu_ref import CpuBackend
        return _Adapter(CpuBackend(**kw))
    if name == "ffmpeg":
        from .ffmpeg_subprocess import FfmpegBackend
        return _Adapter(FfmpegBackend(**kw), raw_args=True)
    raise ValueError(f"unknown backend {name}")


__all__ = ["BackendError", "PieceJob", "PieceResult", "get_backend", "load_clip"]
