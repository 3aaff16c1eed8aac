"""``ffmpeg`` subprocess backend: the reference's exact worker behaviour, for hosts that
have the binary (config 1).  This image has none; tests put a fake ``ffmpeg`` on PATH.

Reference ``convert`` (client.go:101-130): argv = ``-i <idx>.mp4`` + args split on
single spaces + ``c<idx>.mp4``; stderr written to ``c<idx>.mp4.log``.  Fixed here:
the exit status is checked (D11), the log is truncated (D12), args are split with
shell-like quoting (D10).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shlex
import shutil
import subprocess

from ..jobs.ffargs import expand_preset
from .common import BackendError, PieceJob, PieceResult


class FfmpegBackend:
    name = "ffmpeg"

    def __init__(self, binary: str | None = None, threads: int = 1, timeout: float | None = None):
        self.bin = binary or shutil.which("ffmpeg")
        if not self.bin:
            raise BackendError("ffmpeg backend requested but no ffmpeg binary is on PATH")
        self.pool = cf.ThreadPoolExecutor(max_workers=max(1, threads))
        self.timeout = timeout

    def _one(self, j: PieceJob, args: str) -> PieceResult:
        argv = [self.bin, "-y", "-i", j.in_path] + shlex.split(expand_preset(args)) + [j.out_path]
        try:
            p = subprocess.run(argv, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=self.timeout)
        except subprocess.TimeoutExpired:
            return PieceResult(j.idx, False, "ffmpeg timed out")
        if j.log_path:
            with open(j.log_path, "wb") as f:
                f.write(p.stderr)
        if p.returncode != 0:
            tail = p.stderr.decode(errors="replace").strip().splitlines()[-1:] or [""]
            return PieceResult(j.idx, False, f"ffmpeg exit {p.returncode}: {tail[0][:120]}")
        if not os.path.exists(j.out_path):
            return PieceResult(j.idx, False, "ffmpeg produced no output")
        return PieceResult(j.idx, True, stats={"backend": "ffmpeg", "bytes": os.path.getsize(j.out_path)})

    def transcode_args(self, jobs: list[PieceJob], args: str) -> list[PieceResult]:
        return list(self.pool.map(lambda j: self._one(j, args), jobs))

    def close(self):
        self.pool.shutdown(wait=False)
