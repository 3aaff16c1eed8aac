"""Merge encoded pieces back into one stream (the reference's concat step).

Reference: ``makeFileList`` writes ``filelist.txt`` with ``file '<i>.mp4'``
lines, only if absent (server.go:325-347); ``makeConcatScript`` writes
``concat.sh`` = ``ffmpeg -f concat -i filelist.txt -c copy output.mp4``, only if
absent, mode 0755 (server.go:349-361); the operator runs it by hand.

Here the concatenation is native (C++ Annex-B concat + MP4 remux): every piece
is a closed GOP that starts with SPS/PPS + IDR, so an ordered byte concat is a
conformant stream.  ``concat.sh`` is still emitted for operator parity, but it
calls this module instead of ffmpeg.
"""
from __future__ import annotations

import os
import re
import sys

from ..ops import native
from . import mp4, mp4_hevc

_LINE = re.compile(r"^\s*file\s+'([^']+)'\s*$")


def make_filelist(pieces: int | list[str], d: str, ext: str = "mp4") -> str:
    """``pieces``: a count (the reference's 0..n-1) or the piece index tokens in order."""
    p = os.path.join(d, "filelist.txt")
    names = [str(i) for i in range(pieces)] if isinstance(pieces, int) else list(pieces)
    if not os.path.exists(p):
        with open(p, "w") as f:
            for i in names:
                f.write(f"file '{i}.{ext}'\n")
    return p


def make_concat_script(d: str) -> str:
    p = os.path.join(d, "concat.sh")
    if not os.path.exists(p):
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        with open(p, "w") as f:
            f.write("#!/bin/sh\ncd \"$(dirname \"$0\")\" && "
                    f"PYTHONPATH=\"{root}${{PYTHONPATH:+:$PYTHONPATH}}\" "
                    f"{sys.executable or 'python3'} -m govideocompressor_amd.cli merge "
                    "--list filelist.txt -o output.mp4\n")
        os.chmod(p, 0o755)
    return p


def read_filelist(path: str) -> list[str]:
    base = os.path.dirname(os.path.abspath(path))
    out = []
    with open(path) as f:
        for line in f:
            if not line.strip() or line.lstrip().startswith("#"):
                continue
            m = _LINE.match(line)
            if not m:
                raise ValueError(f"bad filelist line: {line.rstrip()}")
            out.append(os.path.join(base, m.group(1)))
    return out


def load_annexb(path: str) -> bytes:
    with open(path, "rb") as f:
        data = f.read()
    if mp4.is_mp4(data) or path.lower().endswith((".mp4", ".m4v", ".mov")):
        return mp4.annexb_from_mp4(data)
    return data


def load_audio(path: str) -> list:
    """The audio tracks of an MP4 piece (none for Annex-B pieces)."""
    with open(path, "rb") as f:
        head = f.read(8)
    if not (mp4.is_mp4(head) or path.lower().endswith((".mp4", ".m4v", ".mov"))):
        return []
    with open(path, "rb") as f:
        return mp4.file_audio(f.read())


def piece_fps(path: str) -> float | None:
    """Frame rate recorded in an MP4 piece (mdhd / stts), None for Annex-B pieces."""
    with open(path, "rb") as f:
        data = f.read()
    if data[4:8] != b"ftyp" and not path.lower().endswith((".mp4", ".m4v", ".mov")):
        return None
    return mp4_hevc.track_fps(data)


def merge_files(files: list[str], out_path: str, fps: float | None = None) -> int:
    """Concatenate pieces in order into ``out_path`` (.mp4 -> MP4 mux, otherwise Annex-B).
    Every piece must carry the same codec.  Returns the number of bytes written."""
    missing = [f for f in files if not os.path.exists(f)]
    if missing:
        raise FileNotFoundError(f"missing pieces: {missing[:5]}{'...' if len(missing) > 5 else ''}")
    h = native.host()
    parts = [load_annexb(f) for f in files]
    codecs = {("hevc" if mp4_hevc.is_hevc_annexb(p) else "h264") for p in parts if p}
    if len(codecs) > 1:
        raise ValueError(f"pieces mix codecs {sorted(codecs)}: re-encode them with one -vcodec")
    stream = h.concat(parts)
    if out_path.lower().endswith((".mp4", ".m4v", ".mov")):
        hevc = mp4_hevc.is_hevc_annexb(stream)
        if fps is None and files:
            # the HEVC SPS carries no timing: take the pieces' own MP4 rate
            fps = piece_fps(files[0])
        if fps is None and not hevc:
            fps = h.stream_info(stream)["fps"] or None
        # audio: every piece's track(s) appended in piece order (concat.sh -c copy keeps
        # them, server.go:357); pieces without audio contribute nothing
        audio = [load_audio(f) for f in files]
        extra = []
        if any(audio):
            n = max(len(a) for a in audio)
            # piece start times: an audio track that begins in a later piece keeps its delay
            nfr = [h.hevc_stream_info(p)["frames"] if mp4_hevc.is_hevc_annexb(p) else h.stream_info(p)["frames"]
                   for p in parts]
            t_of = [sum(nfr[:i]) / (fps or 30.0) for i in range(len(parts))]
            for k in range(n):
                idx = [i for i, a in enumerate(audio) if len(a) > k]
                extra.append(mp4.concat([audio[i][k] for i in idx], [t_of[i] for i in idx]))
        data = mp4.mux_video(stream, fps or 30.0, "hevc" if hevc else "h264", extra)
    else:
        data = stream
    tmp = out_path + ".part"
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, out_path)
    return len(data)


def merge_dir(d: str, out_name: str = "output.mp4") -> str:
    files = read_filelist(os.path.join(d, "filelist.txt"))
    out = os.path.join(d, out_name)
    merge_files(files, out)
    return out
