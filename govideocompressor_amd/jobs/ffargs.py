"""Interpret the reference's ffmpeg argument strings as an encoder configuration.

The reference ships raw ffmpeg arguments to its workers (``-f`` flag,
server.go:29) with two shorthands (server.go:67-71):

    "265" -> "-threads 4 -vcodec libx265 -crf 26"
    "264" -> "-threads 4 -vcodec libx264"          (libx264 defaults: CRF 23)

and the worker splits them on single spaces (client.go:105).  Here the same
strings select the native codec and its rate control.  Supported subset:
``-vcodec/-c:v/-codec:v`` (libx264, h264, libx265, hevc, h265), ``-crf``,
``-qp``, ``-b:v`` (ABR, :mod:`..rc.abr`), ``-pass 1|2`` + ``-passlogfile``,
``-maxrate``/``-bufsize`` (VBV), ``-s WxH``, ``-r``, ``-g``, ``-pix_fmt``
(yuv420p, yuv420p10le), ``-preset`` (:mod:`..rc.presets`), ``-tune``,
``-profile:v`` (accepted), ``-threads`` / ``-y`` / ``-an`` (accepted, no effect),
``-acodec copy`` / ``-c:a copy`` (audio passthrough: the piece's audio track is
copied into the output container).
Anything else is an error reported back as ``fail;<idx>;<reason>`` rather than
silently ignored (reference defect D11: ffmpeg failures were only noticed at
upload time).
"""
from __future__ import annotations

import shlex
from dataclasses import dataclass, field

PRESETS = {
    "265": "-threads 4 -vcodec libx265 -crf 26",
    "264": "-threads 4 -vcodec libx264",
}

_CODECS = {"libx264": "h264", "h264": "h264", "avc": "h264", "libx265": "hevc", "hevc": "hevc", "h265": "hevc",
           "copy": "copy"}


class FfArgsError(ValueError):
    pass


@dataclass
class EncoderConfig:
    codec: str = "h264"
    crf: float | None = 23.0
    qp: int | None = None
    bitrate: int | None = None      # bits/s
    two_pass: int = 0               # 0: one pass, 1/2: pass index
    size: tuple[int, int] | None = None
    fps: float | None = None
    keyint: int | None = None
    pix_fmt: str = "yuv420p"
    preset: str = "medium"
    maxrate: int | None = None      # VBV, bits/s
    bufsize: int | None = None      # VBV, bits
    passlogfile: str | None = None
    audio: str = "copy"             # "copy" (ffmpeg's default for -acodec copy pieces) or "none" (-an)
    ignored: list[str] = field(default_factory=list)

    @property
    def bit_depth(self) -> int:
        return 10 if self.pix_fmt.endswith("10le") or self.pix_fmt.endswith("10") else 8

    def as_dict(self) -> dict:
        return dict(codec=self.codec, crf=self.crf, qp=self.qp, bitrate=self.bitrate, two_pass=self.two_pass,
                    size=self.size, fps=self.fps, keyint=self.keyint, pix_fmt=self.pix_fmt, preset=self.preset,
                    maxrate=self.maxrate, bufsize=self.bufsize, audio=self.audio)


def expand_preset(args: str) -> str:
    """The reference's ``-f 264`` / ``-f 265`` shorthands (server.go:67-71)."""
    return PRESETS.get(args.strip(), args)


def _bitrate(v: str) -> int:
    v = v.strip().lower()
    mul = 1
    if v.endswith("k"):
        mul, v = 1000, v[:-1]
    elif v.endswith("m"):
        mul, v = 1000_000, v[:-1]
    return int(float(v) * mul)


def parse(args: str) -> EncoderConfig:
    """Parse an ffmpeg-style argument string into an EncoderConfig."""
    try:
        return _parse(args)
    except FfArgsError:
        raise
    except ValueError as e:  # numeric conversions, shlex quoting
        raise FfArgsError(f"bad argument value: {e}") from None


def _parse(args: str) -> EncoderConfig:
    args = expand_preset(args)
    if not args.strip():
        # reference: empty args make every worker fail with "转换参数为空" (client.go:87-90)
        raise FfArgsError("conversion arguments are empty")
    toks = shlex.split(args)
    cfg = EncoderConfig()
    crf_given = False
    i = 0

    def val() -> str:
        nonlocal i
        if i + 1 >= len(toks):
            raise FfArgsError(f"option {toks[i]} needs a value")
        i += 1
        return toks[i]

    while i < len(toks):
        t = toks[i]
        if t in ("-vcodec", "-c:v", "-codec:v"):
            c = val().lower()
            if c not in _CODECS:
                raise FfArgsError(f"unsupported video codec {c}")
            cfg.codec = _CODECS[c]
        elif t == "-crf":
            cfg.crf = float(val())
            crf_given = True
        elif t == "-qp":
            cfg.qp = int(val())
            cfg.crf = None
        elif t == "-b:v":
            cfg.bitrate = _bitrate(val())
            if not crf_given:
                cfg.crf = None
        elif t == "-pass":
            cfg.two_pass = int(val())
            if cfg.two_pass not in (1, 2):
                raise FfArgsError("-pass must be 1 or 2")
        elif t == "-passlogfile":
            cfg.passlogfile = val()
        elif t == "-maxrate":
            cfg.maxrate = _bitrate(val())
        elif t == "-bufsize":
            cfg.bufsize = _bitrate(val())
        elif t == "-s":
            v = val().lower()
            try:
                w, h = v.split("x")
                cfg.size = (int(w), int(h))
            except ValueError as e:
                raise FfArgsError(f"bad -s value {v}") from e
            if cfg.size[0] % 2 or cfg.size[1] % 2:
                raise FfArgsError("-s dimensions must be even")
        elif t == "-r":
            cfg.fps = float(val())
        elif t == "-g":
            cfg.keyint = int(val())
        elif t == "-pix_fmt":
            pf = val()
            if pf not in ("yuv420p", "yuv420p10le"):
                raise FfArgsError(f"unsupported pixel format {pf}")
            cfg.pix_fmt = pf
        elif t in ("-preset", "-tune", "-profile:v", "-level", "-x264-params", "-x265-params"):
            v = val()
            if t == "-preset":
                from ..rc import presets
                try:
                    cfg.preset = presets.check(v)
                except presets.PresetError as e:
                    raise FfArgsError(str(e)) from None
            else:
                cfg.ignored.append(f"{t} {v}")
        elif t in ("-acodec", "-c:a", "-codec:a"):
            a = val().lower()
            if a != "copy":
                raise FfArgsError(f"audio codec {a}: only stream copy (-acodec copy) is supported")
            cfg.audio = "copy"
        elif t == "-an":
            cfg.audio = "none"
        elif t in ("-threads", "-ac", "-ar", "-b:a", "-map", "-f"):
            cfg.ignored.append(f"{t} {val()}")
        elif t in ("-y", "-n", "-hide_banner"):
            cfg.ignored.append(t)
        else:
            raise FfArgsError(f"unsupported option {t}")
        i += 1
    if cfg.codec == "hevc" and not crf_given and cfg.qp is None and cfg.bitrate is None:
        cfg.crf = 28.0  # x265 default CRF
    if cfg.two_pass and cfg.bitrate is None:
        raise FfArgsError("-pass needs a target bitrate (-b:v)")
    if (cfg.maxrate is None) != (cfg.bufsize is None):
        raise FfArgsError("-maxrate and -bufsize go together (VBV)")
    if cfg.bitrate is not None and cfg.bitrate <= 0:
        raise FfArgsError("-b:v must be positive")
    return cfg
