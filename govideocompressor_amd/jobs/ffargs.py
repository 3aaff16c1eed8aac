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
(yuv420p, yuv420p10le), ``-preset`` (:mod:`..rc.presets`), ``-threads`` / ``-y`` /
``-an`` (accepted, no effect), ``-acodec copy`` / ``-c:a copy`` (audio passthrough: the
piece's audio track is copied into the output container), and the codec-tuning options,
each mapped onto encoder knobs (:data:`H264_PARAMS`, :data:`HEVC_PARAMS`):

* ``-profile:v`` -- H.264 ``baseline`` (Constrained Baseline: CAVLC, no B, no 8x8),
  ``main`` (CABAC + B, no 8x8 transform), ``high``; HEVC ``main``, ``main10``,
  ``mainstillpicture`` (intra only);
* ``-level`` -- written as level_idc; a picture size / rate above the level's limits is an
  error at encode time;
* ``-tune`` -- ``psnr`` (no AQ), ``zerolatency`` (no B pictures, no lookahead / MB-tree),
  ``fastdecode`` (H.264: CAVLC, no deblocking; HEVC: no deblocking, no SAO);
* ``-x264-params`` / ``-x265-params`` ``key=value:key=value`` -- the documented subset in
  :data:`H264_PARAMS` / :data:`HEVC_PARAMS`.

Anything else -- an unknown option, profile, tune or codec parameter, or a value the native
encoders cannot honour -- is an error reported back as ``fail;<idx>;<reason>`` rather
than silently ignored (reference defect D11: ffmpeg failures were only noticed at upload
time; SURVEY.md 5.6: unknown flags are hard errors).
"""
from __future__ import annotations

import re
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
    level: int | None = None        # level_idc (-level)
    profile: str | None = None      # -profile:v
    tune: str | None = None         # -tune
    # encoder knob overrides (H264Params / HevcParams field -> value) from -profile:v, -tune,
    # -x264-params / -x265-params, applied after the -preset table
    opts: dict = field(default_factory=dict)
    ignored: list[str] = field(default_factory=list)

    @property
    def bit_depth(self) -> int:
        return 10 if self.pix_fmt.endswith("10le") or self.pix_fmt.endswith("10") else 8

    def as_dict(self) -> dict:
        return dict(codec=self.codec, crf=self.crf, qp=self.qp, bitrate=self.bitrate, two_pass=self.two_pass,
                    size=self.size, fps=self.fps, keyint=self.keyint, pix_fmt=self.pix_fmt, preset=self.preset,
                    maxrate=self.maxrate, bufsize=self.bufsize, audio=self.audio, level=self.level,
                    profile=self.profile, tune=self.tune, opts=dict(self.opts))

    def apply_opts(self, params):
        """``params`` (H264Params / HevcParams, after the preset) with this config's knob
        overrides and level."""
        import dataclasses
        fields = {f.name for f in dataclasses.fields(params)}
        over = dict(self.opts)
        if self.level is not None:
            over["level_idc"] = self.level
        bad = sorted(k for k in over if k not in fields)
        if bad:
            raise FfArgsError(f"{type(params).__name__} has no knob(s) {', '.join(bad)}")
        if "direct" in fields:  # H.264: b-pyramid needs spatial direct prediction here
            if over.get("pyramid") and over.get("direct", "spatial") != "spatial":
                raise FfArgsError("b-pyramid needs direct=spatial with this encoder")
            if over.get("pyramid") and "direct" not in over:
                over.update(direct="spatial", spatial_wavefront=True)
            res = dataclasses.replace(params, **over)
            if res.pyramid and res.direct != "spatial":  # a preset's pyramid under direct=temporal
                res = dataclasses.replace(res, pyramid=False)
            return res
        return dataclasses.replace(params, **over)


def _flag(v: str) -> bool:
    if v in ("1", "true", "yes", "on", ""):
        return True
    if v in ("0", "false", "no", "off"):
        return False
    raise FfArgsError(f"expected a boolean, got {v!r}")


def _int_in(lo: int, hi: int):
    def conv(v: str) -> int:
        x = int(v)
        if not lo <= x <= hi:
            raise FfArgsError(f"value {x} outside {lo}..{hi}")
        return x
    return conv


def _float_in(lo: float, hi: float):
    def conv(v: str) -> float:
        x = float(v)
        if not lo <= x <= hi:
            raise FfArgsError(f"value {x} outside {lo}..{hi}")
        return x
    return conv


def _only(*allowed):
    def conv(v: str):
        if v not in allowed:
            raise FfArgsError(f"value {v!r} not supported (supported: {', '.join(allowed)})")
        return v
    return conv


def _aq_mode(v: str) -> float | None:
    m = int(v)
    if m == 0:
        return 0.0
    if m == 1:
        return None  # variance AQ at the configured strength
    raise FfArgsError(f"aq-mode {m}: only 0 (off) and 1 (variance AQ) are implemented")


def _subme(v: str) -> int:
    m = int(v)
    if m < 0 or m > 11:
        raise FfArgsError("subme in 0..11")
    return 0 if m == 0 else (1 if m == 1 else 2)


def _deblock(v: str) -> bool:
    # x264 / x265 "deblock=a,b" (offsets) or a boolean; only the default offsets 0,0
    if "," in v or re.fullmatch(r"-?\d+", v or "x") and v not in ("0", "1"):
        parts = [int(x) for x in v.split(",")]
        if any(parts):
            raise FfArgsError("deblock offsets other than 0,0 are not supported")
        return True
    return _flag(v)


def _partitions(v: str) -> bool:
    parts = set(v.split(","))
    if parts <= {"none"}:
        return False
    if parts <= {"p8x8", "i4x4", "i8x8", "b8x8", "all", "p4x4"} and "p4x4" not in parts:
        return True
    raise FfArgsError(f"partitions {v}: supported are none, p8x8/i4x4/i8x8/b8x8 combinations")


# -x264-params keys -> (H264Params field | EncoderConfig attribute prefixed '@', converter).
# A converter result of None leaves the field at its preset value.
H264_PARAMS = {
    "bframes": ("bframes", _int_in(0, 3)),
    "keyint": ("@keyint", _int_in(1, 100000)),
    "aq-mode": ("aq_strength", _aq_mode),
    "aq-strength": ("aq_strength", _float_in(0.0, 3.0)),
    "scenecut": ("scenecut", _int_in(0, 100)),
    "cabac": ("cabac", _flag),
    "no-cabac": ("cabac", lambda v: not _flag(v)),
    "8x8dct": ("t8x8", _flag),
    "no-8x8dct": ("t8x8", lambda v: not _flag(v)),
    "mbtree": ("mbtree", _flag),
    "no-mbtree": ("mbtree", lambda v: not _flag(v)),
    "rc-lookahead": ("lookahead", lambda v: int(v) > 0),
    "merange": ("me_range", _int_in(4, 16)),
    "subme": ("subpel", _subme),
    "deblock": ("deblock", _deblock),
    "no-deblock": ("deblock", lambda v: not _flag(v)),
    "partitions": ("partitions", _partitions),
    "ref": ("refs", _int_in(1, 4)),
    "weightp": ("weightp", lambda v: _int_in(0, 2)(v) > 0),
    "weightb": ("weightb", _flag),
    "no-weightb": ("weightb", lambda v: not _flag(v)),
    "trellis": ("trellis", lambda v: 2 if _int_in(0, 2)(v) > 0 else 0),
    # direct=spatial: decided in an MB wavefront (bframe.hip b_spatial_decide), -1.9 % BD-rate
    # and ~26 % fewer frames/s than temporal on the benchmark content (profiles/r3_direct_rd.md)
    "direct": ("direct", _only("temporal", "spatial")),
    "b-adapt": ("@b-adapt", _only("0")),
    # b-pyramid=normal: the middle B of a run is a reference; this encoder needs spatial direct
    # for it (decided in the MB wavefront), so it implies direct=spatial (apply_opts)
    "b-pyramid": ("pyramid", lambda v: _only("none", "normal")(v) == "normal"),
    "crf": ("@crf", _float_in(0.0, 51.0)),
    "qp": ("@qp", _int_in(0, 51)),
    "threads": ("@threads", int),
}
HEVC_PARAMS = {
    "bframes": ("bframes", _int_in(0, 8)),
    "b-pyramid": ("pyramid", _flag),
    "no-b-pyramid": ("pyramid", lambda v: not _flag(v)),
    "tmvp": ("tmvp", _flag),
    "no-tmvp": ("tmvp", lambda v: not _flag(v)),
    "keyint": ("@keyint", _int_in(1, 100000)),
    "aq-mode": ("aq_strength", _aq_mode),
    "aq-strength": ("aq_strength", _float_in(0.0, 3.0)),
    "cutree": ("cutree", _flag),
    "no-cutree": ("cutree", lambda v: not _flag(v)),
    "sao": ("sao", _flag),
    "no-sao": ("sao", lambda v: not _flag(v)),
    "wpp": ("wpp", _flag),
    "no-wpp": ("wpp", lambda v: not _flag(v)),
    "max-merge": ("max_merge", _int_in(1, 5)),
    "signhide": ("sdh", _flag),
    "no-signhide": ("sdh", lambda v: not _flag(v)),
    "tu-inter-depth": ("tu_inter_depth", lambda v: _int_in(1, 2)(v) - 1),
    "scenecut": ("scenecut", _int_in(0, 100)),
    "rc-lookahead": ("lookahead", lambda v: int(v) > 0),
    "merange": ("me_range", _int_in(4, 16)),
    "deblock": ("deblock", _deblock),
    "no-deblock": ("deblock", lambda v: not _flag(v)),
    "ctu": ("ctu64", lambda v: {"32": False, "64": True}[v] if v in ("32", "64") else _only("32 or 64")(v)),
    "ref": ("@ref", _int_in(1, 1)),
    "crf": ("@crf", _float_in(0.0, 51.0)),
    "qp": ("@qp", _int_in(0, 51)),
    "pools": ("@threads", str),
    "frame-threads": ("@threads", int),
}

_H264_PROFILES = {"baseline": dict(cabac=False), "main": dict(t8x8=False), "high": {}}
_HEVC_PROFILES = {"main": {}, "main10": {}, "mainstillpicture": dict(intra_only=True), "msp": dict(intra_only=True)}
_TUNES = {
    "h264": {"psnr": dict(aq_strength=0.0), "zerolatency": dict(bframes=0, lookahead=False, mbtree=False),
             "fastdecode": dict(cabac=False, deblock=False)},
    "hevc": {"psnr": dict(aq_strength=0.0), "zerolatency": dict(bframes=0, lookahead=False, cutree=False),
             "fastdecode": dict(deblock=False, sao=False)},
}


def _level(v: str) -> int:
    """"4.1" / "41" / "4" -> level_idc 41 (H.264 numbering; HEVC converts to 30 x level)."""
    try:
        x = float(v)
    except ValueError:
        raise FfArgsError(f"bad -level {v}") from None
    if x >= 10:
        x = x / 10.0
    if not 1.0 <= x <= 6.2:
        raise FfArgsError(f"-level {v} outside 1..6.2")
    return int(round(x * 10))


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
    codec_params: list[tuple[str, str]] = []  # (-x264-params | -x265-params, value), checked at the end
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
        elif t == "-preset":
            from ..rc import presets
            try:
                cfg.preset = presets.check(val())
            except presets.PresetError as e:
                raise FfArgsError(str(e)) from None
        elif t in ("-profile:v", "-profile", "-vprofile"):
            cfg.profile = val().lower()
        elif t == "-tune":
            cfg.tune = val().lower()
        elif t == "-level":
            cfg.level = _level(val())
        elif t in ("-x264-params", "-x265-params", "-x264opts"):
            codec_params.append((t, val()))
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
    crf_given |= _codec_options(cfg, codec_params)
    if cfg.codec == "hevc" and not crf_given and cfg.qp is None and cfg.bitrate is None:
        cfg.crf = 28.0  # x265 default CRF
    if cfg.two_pass and cfg.bitrate is None:
        raise FfArgsError("-pass needs a target bitrate (-b:v)")
    if (cfg.maxrate is None) != (cfg.bufsize is None):
        raise FfArgsError("-maxrate and -bufsize go together (VBV)")
    if cfg.bitrate is not None and cfg.bitrate <= 0:
        raise FfArgsError("-b:v must be positive")
    return cfg


def _codec_options(cfg: EncoderConfig, codec_params: list[tuple[str, str]]) -> bool:
    """-profile:v / -tune / -level / -x26x-params -> cfg.opts (and rate / GOP fields).
    Returns whether a codec parameter set the rate (crf / qp)."""
    codec = cfg.codec
    rate_set = False
    if codec == "copy":
        if cfg.profile or cfg.tune or cfg.level or codec_params:
            raise FfArgsError("codec options given with -vcodec copy")
        return False
    if cfg.profile is not None:
        table = _H264_PROFILES if codec == "h264" else _HEVC_PROFILES
        if cfg.profile not in table:
            raise FfArgsError(f"-profile:v {cfg.profile} is not supported for {codec} "
                              f"(supported: {', '.join(table)})")
        cfg.opts.update(table[cfg.profile])
        if codec == "hevc" and cfg.profile == "main" and cfg.bit_depth != 8:
            raise FfArgsError("-profile:v main needs 8-bit input (-pix_fmt yuv420p); use main10")
        if codec == "hevc" and cfg.profile == "main10":
            cfg.pix_fmt = "yuv420p10le"
    if cfg.tune is not None:
        for tn in cfg.tune.split(","):
            if tn not in _TUNES[codec]:
                raise FfArgsError(f"-tune {tn} is not supported for {codec} "
                                  f"(supported: {', '.join(_TUNES[codec])})")
            cfg.opts.update(_TUNES[codec][tn])
    if cfg.level is not None and codec == "hevc":
        cfg.level = cfg.level * 3  # general_level_idc = 30 x level
    for flag, text in codec_params:
        want = "-x265-params" if codec == "hevc" else "-x264-params"
        if flag != want and not (flag == "-x264opts" and codec == "h264"):
            raise FfArgsError(f"{flag} given for codec {codec}")
        table = HEVC_PARAMS if codec == "hevc" else H264_PARAMS
        for item in filter(None, text.split(":")):
            k, _, v = item.partition("=")
            k = k.strip().lower()
            if k not in table:
                raise FfArgsError(f"{flag} key {k!r} is not supported (supported: {', '.join(sorted(table))})")
            dest, conv = table[k]
            try:
                x = conv(v.strip())
            except FfArgsError as e:
                raise FfArgsError(f"{flag} {k}: {e}") from None
            except ValueError:
                raise FfArgsError(f"{flag} {k}: bad value {v!r}") from None
            if dest.startswith("@"):
                attr = dest[1:]
                if attr == "keyint":
                    cfg.keyint = x
                elif attr == "crf":
                    cfg.crf, cfg.qp, rate_set = x, None, True
                elif attr == "qp":
                    cfg.qp, cfg.crf, rate_set = x, None, True
                else:
                    cfg.ignored.append(f"{flag} {k}={v}")  # validated; value equal to what runs
            elif x is not None:
                cfg.opts[dest] = x
    # knob interactions the encoders would otherwise resolve silently
    if codec == "h264" and cfg.opts.get("cabac") is False:
        for k in ("bframes", "t8x8", "partitions"):
            if cfg.opts.get(k):
                raise FfArgsError(f"{k} needs CABAC (the CAVLC path is Constrained Baseline)")
    return rate_set
