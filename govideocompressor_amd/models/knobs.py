"""Environment knobs: the one place that maps ``MIVC_*`` variables onto encoder settings.

Until round 4 about 25 ``H264Params`` defaults were read from ``MIVC_*`` variables at import
time, so a stray variable silently changed the encoder behind a bench line that claimed the
default configuration (round-4 review).  Now the dataclass defaults are constants; the
variables below are applied only by entry points that ask for them
(:func:`encoder_overrides`: ``bench.py --allow-knobs``, ``bench/run.py --allow-knobs``, the
tools/gpu sweep scripts), and :func:`check_environment` refuses

* any ``MIVC_*`` name that is not listed here (a typo would otherwise be a silent no-op), and
* an encoder knob when the caller did not allow knobs.

``RUNTIME`` variables change scheduling, resources, logging or the job plumbing, never the
coded bytes (the CABAC coder grouping and pool sizes, the intra wavefront's workgroup size,
pinned-memory budget, entropy threads: the GPU tests assert byte identity across them), so
they are always allowed; bench.py reports every one that is set.

Reference parity: the reference's only encoder configuration is the ffmpeg argument string
(``-f 264|265|args``, server.go:65-71); these knobs are development settings of this encoder
(x264's ``--b-adapt``, ``--trellis``, ... equivalents), not part of the job API.
"""
from __future__ import annotations

import dataclasses
import os

# env name -> H264Params field
H264 = {
    "MIVC_I8X8": "i8x8",
    "MIVC_I4X4_IN_P": "i4x4_in_p",
    "MIVC_LA_RANGE": "la_range",
    "MIVC_LA_WEIGHTS": "la_weights",
    "MIVC_B_ADAPT": "b_adapt",
    "MIVC_B_BIAS": "b_bias",
    "MIVC_BADAPT_GUARD": "badapt_guard",
    "MIVC_BADAPT_SHARED": "badapt_shared",
    "MIVC_BADAPT_RANGE": "badapt_range",
    "MIVC_LA_SEED": "lowres_seed",
    "MIVC_B_ME_RANGE": "b_me_range",
    "MIVC_SKIP_REFINE": "skip_refine",
    "MIVC_REFINE_SKIP": "refine_skip",
    "MIVC_BPARTS": "bpartitions",
    "MIVC_PART_OVERHEAD": "part_overhead",
    "MIVC_PART_MIN_SATD": "part_min_satd",
    "MIVC_P_EARLY_SAD": "p_early_sad",
    "MIVC_B_EARLY_SAD": "b_early_sad",
    "MIVC_B_GATE": "b_gate",
    "MIVC_TRELLIS": "trellis",
    "MIVC_DIRECT": "direct",
    "MIVC_DIRECT_BIAS": "direct_bias",
    "MIVC_SPATIAL_GATE": "spatial_gate",
    "MIVC_SPATIAL_WAVEFRONT": "spatial_wavefront",
    "MIVC_SPATIAL_FIX_TOL": "spatial_fix_tol",
    "MIVC_TDIRECT_BIAS": "tdirect_bias",
    "MIVC_PYRAMID": "pyramid",
    "MIVC_TRELLIS_LAMBDA": "trellis_lambda",
    "MIVC_INTRA_TRELLIS": "intra_trellis",
    "MIVC_REFS": "refs",
    "MIVC_REF_RANGE": "ref_range",
    "MIVC_REF_GATE": "ref_gate",
    "MIVC_SLICES": "slices",
}
# env name -> HevcParams field
HEVC = {
    "MIVC_HEVC_CTU64": "ctu64",
    "MIVC_HEVC_LA_WEIGHTS": "la_weights",
    "MIVC_HEVC_MERGE_SKIP": "merge_skip",
    "MIVC_HEVC_REFS": "refs",
    "MIVC_HEVC_REF_GATE": "ref_gate",
    "MIVC_HEVC_REF_RANGE": "ref_range",
    "MIVC_HEVC_BFRAMES": "bframes",
    "MIVC_HEVC_INTER8": "inter8",
    "MIVC_HEVC_INTER8_OVERHEAD": "inter8_overhead",
    "MIVC_HEVC_TU_INTER_DEPTH": "tu_inter_depth",
    "MIVC_HEVC_SDH": "sdh",
}
# bench.py shape knobs (they change what is measured, so they also need --allow-knobs)
# (MIVC_HIP_LIB: an alternative kernel library, tools/build_variant.py -- same-box A/B timing)
BENCH = {"MIVC_BENCH_SLOTS", "MIVC_BENCH_FRAMES", "MIVC_BENCH_BFRAMES", "MIVC_HIP_LIB"}
# never change the coded bytes (see the module docstring)
RUNTIME = {
    "MIVC_ENTROPY_THREADS", "MIVC_HEVC_ENTROPY", "MIVC_HEVC_ENTROPY_PROF", "MIVC_HEVC_ENTROPY_WAVES", "MIVC_HEVC_ENTROPY_WG", "MIVC_PINNED_BUDGET_MB", "MIVC_CABAC_GROUP", "MIVC_CABAC_SYMS_PER_MB",
    "MIVC_CABAC_HOST_MB", "MIVC_CABAC_PEAK_SYMS_PER_MB", "MIVC_INTRA_WAVES", "MIVC_INTRA_WG", "MIVC_HEVC_SAO_TILE", "MIVC_STAGE_TIMING", "MIVC_LOG_JSON", "MIVC_DIST_BACKEND",
    "MIVC_DIST_FORCE", "MIVC_HOST_LIB", "MIVC_NO_AUTOBUILD", "MIVC_GPU_ARCH", "MIVC_TRANSPORT", "MIVC_FAULT",
    "MIVC_WORKER_ID", "MIVC_TRANSCODE_GROUP", "MIVC_SRC_ROOT", "MIVC_OUT_ROOT", "MIVC_FLEET_STATE",
    "MIVC_FLEET_GPUS", "MIVC_CONFIG", "MIVC_RETRY_S", "MIVC_LEASES", "MIVC_HTTP_PORT", "MIVC_BACKEND",
}


def _parse(cls, field: str, raw: str):
    default = {f.name: f for f in dataclasses.fields(cls)}[field].default
    if isinstance(default, bool):
        return raw.strip().lower() not in ("0", "false", "no", "off", "")
    if isinstance(default, int):
        return int(raw)
    if isinstance(default, float):
        return float(raw)
    return raw


def encoder_overrides(cls, env=None) -> dict:
    """``{field: value}`` of the encoder knobs set in ``env`` (default os.environ) that apply
    to ``cls`` (H264Params or HevcParams)."""
    env = os.environ if env is None else env
    table = HEVC if cls.__name__ == "HevcParams" else H264
    return {f: _parse(cls, f, env[k]) for k, f in table.items() if k in env}


def set_knobs(env=None) -> dict:
    """Every ``MIVC_*`` variable that is set, by kind: {"encoder": ..., "bench": ...,
    "runtime": ..., "unknown": ...}."""
    env = os.environ if env is None else env
    out: dict = {"encoder": {}, "bench": {}, "runtime": {}, "unknown": {}}
    for k, v in sorted(env.items()):
        if not k.startswith("MIVC_"):
            continue
        kind = ("encoder" if (k in H264 or k in HEVC) else "bench" if k in BENCH
                else "runtime" if k in RUNTIME else "unknown")
        out[kind][k] = v
    return out


def check_environment(allow_knobs: bool, env=None) -> dict:
    """Refuse unknown ``MIVC_*`` names always, encoder / bench knobs unless ``allow_knobs``.
    Returns :func:`set_knobs`."""
    s = set_knobs(env)
    if s["unknown"]:
        raise SystemExit(f"unknown MIVC_* variable(s) {sorted(s['unknown'])}: not an encoder knob "
                         f"(models/knobs.py) -- unset them (a typo would silently change nothing)")
    if not allow_knobs and (s["encoder"] or s["bench"]):
        raise SystemExit(f"encoder / bench knob(s) {sorted({**s['encoder'], **s['bench']})} set in the environment: "
                         f"they change the measured configuration; pass --allow-knobs to apply them")
    return s
