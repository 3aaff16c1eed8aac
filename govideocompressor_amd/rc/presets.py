"""``-preset`` (x264/x265 speed presets) -> encoder knobs.

The reference passes ``-preset`` straight to libx264/libx265 (raw ffmpeg args,
client.go:105-112).  The gfx950 encoders expose the same trade-off through their
search and analysis parameters; each preset maps onto the x264 preset's intent:

==========  ========================================================================
preset      H.264 knobs (x264 equivalent)
==========  ========================================================================
ultrafast   CAVLC, no B, no deblock, no AQ/MB-tree/lookahead, integer-pel ME radius 4,
            Intra16x16 only, 1 reference (x264: --no-cabac --bframes 0 --no-deblock
            --aq-mode 0 --subme 0 --me dia --partitions none --rc-lookahead 0 --ref 1
            --weightp 0 --trellis 0)
superfast   CABAC + 3 B, half-pel, radius 4, no MB-tree, no P/B partitions, 1 reference, no
            trellis (--subme 1 --me dia --no-mbtree --partitions i8x8,i4x4 --ref 1)
veryfast    half-pel, radius 8, 1 reference, no trellis (--subme 2 --ref 1 --trellis 0)
faster      quarter-pel, radius 8, one skip-refine pass, 2 references (--subme 4 --ref 2)
fast        quarter-pel, radius 8, 2 skip-refine passes, 2 references (--subme 6 --ref 2)
medium      defaults (x264 defaults, the reference's "264" preset: --ref 3, weightp, trellis 1;
            4 skip-refine passes)
slow        radius 12, B radius 6, Intra4x4 in P pictures, 4 references, 5 skip-refine passes,
            adaptive B placement (--me umh --subme 8 --ref 5 --b-adapt 1)
slower      radius 16, B radius 8, lookahead radius 8, 4 references, spatial direct, b-pyramid,
            6 skip-refine passes (--subme 9 --me umh --ref 8 --direct spatial --b-pyramid normal)
veryslow    slower + 8 skip-refine passes (--subme 10 --me umh --merange 24 --ref 16)
placebo     = veryslow
==========  ========================================================================

HEVC (x265): ultrafast..veryfast use radius 4 / half-pel (ultrafast and superfast with 32x32
CTUs, as x265), fast and medium the defaults (3
merge candidates, as x265), slow and slower radius 12 (slower 4 candidates), veryslow/placebo
radius 16 and 5 candidates;
slow and slower presets add the inter residual quadtree (--tu-inter-depth 1), veryslow and
placebo also sign data hiding (--signhide); --ref follows x265 (1 up to superfast, 2 for
veryfast / faster, 3 for fast / medium, 4 from slow).
"""
from __future__ import annotations

import dataclasses

NAMES = ("ultrafast", "superfast", "veryfast", "faster", "fast", "medium", "slow", "slower", "veryslow", "placebo")

H264 = {
    "ultrafast": dict(cabac=False, bframes=0, deblock=False, aq_strength=0.0, mbtree=False, lookahead=False,
                      scenecut=0, subpel=0, me_range=4, i4x4=False, skip_refine=0, refs=1, weightp=False, trellis=0),
    "superfast": dict(subpel=1, me_range=4, mbtree=False, skip_refine=0, b_me_range=2, refs=1, trellis=0,
                      partitions=False, bpartitions=False),
    "veryfast": dict(subpel=1, me_range=8, skip_refine=1, refs=1, trellis=0),
    "faster": dict(subpel=2, me_range=8, skip_refine=1, refs=2),
    "fast": dict(subpel=2, me_range=8, skip_refine=2, refs=2),
    "medium": dict(),
    # slow and up: B gate 1200 (-1.95 % BD-rate, -11 % fps on the content suite,
    # profiles/r4_knob_sweep.md); slower and up: spatial direct decided exactly in the MB
    # wavefront (-2.2 % vs temporal, profiles/r3_direct_rd.md -- the parallel fast path loses,
    # profiles/r4_trellis_spatial_rd.md).  Skip-refine passes beyond medium's 4: each one
    # ~-0.7 % BD-rate and ~-0.65 % fps at the headline (profiles/r4_knob_sweep.md)
    # slow also places its B pictures adaptively (x264 --b-adapt 1 at --b-bias 100 on weighted
    # lowres costs, one pattern per batch): -1.85 % BD-rate on the content suite for -3.2 % fps
    # at the headline (profiles/r5_badapt_rd.md) -- medium keeps the fixed pattern's throughput.
    # slower and up also keep the middle B of a run as a reference (x264 --b-pyramid normal):
    # wavefront spatial direct + pyramid -3.37 % BD-rate against medium's temporal direct, vs
    # -2.95 % without the pyramid (profiles/r6_spatial_direct_rd.md)
    "slow": dict(me_range=12, b_me_range=6, i4x4_in_p=True, refs=4, b_gate=1200, skip_refine=5, b_adapt=1, b_bias=100),
    "slower": dict(me_range=16, b_me_range=8, i4x4_in_p=True, la_range=8, skip_refine=6, refs=4, direct="spatial",
                   spatial_wavefront=True, pyramid=True, b_gate=1200),
    "veryslow": dict(me_range=16, b_me_range=8, i4x4_in_p=True, la_range=8, skip_refine=8, refs=4, direct="spatial",
                     spatial_wavefront=True, pyramid=True, b_gate=1200),
}
H264["placebo"] = H264["veryslow"]

# --ref as x265's presets (1 / 1 / 2 / 2 / 3 / 3 / 4 / 5 / 5: capped at 4 list-0 pictures here)
HEVC = {
    "ultrafast": dict(me_range=4, subpel=1, max_merge=3, la_range=4, ctu64=False, refs=1),
    "superfast": dict(me_range=4, subpel=1, max_merge=3, la_range=4, ctu64=False, refs=1),
    "veryfast": dict(me_range=4, subpel=2, max_merge=3, refs=2),
    "faster": dict(me_range=8, max_merge=3, refs=2),
    "fast": dict(me_range=8),
    "medium": dict(),
    "slow": dict(me_range=12, tu_inter_depth=1, refs=4),
    "slower": dict(me_range=12, la_range=8, tu_inter_depth=1, max_merge=4, refs=4),
    "veryslow": dict(me_range=16, la_range=8, tu_inter_depth=1, sdh=True, max_merge=5, refs=4),
}
HEVC["placebo"] = HEVC["veryslow"]


class PresetError(ValueError):
    pass


def check(name: str) -> str:
    n = (name or "medium").lower()
    if n not in NAMES:
        raise PresetError(f"unknown preset {name} (one of {', '.join(NAMES)})")
    return n


def apply(params, name: str):
    """A copy of ``params`` (H264Params or HevcParams) with the preset's knobs."""
    n = check(name)
    table = HEVC if type(params).__name__ == "HevcParams" else H264
    fields = {f.name for f in dataclasses.fields(params)}
    over = {k: v for k, v in table[n].items() if k in fields}
    return dataclasses.replace(params, **over)
