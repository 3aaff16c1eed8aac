"""Multi-content RD suite: encoder configurations x content classes x CRFs, BD-rate per class.

Every default of the H.264 encoder (GOP decisions, direct mode, search ranges, gates) must
hold up on more than the headline's easy panning content: this runs each content class of
csrc/kernels/synth.hip (default, fast pan, static + small movers, fade, zoom, cuts, heavy
noise) through several configurations at four CRFs and reports bitrate, PSNR-Y, frames/s
and the Bjontegaard delta rate of every configuration against the first, per class.

usage (GPU):  python tools/content_rd.py run OUT.json [--slots 32 --frames 60 --size 1920x1080]
              python tools/content_rd.py table OUT.json > profiles/r4_content_rd.md
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CRFS = (18, 23, 28, 33)
HEVC_CRFS = (22, 26, 30, 34)


def _nbytes(r) -> int:
    return r.nbytes() if hasattr(r, "nbytes") else len(r.bitstream)
# name -> H264Params overrides.  "r3" = round 3's GOP / direct decisions
CONFIGS = {
    "r3": dict(b_adapt=0, pyramid=False, direct="temporal"),
    "badapt": dict(b_adapt=1, pyramid=False, direct="temporal"),
    "spatial": dict(b_adapt=1, pyramid=False, direct="spatial"),
    "pyramid": dict(b_adapt=1, pyramid=True, direct="spatial"),
    "bias20": dict(b_adapt=1, b_bias=20),
    "bias40": dict(b_adapt=1, b_bias=40),
    "bias70": dict(b_adapt=1, b_bias=70),
    "bias100": dict(b_adapt=1, b_bias=100),
    "badapt_ng": dict(b_adapt=1, badapt_guard=False),  # without x264's intra-MB guards
    "slices4": dict(slices=4),
    "noseed": dict(lowres_seed=False),
    "trellis1": dict(trellis=1),  # round 3's trellis scope (4x4 luma only)
    "bf0": dict(bframes=0),       # P pictures only
    "la4": dict(la_range=4),      # lowres search +-4 around the quarter-resolution seed (default +-6)
    # knob sweep (VERDICT r3 task 2: re-tune the gates and ranges on all classes together)
    "bgate1200": dict(b_gate=1200),
    "bgate1800": dict(b_gate=1800),
    "skr1": dict(skip_refine=1),
    "skr3": dict(skip_refine=3),
    "skr4": dict(skip_refine=4),
    "skr5": dict(skip_refine=5),
    "pms1000": dict(part_min_satd=1000),
    "pms4000": dict(part_min_satd=4000),
    "mer6": dict(me_range=6),
    "mer12": dict(me_range=12),
    "besad0": dict(b_early_sad=0),
    "bq3": dict(b_qp_offset=3.0),   # B pictures above their references (x264 pbratio 1.3 = +2.27)
    "bq4": dict(b_qp_offset=4.0),
    "bgate4800": dict(b_gate=4800),
    "bme8": dict(b_me_range=8),
    "refgate750": dict(ref_gate=750),
    "refgate3000": dict(ref_gate=3000),
    "tl07": dict(trellis_lambda=0.7),
    "tl14": dict(trellis_lambda=1.4),
    "itr0": dict(intra_trellis=0),  # dead-zone levels on intra MBs (round 4)
    "itr1": dict(intra_trellis=2),  # RD levels on intra MBs too
    "law0": dict(la_weights=False),  # lookahead without lowres weighting (round 4)
    "ba100w": dict(b_adapt=1, b_bias=100),  # b-adapt at --b-bias 100 (lowres weighting on)
    "ba100w0": dict(b_adapt=1, b_bias=100, la_weights=False),
    "ba40w": dict(b_adapt=1, b_bias=40),
    "ba100s": dict(b_adapt=1, b_bias=100, badapt_shared=True),   # one pattern per batch
    "ba100p": dict(b_adapt=1, b_bias=100, badapt_shared=False),  # one pattern per slot
    "ba70s": dict(b_adapt=1, b_bias=70, badapt_shared=True),
    "ba100r1": dict(b_adapt=1, b_bias=100, badapt_range=1),  # la_multi refinement +-1
    # fast spatial direct with the fixed GOP pattern: exact motion re-predicted (tol -1, round 4's
    # first version) / estimate kept as explicit motion beyond 0 / 4 quarter samples; b-pyramid
    "sp_repredict": dict(direct="spatial", spatial_fix_tol=-1),
    "sp_tol0": dict(direct="spatial", spatial_fix_tol=0),
    "sp_tol4": dict(direct="spatial", spatial_fix_tol=4),
    "sp_pyramid": dict(direct="spatial", pyramid=True),
    # spatial direct decided exactly inside the MB wavefront (b_spatial_decide), + b-pyramid
    "sp_wave": dict(direct="spatial", spatial_wavefront=True),
    "sp_wave_pyr": dict(direct="spatial", spatial_wavefront=True, pyramid=True),
    "i4p": dict(i4x4_in_p=True),  # x264's analysis: Intra4x4 trials in P / B pictures too
    "default": dict(),  # the current defaults
}
# HEVC (GpuHevcEncoder) configurations: x265 --signhide, --bframes variants
HEVC_CONFIGS = {
    "default": dict(),
    "signhide": dict(sdh=True),
    "bf0": dict(bframes=0),
    "bf3": dict(bframes=3, b_qp_offset=2),
    "bqp2": dict(b_qp_offset=2),
    "bqp3": dict(b_qp_offset=3),
    "bqp6": dict(b_qp_offset=6),
    "bqp4": dict(b_qp_offset=4),
    "bqp8": dict(b_qp_offset=8),
    # x265 --ref (round 6): farther list-0 pictures of P pictures, gated / ungated searches
    "ref2": dict(refs=2),
    "ref3": dict(refs=3),
    "ref3g0": dict(refs=3, ref_gate=0),
    "ref3g1500": dict(refs=3, ref_gate=1500),
    "ref3g6000": dict(refs=3, ref_gate=6000),
    # 8x8 inter CUs in P pictures (round 6), split overhead in bits
    "i8o8": dict(inter8=True, inter8_overhead=8),
    "i8o16": dict(inter8=True, inter8_overhead=16),
    "i8o24": dict(inter8=True, inter8_overhead=24),
    "i8o16m1000": dict(inter8=True, inter8_overhead=16, inter8_min_satd=1000),
    # x265 --b-adapt (round 6): adaptive B runs, one pattern per batch
    "ba_b2": dict(b_adapt=1, bframes=2),
    "ba_b3": dict(b_adapt=1, bframes=3),
    "ba_b3bias100": dict(b_adapt=1, bframes=3, b_bias=100),
    "ba_b4": dict(b_adapt=1, bframes=4),
    # x265 medium's --tu-inter-depth 1 and --signhide, re-measured on the round-6 encoder
    "tud1": dict(tu_inter_depth=1),
    "sdh": dict(sdh=True),
}


def run(args):
    import torch
    from govideocompressor_amd.models.h264_gpu import CONTENT_KINDS, GpuH264Encoder, H264Params, synth_clip

    w, h = (int(x) for x in args.size.split("x"))
    out = {"size": args.size, "slots": args.slots, "frames": args.frames, "codec": args.codec, "points": []}
    kinds = args.kinds.split(",") if args.kinds else list(CONTENT_KINDS)
    table = HEVC_CONFIGS if args.codec == "hevc" else CONFIGS
    configs = {k: table[k] for k in (args.configs.split(",") if args.configs else table)}
    crfs = HEVC_CRFS if args.codec == "hevc" else CRFS
    if args.codec == "hevc":
        from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams
        make = lambda over: GpuHevcEncoder(HevcParams(width=w, height=h, **over), slots=args.slots)  # noqa: E731
    else:
        make = lambda over: GpuH264Encoder(H264Params(width=w, height=h, **over), slots=args.slots)  # noqa: E731
    clips = {}
    for kind in kinds:
        clips[kind] = synth_clip(args.slots, args.frames, w, h, seed=17, kind=kind)
    for cname, over in configs.items():
        enc = make(over)
        for kind in kinds:
            y, u, v = clips[kind]
            for crf in crfs:
                enc.p.crf = float(crf)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                res = enc.encode(y, u, v, metrics=True)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                bits = sum(8 * _nbytes(r) for r in res)
                kbps = bits / (args.slots * args.frames / 30.0) / 1000.0
                stats = getattr(enc, "stats", {}) or {}
                pt = dict(config=cname, kind=kind, crf=crf, kbps=kbps, psnr=float(np.mean([r.psnr_y for r in res])),
                          ssim=float(np.mean([getattr(r, "ssim_y", 0.0) for r in res])), fps=args.slots * args.frames / dt,
                          b_ratio=stats.get("b_ratio", 0.0), scenecuts=stats.get("scenecuts", 0),
                          spatial_fix_ratio=stats.get("spatial_fix_ratio"),
                          spatial_conv_ratio=stats.get("spatial_conv_ratio"))
                out["points"].append(pt)
                print(json.dumps(pt), flush=True)
        enc.close()
        del enc
        torch.cuda.empty_cache()
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)


def table(args):
    from rd_table import bd_rate
    d = json.load(open(args.out))
    pts = d["points"]
    kinds = list(dict.fromkeys(p["kind"] for p in pts))
    configs = list(dict.fromkeys(p["config"] for p in pts))
    print(f"# Multi-content RD suite, {d.get('codec', 'h264').upper()} ({d['size']}, {d['slots']} segments x "
          f"{d['frames']} frames per class, GPU lookahead CRF)\n")
    print("Content classes of csrc/kernels/synth.hip; PSNR-Y / SSIM-Y are per-frame means over every")
    print(f"segment; fps = the whole encode call of {d['slots']} segments (lookahead, encode, entropy).\n")
    print("| class | config | CRF | kb/s | PSNR-Y dB | SSIM-Y | B share | fps |")
    print("|---|---|---|---|---|---|---|---|")
    for k in kinds:
        for c in configs:
            for p in (q for q in pts if q["kind"] == k and q["config"] == c):
                print(f"| {k} | {c} | {p['crf']} | {p['kbps']:.1f} | {p['psnr']:.3f} | {p['ssim']:.4f} | "
                      f"{p['b_ratio']:.2f} | {p['fps']:.0f} |")
    base = configs[0]
    print(f"\n| class | " + " | ".join(f"{c} vs {base} (BD-rate, PSNR-Y)" for c in configs[1:]) + " |")
    print("|---|" + "---|" * (len(configs) - 1))
    allv = {c: [] for c in configs[1:]}
    for k in kinds:
        ref = [(p["crf"], p["kbps"], p["psnr"]) for p in pts if p["kind"] == k and p["config"] == base]
        row = []
        for c in configs[1:]:
            tst = [(p["crf"], p["kbps"], p["psnr"]) for p in pts if p["kind"] == k and p["config"] == c]
            v = bd_rate(ref, tst)
            allv[c].append(v)
            row.append(f"{v:+.2f} %")
        print(f"| {k} | " + " | ".join(row) + " |")
    print("| **mean** | " + " | ".join(f"{np.mean(allv[c]):+.2f} %" for c in configs[1:]) + " |")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=("run", "table"))
    ap.add_argument("out")
    ap.add_argument("--slots", type=int, default=32)
    ap.add_argument("--frames", type=int, default=60)
    ap.add_argument("--size", default="1920x1080")
    ap.add_argument("--kinds", default="")
    ap.add_argument("--configs", default="")
    ap.add_argument("--codec", default="h264", choices=("h264", "hevc"))
    args = ap.parse_args()
    run(args) if args.cmd == "run" else table(args)


if __name__ == "__main__":
    main()
