"""RD table + Bjontegaard delta rate from bench.py logs (tools/gpu/rd_table.sh).

usage: python tools/rd_table.py gpurun_out > profiles/r2_rd_table.md
"""
import json
import os
import sys

import numpy as np

CFGS = [("bframes3", "High CABAC 8x8dct + 3 B (temporal direct)"),
        ("bframes3no8x8dct", "Main CABAC + 3 B (temporal direct)"), ("bframes0no8x8dct", "Main CABAC, P only"),
        ("bframes0cavlc", "Constrained Baseline CAVLC (round 1)")]
CRFS = [18, 23, 28, 33]


def load(d):
    out = {}
    for tag, _ in CFGS:
        pts = []
        for crf in CRFS:
            p = os.path.join(d, f"rd_{crf}_{tag}.log")
            line = [x for x in open(p).read().splitlines() if x.startswith("{")][-1]
            j = json.loads(line)
            q = j["quality"]
            pts.append((crf, q["bitrate_kbps"], q["psnr_y_db"], q["ssim_y"], j["value"]))
        out[tag] = pts
    return out


def bd_rate(ref, test):
    """Bjontegaard delta bit rate (%) of test vs ref: cubic fit of log-rate over PSNR,
    integrated over the overlapping PSNR range."""
    r1, p1 = np.log([x[1] for x in ref]), np.array([x[2] for x in ref])
    r2, p2 = np.log([x[1] for x in test]), np.array([x[2] for x in test])
    f1, f2 = np.polyfit(p1, r1, 3), np.polyfit(p2, r2, 3)
    lo, hi = max(p1.min(), p2.min()), min(p1.max(), p2.max())
    i1 = np.polyval(np.polyint(f1), hi) - np.polyval(np.polyint(f1), lo)
    i2 = np.polyval(np.polyint(f2), hi) - np.polyval(np.polyint(f2), lo)
    return (np.exp((i2 - i1) / (hi - lo)) - 1) * 100


def main():
    data = load(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
    print("# RD table: 1080p30 synthetic content, 256 segments x 60 frames, GPU lookahead CRF (bench.py)\n")
    print("Quality measured by bench.py on its first (untimed) warmup step; PSNR-Y / SSIM-Y are the")
    print("per-frame means over every segment. fps = the timed step of the same run.\n")
    print("| encoder | CRF | kb/s | PSNR-Y dB | SSIM-Y | fps |")
    print("|---|---|---|---|---|---|")
    for tag, name in CFGS:
        for crf, kbps, psnr, ssim, fps in data[tag]:
            print(f"| {name} | {crf} | {kbps:.1f} | {psnr:.3f} | {ssim:.4f} | {fps:.0f} |")
    base = data["bframes0cavlc"]
    print("\n| encoder | BD-rate vs round-1 Baseline CAVLC (PSNR-Y) |")
    print("|---|---|")
    for tag, name in CFGS[:3]:
        print(f"| {name} | {bd_rate(base, data[tag]):+.1f} % |")
    print(f"| High 8x8dct + 3 B vs Main + 3 B | {bd_rate(data['bframes3no8x8dct'], data['bframes3']):+.1f} % |")
    print(f"| Main + 3 B vs Main P only | {bd_rate(data['bframes0no8x8dct'], data['bframes3no8x8dct']):+.1f} % |")


if __name__ == "__main__":
    main()
