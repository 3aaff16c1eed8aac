"""HEVC RD sweep: kb/s and PSNR-Y at several CRFs for encoder configurations given as
``name:knob=value,knob=value`` and Bjontegaard delta rates against the first one (GPU).

    python tools/hevc_rd.py "p_only:bframes=0,merge_exact=0" "b3:bframes=3" [--crfs 22 26 30 34]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from govideocompressor_amd.models.h264_gpu import synth_clip  # noqa: E402
from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams  # noqa: E402
from tools.rd_table import bd_rate  # noqa: E402


def parse(spec):
    name, _, kv = spec.partition(":")
    kw = {}
    for item in filter(None, kv.split(",")):
        k, v = item.split("=")
        kw[k] = type(getattr(HevcParams(width=16, height=16), k))(float(v) if "." in v else int(v))
    return name, kw


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+")
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--slots", type=int, default=16)
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--crfs", type=float, nargs="+", default=[22.0, 26.0, 30.0, 34.0])
    a = ap.parse_args()
    y, u, v = synth_clip(a.slots, a.frames, a.w, a.h, seed=3)
    pts = {}
    for spec in a.configs:
        name, kw = parse(spec)
        enc = GpuHevcEncoder(HevcParams(width=a.w, height=a.h, crf=a.crfs[0], **kw), slots=a.slots)
        enc.encode(y, u, v, metrics=False)  # warm-up
        for crf in a.crfs:
            enc.p.crf = crf
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = enc.encode(y, u, v)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            kbps = sum(sum(r.bits) for r in res) / (a.slots * a.frames / 30.0) / 1000.0
            psnr = sum(r.psnr_y for r in res) / len(res)
            pts.setdefault(name, []).append((crf, kbps, psnr))
            print(json.dumps(dict(config=name, knobs=kw, crf=crf, kbps=round(kbps, 1), psnr_y=round(psnr, 3),
                                  fps=round(a.slots * a.frames / dt, 1))), flush=True)
        enc.close()
    names = list(pts)
    print(f"\n| config | BD-rate vs {names[0]} (PSNR-Y) |\n|---|---|")
    for n in names[1:]:
        print(f"| {n} | {bd_rate(pts[names[0]], pts[n]):+.1f} % |")


if __name__ == "__main__":
    main()
