"""HEVC encoder knob sweep on synthetic content: kb/s, PSNR-Y and encode time per value of
one HevcParams field (GPU).

    python tools/hevc_knob_sweep.py merge_refine 0 1 2 3 [--w 640 --h 360 --crf 26]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("knob")
    ap.add_argument("values", nargs="+")
    ap.add_argument("--w", type=int, default=640)
    ap.add_argument("--h", type=int, default=360)
    ap.add_argument("--slots", type=int, default=8)
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--crf", type=float, default=26.0)
    a = ap.parse_args()
    y, u, v = synth_clip(a.slots, a.frames, a.w, a.h, seed=3)
    for raw in a.values:
        val = type(getattr(HevcParams(width=16, height=16), a.knob))(float(raw) if "." in raw else int(raw))
        enc = GpuHevcEncoder(HevcParams(width=a.w, height=a.h, crf=a.crf, **{a.knob: val}), slots=a.slots)
        enc.encode(y, u, v)  # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = enc.encode(y, u, v)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        enc.close()
        bits = sum(sum(r.bits) for r in res)
        print(json.dumps({a.knob: raw, "kbps": round(bits / (a.slots * a.frames / 30.0) / 1000.0, 1),
                          "psnr_y": round(sum(r.psnr_y for r in res) / len(res), 3), "s": round(dt, 3)}), flush=True)


if __name__ == "__main__":
    main()
