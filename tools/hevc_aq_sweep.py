"""HEVC rate/quality of the adaptive-QP knobs (variance AQ, cutree) on synthetic content:
kb/s and PSNR-Y per configuration at one CRF (GPU)."""
import argparse
import json
import time

import torch

from govideocompressor_amd.models.h264_gpu import synth_clip
from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w", type=int, default=640)
    ap.add_argument("--h", type=int, default=360)
    ap.add_argument("--slots", type=int, default=8)
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--crf", type=float, nargs="+", default=[26.0])
    a = ap.parse_args()
    y, u, v = synth_clip(a.slots, a.frames, a.w, a.h, seed=3)
    for crf in a.crf:
        for aq, tree in ((0.0, False), (1.0, False), (0.0, True), (1.0, True)):
            enc = GpuHevcEncoder(HevcParams(width=a.w, height=a.h, crf=crf, aq_strength=aq, cutree=tree), slots=a.slots)
            t0 = time.perf_counter()
            res = enc.encode(y, u, v)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            enc.close()
            bits = sum(sum(r.bits) for r in res)
            kbps = bits / (a.slots * a.frames / 30.0) / 1000.0
            psnr = sum(r.psnr_y for r in res) / len(res)
            print(json.dumps(dict(crf=crf, aq=aq, cutree=tree, kbps=round(kbps, 1), psnr_y=round(psnr, 3),
                                  mean_qp=float(enc.last_qps.mean()), s=round(dt, 2))), flush=True)


if __name__ == "__main__":
    main()
