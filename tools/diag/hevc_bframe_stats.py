"""Per picture-type bits / PSNR-Y / CU mix of the GPU HEVC encoder (B-picture tuning aid).

    python tools/diag/hevc_bframe_stats.py [--w 640 --h 360 --slots 8 --frames 30] [knob=value ...]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402

from govideocompressor_amd.models.h264_gpu import synth_clip  # noqa: E402
from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams  # noqa: E402
from govideocompressor_amd.ops import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w", type=int, default=640)
    ap.add_argument("--h", type=int, default=360)
    ap.add_argument("--slots", type=int, default=8)
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--crf", type=float, default=26.0)
    ap.add_argument("knobs", nargs="*")
    a = ap.parse_args()
    kw = {}
    for kv in a.knobs:
        k, v = kv.split("=")
        kw[k] = type(getattr(HevcParams(width=16, height=16), k))(float(v) if "." in v else int(v))
    host = native.host()
    y, u, v = synth_clip(a.slots, a.frames, a.w, a.h, seed=3)
    enc = GpuHevcEncoder(HevcParams(width=a.w, height=a.h, crf=a.crf, **kw), slots=a.slots)
    enc.cu_stats = {}
    res = enc.encode(y, u, v, keep_recon=True)
    rec = enc.last_recon
    src = y.cpu().numpy().astype(np.float64)
    agg = {}
    for b, r in enumerate(res):
        pics = host.hevc_decode(r.bitstream)
        bits = dict(zip(r.order, r.bits))
        for d, p in enumerate(pics):
            kind = {2: "I", 1: "P", 0: "B"}[p["slice_type"]]
            g = rec[d][0][b].cpu().numpy()[:a.h, :a.w].astype(np.float64)
            mse = np.mean((g - src[b, d]) ** 2)
            cu = p["cu"]
            inter = cu[:, 0] == 1
            e = agg.setdefault(kind, dict(n=0, bits=0.0, psnr=0.0, intra=0, l0=0, l1=0, bi=0, gran=0, qp=0.0))
            e["n"] += 1
            e["bits"] += bits[d]
            e["psnr"] += 10 * np.log10(255 ** 2 / max(mse, 1e-9))
            e["intra"] += int((~inter).sum())
            e["gran"] += len(cu)
            for name, dv in (("l0", 1), ("l1", 2), ("bi", 3)):
                e[name] += int((inter & (np.where(cu[:, 12] == 0, 1, cu[:, 12]) == dv)).sum())
            e["qp"] += p["qp"]
    out = {}
    for k, e in agg.items():
        n = e["n"]
        out[k] = dict(n=n, kbits=round(e["bits"] / n / 1000, 1), psnr=round(e["psnr"] / n, 2), qp=round(e["qp"] / n, 1),
                      intra=round(e["intra"] / e["gran"], 3), l0=round(e["l0"] / e["gran"], 3),
                      l1=round(e["l1"] / e["gran"], 3), bi=round(e["bi"] / e["gran"], 3))
    tot = sum(sum(r.bits) for r in res)
    print(json.dumps(dict(knobs=kw, kbps=round(tot / (a.slots * a.frames / 30.0) / 1000, 1),
                          psnr=round(float(np.mean([r.psnr_y for r in res])), 3), types=out, cus=enc.cu_stats)))
    enc.close()


if __name__ == "__main__":
    main()
