"""Diagnostics: per-picture bits and MB-kind histograms of the GPU encoder, P-only vs B."""
import sys

import numpy as np
import torch

from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, gop_plan, synth_clip
from govideocompressor_amd.ops import native

w, h, F = int(sys.argv[1]) if len(sys.argv) > 1 else 352, int(sys.argv[2]) if len(sys.argv) > 2 else 288, 13
host = native.host()
y, u, v = synth_clip(2, F, w, h, seed=7)
for nb in (0, 3):
    for crf in (None,):
        enc = GpuH264Encoder(H264Params(width=w, height=h, crf=crf, qp=27, bframes=nb), slots=2)
        res = enc.encode(y, u, v)
        torch.cuda.synchronize()
        r = res[0]
        plan = gop_plan(F, nb)
        print(f"bframes={nb}: total {sum(len(x.bitstream) for x in res)} B, psnr {np.mean([x.psnr_y for x in res]):.2f}")
        print("  bits/pic (coding order):", [(p.kind + str(p.d), b) for p, b in zip(plan, r.bits)])
        pics = host.decode(r.bitstream)
        for p in plan:
            if p.kind == "I":
                continue
            k = np.asarray(pics[p.d]["mb_kind"])
            vals, cnt = np.unique(k, return_counts=True)
            print(f"  {p.kind}{p.d} kinds:", dict(zip(vals.tolist(), cnt.tolist())), "qp", int(np.median(pics[p.d]["mb_qp"])))
        enc.close()
