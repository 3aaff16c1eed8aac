"""B-picture diagnostics on the GPU: bits / PSNR and the chosen picture types for
bframes 0 / 3, b-adapt 0 / 1, fixed QP and CRF, small clip and 1080p bench content."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip


def run(w, h, B, F, over, label, kind="default"):
    y, u, v = synth_clip(B, F, w, h, seed=7, kind=kind) if kind != "default" else synth_clip(B, F, w, h, seed=7)
    enc = GpuH264Encoder(H264Params(width=w, height=h, **over), slots=B)
    res = enc.encode(y, u, v)
    bits = sum(len(r.bitstream) for r in res) * 8
    psnr = float(np.mean([r.psnr_y for r in res]))
    plans = enc.last_plans
    types = ["".join(p.kind for p in sorted(plans[b], key=lambda q: q.d)) for b in range(min(2, B))]
    fb = {}
    for b, r in enumerate(res):
        for t, pic in enumerate(plans[b]):
            fb.setdefault(pic.kind, []).append(r.bits[t])
    qps = enc.last_qps[:2].tolist()
    out = dict(label=label, w=w, h=h, kbits=bits / 1000, psnr=round(psnr, 3),
               b_ratio=enc.stats.get("b_ratio"), mean_qp=enc.stats.get("mean_qp"), types=types, qps=qps,
               bits_by_type={k: int(np.mean(v)) for k, v in fb.items()})
    enc.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    small = dict(crf=None, qp=27)
    for nb, ba in ((0, 0), (3, 0), (3, 1)):
        run(352, 288, 2, 13, dict(small, bframes=nb, b_adapt=ba), f"cif qp27 bf{nb} ba{ba}")
    if len(sys.argv) > 1:
        for nb, ba in ((0, 0), (3, 0), (3, 1)):
            run(1920, 1080, 16, 30, dict(crf=23.0, bframes=nb, b_adapt=ba), f"1080p crf23 bf{nb} ba{ba}")
