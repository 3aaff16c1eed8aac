"""Encoder knob sweep on one GPU: time / bitrate / PSNR of the batched H.264 encoder
for a list of H264Params overrides.

    python tools/exp_encoder_knobs.py [B] [F] 'me_range=8' 'me_range=4' ...
"""
import json
import sys
import time

import torch

from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip


def parse(kv: str) -> dict:
    out = {}
    for item in kv.split(","):
        if not item:
            continue
        k, v = item.split("=")
        out[k] = type(getattr(H264Params(16, 16), k))(v) if not isinstance(getattr(H264Params(16, 16), k), bool) \
            else v in ("1", "true", "True")
    return out


def main():
    B, F = int(sys.argv[1]), int(sys.argv[2])
    y, u, v = synth_clip(B, F, 1920, 1080, seed=11)
    for spec in sys.argv[3:] or [""]:
        p = H264Params(width=1920, height=1080, crf=23, **parse(spec))
        enc = GpuH264Encoder(p, slots=B)
        enc.encode(y, u, v, metrics=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = enc.encode(y, u, v, metrics=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        nbytes = sum(r.nbytes() for r in res)
        psnr = sum(r.psnr_y for r in res) / B
        print(json.dumps({"spec": spec, "fps": round(B * F / dt, 1), "kbps": round(nbytes * 8 / (B * F / 30) / 1000, 1),
                          "psnr_y": round(psnr, 3), "mean_qp": enc.stats.get("mean_qp")}), flush=True)
        enc.close()
        del enc
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
