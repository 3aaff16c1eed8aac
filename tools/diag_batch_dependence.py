"""Diagnostic (GPU): does a segment's H.264 bitstream depend on the batch it is encoded in --
its width, its neighbours, or what the same encoder coded before?  Prints, per case, whether
piece 2's bytes match a width-1 encode, and the first NAL (coding order) that differs."""
import sys

import torch

sys.path.insert(0, '.')
from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip  # noqa: E402

W, H, F = 320, 192, 8


def enc(y, u, v, **kw):
    B = y.shape[0]
    e = GpuH264Encoder(H264Params(width=W, height=H, crf=23.0, **kw), slots=B)
    r = e.encode(y, u, v, idr_ids=[7] * B, metrics=False)[0]
    plan = [(p.d, p.kind) for p in e.last_plans[0]]
    e.close()
    return r, plan


def report(name, r, ref):
    a, b = r[0], ref[0]
    diff = [i for i, (p, q) in enumerate(zip(a.nals, b.nals)) if p != q]
    print(f"{name}: {'same' if a.bitstream == b.bitstream else 'DIFFER'} first_nal={diff[:1]} "
          f"plan_same={r[1] == ref[1]} lens={[len(n) for n in a.nals]} vs {[len(n) for n in b.nals]}", flush=True)


for kw in ({}, {"lookahead": False}, {"weightp": False}, {"aq_strength": 0.0, "mbtree": False}):
    one = synth_clip(1, F, W, H, seed=3, slot0=2)
    two = synth_clip(2, F, W, H, seed=3, slot0=2)
    ref = enc(*one, **kw)
    print(kw, flush=True)
    report("  width2 (neighbour piece 3)", enc(*two, **kw), ref)
    dup = [torch.cat([p, p]).contiguous() for p in one]
    report("  width2 (neighbour = copy)", enc(*dup, **kw), ref)
