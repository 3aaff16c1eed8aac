"""Time the wavefront kernels of one frame step versus the number of slots B."""
import sys
import time

import torch

from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip

W, H = 1920, 1080
for B in [int(x) for x in sys.argv[1:]] or [32, 64, 128, 256]:
    p = H264Params(width=W, height=H)
    enc = GpuH264Encoder(p, slots=B)
    y, u, v = synth_clip(B, 4, W, H, seed=5)
    enc.encode(y, u, v)  # warm
    torch.cuda.synchronize()
    # time individual kernels of an I and a P step
    hip = enc.hip
    s = torch.cuda.current_stream().cuda_stream
    P_ = enc._ptr
    enc.qp.fill_(23)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(8)]
    cur, ref = enc.rec[0], enc.rec[1]
    enc._prep(y, u, v, 1)
    torch.cuda.synchronize()
    ev[0].record()
    hip.encode_intra(B, enc.wmb, enc.hmb, P_(enc.src[0]), P_(enc.src[1]), P_(enc.src[2]), P_(cur[0]), P_(cur[1]),
                     P_(cur[2]), P_(enc.qp), 0, P_(enc.hdr[0]), P_(enc.coef[0]), P_(enc.nz), 0, 0, P_(enc.err), 1, s)
    ev[1].record()
    hip.deblock(B, enc.wmb, enc.hmb, P_(cur[0]), P_(cur[1]), P_(cur[2]), P_(enc.hdr[0]), P_(enc.nz), 0, 0, 0,
                P_(enc.err), s)
    ev[2].record()
    torch.cuda.synchronize()
    print(f"B={B} I-intra {ev[0].elapsed_time(ev[1]):.2f} ms  deblock {ev[1].elapsed_time(ev[2]):.2f} ms", flush=True)
    enc.close()
    del enc, y, u, v
    torch.cuda.empty_cache()
