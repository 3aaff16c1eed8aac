"""Time the H.264 deblocking wavefront kernel alone at the headline batch shape
(B slots of 1080p, the records of the last encoded P frame).

    python tools/time_deblock.py [B]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    enc = GpuH264Encoder(H264Params(width=1920, height=1080, lookahead=False), slots=B)
    y, u, v = synth_clip(B, 2, 1920, 1080, seed=5)
    enc.encode(y, u, v, metrics=False, keep_recon=False)
    torch.cuda.synchronize()
    P = lambda t: t.data_ptr()  # noqa: E731
    s = torch.cuda.current_stream().cuda_stream
    cur = enc.rec[0]

    def launch():
        enc.hip.deblock(B, enc.wmb, enc.hmb, P(cur[0]), P(cur[1]), P(cur[2]), P(enc.hdr[1]), P(enc.nz),
                        enc.p.chroma_qp_offset, 0, 0, P(enc.err), s)

    launch()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(5):
        launch()
    ev1.record()
    torch.cuda.synchronize()
    print(f"deblock B={B}: {ev0.elapsed_time(ev1) / 5:.3f} ms, err={int(enc.err.item())}", flush=True)


if __name__ == "__main__":
    main()
