"""A/B timing of deblock kernel variants built as standalone shared objects
(tools/ab/<name>.so, each exporting mivc_launch_deblock), on the same GPU in one run.
Every variant filters the same unfiltered reconstruction; outputs are compared with
the first variant's.

    python tools/ab_deblock.py tools/ab/v1.so tools/ab/v2.so ...
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip  # noqa: E402


def main():
    B = 256
    enc = GpuH264Encoder(H264Params(width=1920, height=1080, lookahead=False), slots=B)
    y, u, v = synth_clip(B, 2, 1920, 1080, seed=5)
    enc.encode(y, u, v, metrics=False, keep_recon=False)
    torch.cuda.synchronize()
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    cur = enc.rec[0]
    base = [x.clone() for x in cur]
    first = None
    for path in sys.argv[1:]:
        lib = ctypes.CDLL(os.path.abspath(path))

        def launch():
            lib.mivc_launch_deblock(B, enc.wmb, enc.hmb, P(cur[0]), P(cur[1]), P(cur[2]), P(enc.hdr[1]), P(enc.nz),
                                    enc.p.chroma_qp_offset, 0, 0, P(enc.err), s)
        for x, b in zip(cur, base):
            x.copy_(b)
        launch()
        torch.cuda.synchronize()
        out = [x.clone() for x in cur]
        if first is None:
            first = out
        ts = []
        for _ in range(3):
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            for _ in range(4):
                launch()
            ev1.record()
            torch.cuda.synchronize()
            ts.append(ev0.elapsed_time(ev1) / 4)
        same = all(torch.equal(a, b) for a, b in zip(out, first))
        print(f"{os.path.basename(path)}: {min(ts):.3f} ms (runs {', '.join(f'{t:.3f}' for t in ts)}) "
              f"same_as_first={same} err={int(enc.err.item())}", flush=True)


if __name__ == "__main__":
    main()
