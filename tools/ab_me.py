"""A/B timing of motion-estimation kernel variants built as standalone shared objects
(each exporting mivc_launch_me), on the same GPU and inputs in one run.

    python tools/ab_me.py [--range R] [--subpel S] tools/ab/a.so tools/ab/b.so ...
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--range", type=int, default=8)
    ap.add_argument("--subpel", type=int, default=2)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    B = 256
    enc = GpuH264Encoder(H264Params(width=1920, height=1080, lookahead=False), slots=B)
    y, u, v = synth_clip(B, 2, 1920, 1080, seed=5)
    enc.encode(y, u, v, metrics=False, keep_recon=False)
    enc._prep(y, u, v, 1)
    enc.qp.fill_(27)
    torch.cuda.synchronize()
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    first = None
    for path in a.libs:
        lib = ctypes.CDLL(os.path.abspath(path))

        def launch():
            lib.mivc_launch_me(B, enc.wmb, enc.hmb, P(enc.src[0]), P(enc.rec[0][0]), P(enc.prev_mv), P(enc.mv),
                               P(enc.me_cost), P(enc.pred), P(enc.intra_cost), P(enc.qp), a.range, a.subpel,
                               P(enc.me_hp), None, s)
        launch()
        torch.cuda.synchronize()
        out = (enc.mv.clone(), enc.me_cost.clone(), enc.pred.clone())
        first = first or out
        ts = []
        for _ in range(3):
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            for _ in range(4):
                launch()
            ev1.record()
            torch.cuda.synchronize()
            ts.append(ev0.elapsed_time(ev1) / 4)
        same = all(torch.equal(x, y) for x, y in zip(out, first))
        print(f"{os.path.basename(path)}: {min(ts):.3f} ms (runs {', '.join(f'{t:.3f}' for t in ts)}) "
              f"same_as_first={same}", flush=True)


if __name__ == "__main__":
    main()
