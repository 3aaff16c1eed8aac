"""Time the H.264 motion-estimation kernel alone for (range, subpel) variants at the
headline batch shape (B slots of 1080p, one P frame), to split its cost by phase.

    python tools/time_me.py [B]
"""
import sys

import torch

from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    enc = GpuH264Encoder(H264Params(width=1920, height=1080, lookahead=False), slots=B)
    y, u, v = synth_clip(B, 2, 1920, 1080, seed=5)
    enc.encode(y, u, v, metrics=False, keep_recon=False)
    enc._prep(y, u, v, 1)
    torch.cuda.synchronize()
    P = lambda t: t.data_ptr()  # noqa: E731
    s = torch.cuda.current_stream().cuda_stream
    enc.qp.fill_(27)

    def run(r, sp, n=5):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        enc.hip.me(B, enc.wmb, enc.hmb, P(enc.src[0]), P(enc.rec[0][0]), P(enc.prev_mv), P(enc.mv), P(enc.me_cost),
                   P(enc.pred), P(enc.intra_cost), P(enc.qp), r, sp, s, P(enc.me_hp))
        ev0.record()
        for _ in range(n):
            enc.hip.me(B, enc.wmb, enc.hmb, P(enc.src[0]), P(enc.rec[0][0]), P(enc.prev_mv), P(enc.mv),
                       P(enc.me_cost), P(enc.pred), P(enc.intra_cost), P(enc.qp), r, sp, s, P(enc.me_hp))
        ev1.record()
        torch.cuda.synchronize()
        return ev0.elapsed_time(ev1) / n

    for r, sp in ((8, 2), (8, 1), (8, 0), (4, 2), (4, 0), (1, 0), (0, 0)):
        print(f"range {r} subpel {sp}: {run(r, sp):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
