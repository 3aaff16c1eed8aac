"""Write the GPU HEVC encoder's test streams (tests/test_gpu_hevc.py configurations) and
their GPU reconstructions to gpurun_out/ for offline comparison with the CPU decoders."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from govideocompressor_amd.models.h264_gpu import synth_clip  # noqa: E402
from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams  # noqa: E402

out = os.path.join("gpurun_out", "hevc_streams")
os.makedirs(out, exist_ok=True)
for bd in (8, 10):
    W, H, F, B = 128, 96, 5, 3
    enc = GpuHevcEncoder(HevcParams(width=W, height=H, crf=None, qp=30, bit_depth=bd), slots=B)
    y, u, v = synth_clip(B, F, W, H, seed=7, bit_depth=bd)
    res = enc.encode(y, u, v, keep_recon=True)
    rec = enc.last_recon
    for b, r in enumerate(res):
        open(os.path.join(out, f"p_bd{bd}_s{b}.265"), "wb").write(r.bitstream)
        planes = np.concatenate([np.concatenate([rec[t][k][b].cpu().numpy().astype(np.uint16).ravel() for k in range(3)])
                                 for t in range(F)])
        np.save(os.path.join(out, f"p_bd{bd}_s{b}_rec.npy"), planes)
    enc.close()
print("ok")
