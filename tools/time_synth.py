"""Time GPU input synthesis at the headline batch shape (B slots x F frames of 1080p)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from govideocompressor_amd.models.h264_gpu import synth_clip  # noqa: E402

B, F = 256, 60
synth_clip(B, 2, 1920, 1080, seed=1)
torch.cuda.synchronize()
for k in range(3):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    c = synth_clip(B, F, 1920, 1080, seed=k)
    ev1.record()
    torch.cuda.synchronize()
    print(f"synth {B}x{F} 1080p: {ev0.elapsed_time(ev1):.1f} ms", flush=True)
    del c
