"""Encode B slots x F frames of synthetic 4K with the GPU H.264 encoder (profiling helper)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip  # noqa: E402

B, F = int(sys.argv[1]), int(sys.argv[2])
enc = GpuH264Encoder(H264Params(width=3840, height=2160, crf=20), slots=B)
y, u, v = synth_clip(B, F, 3840, 2160, seed=3)
t = time.perf_counter()
res = enc.encode(y, u, v, metrics=False)
torch.cuda.synchronize()
print("encode", round(time.perf_counter() - t, 2), "s", flush=True)
