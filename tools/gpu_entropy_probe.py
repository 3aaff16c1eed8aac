"""Probe (GPU): one 1080p HEVC batch (config-4 tools, GPU entropy) for a kernel trace of the
entropy stage: python tools/gpu_entropy_probe.py [slots] [frames]"""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from govideocompressor_amd.models.h264_gpu import synth_clip  # noqa: E402
from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
F = int(sys.argv[2]) if len(sys.argv) > 2 else 8
p = HevcParams(width=1920, height=1080, crf=26.0)
y, u, v = synth_clip(B, F, 1920, 1080, seed=5)
enc = GpuHevcEncoder(p, slots=B)
enc.encode(y, u, v, metrics=False)
torch.cuda.synchronize()
t = time.perf_counter()
res = enc.encode(y, u, v, metrics=False)
torch.cuda.synchronize()
print(f"{B * F / (time.perf_counter() - t):.1f} fps, {sum(len(r.bitstream) for r in res) / B / F / 1024:.1f} KiB/picture",
      flush=True)
enc.close()
if __import__("os").environ.get("MIVC_HEVC_ENTROPY_PROF") == "1":
    for k, v in enc.entropy_profile().items():
        n = max(1, v["ctus"])
        print(k, {kk: (round(vv / n) if kk != "ctus" else vv) for kk, vv in v.items()}, "(cycles per CTU)", flush=True)
