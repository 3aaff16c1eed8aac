"""Phase timing of the ME kernel (debug build with -DMIVC_ME_PROFILE): one MB per workgroup, lin < 64."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip

subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-DMIVC_ME_PROFILE", "-fPIC", "-shared", "-I", "csrc",
                       "csrc/kernels/me.hip", "-o", "/tmp/libme_prof.so"])
lib = ctypes.CDLL("/tmp/libme_prof.so")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
R = int(sys.argv[2]) if len(sys.argv) > 2 else 8
W, H = 1920, 1080
enc = GpuH264Encoder(H264Params(width=W, height=H), slots=B)
y, u, v = synth_clip(B, 2, W, H, seed=5)
enc.encode(y, u, v)
torch.cuda.synchronize()
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
enc._prep(y, u, v, 1)
hp = P(enc.me_hp[0])
lib.mivc_launch_me(B, enc.wmb, enc.hmb, P(enc.src[0]), P(enc.rec[0][0]), P(enc.prev_mv), P(enc.mv), P(enc.me_cost),
                   P(enc.pred), P(enc.intra_cost), P(enc.qp), R, 2, hp, None, 0, 0, s, None, 0, None)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (64 * 12))()
lib.mivc_me_prof_read(buf)
a = np.array(buf, dtype=np.int64).reshape(64, 12)[:, :10]
names = ["p0cand", "window", "intsearch", "planes", "halfpel", "qpel", "pred_prep", "pred", "intra"]
for k in range(3):
    lib.mivc_launch_me(B, enc.wmb, enc.hmb, P(enc.src[0]), P(enc.rec[0][0]), P(enc.prev_mv), P(enc.mv),
                       P(enc.me_cost), P(enc.pred), P(enc.intra_cost), P(enc.qp), R, 2, hp, None, 1, 0, s)
torch.cuda.synchronize()
lib.mivc_me_prof_read(buf)
a = np.array(buf, dtype=np.int64).reshape(64, 12)[:, :10]
d = np.diff(a, axis=1)
print("B", B, "R", R, "median cycles per phase:", {n: int(np.median(d[:, i])) for i, n in enumerate(names)}, "total", int(np.median(a[:, 9] - a[:, 0])))
