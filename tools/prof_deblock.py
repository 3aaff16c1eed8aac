"""Phase timing of the deblock wavefront kernel (debug build with -DMIVC_DEBLOCK_PROFILE)."""
import ctypes
import subprocess

import numpy as np
import torch

from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip

subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-DMIVC_DEBLOCK_PROFILE", "-fPIC", "-shared", "-I",
                       "csrc", "csrc/kernels/deblock.hip", "-o", "/tmp/libdb_prof.so"])
lib = ctypes.CDLL("/tmp/libdb_prof.so")
W, H, B = 1920, 1080, 8
enc = GpuH264Encoder(H264Params(width=W, height=H), slots=B)
y, u, v = synth_clip(B, 2, W, H, seed=5)
enc.encode(y, u, v)
torch.cuda.synchronize()
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
cur = enc.rec[0]
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
lib.mivc_launch_deblock(B, enc.wmb, enc.hmb, P(cur[0]), P(cur[1]), P(cur[2]), P(enc.hdr[1]), P(enc.nz), 0, 0, 0,
                        P(enc.err), s)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 256)()
lib.mivc_db_prof_read(buf)
a = np.array(buf, dtype=np.int64).reshape(16, 16)
names = ["load", "bs", "edges", "store", "publish"]
for mb in range(2, 10):
    d = np.diff(a[mb, :6])
    print(f"mb {mb}: " + " ".join(f"{n}={x}" for n, x in zip(names, d)) + f"  total={a[mb, 5] - a[mb, 0]}  gap={a[mb,0]-a[mb-1,5]}")
