"""Phase timing of the intra wavefront kernel (debug build with -DMIVC_INTRA_PROFILE).

Build the instrumented library on the CPU first (no compiling inside a GPU call):
    hipcc --offload-arch=gfx950 -O3 -DMIVC_INTRA_PROFILE -fPIC -shared -I csrc \
          csrc/kernels/encode_intra.hip -o abso/libintra_prof.so
then run ``python tools/prof_intra.py`` on the GPU box.
"""
import ctypes
import os

import numpy as np
import torch

from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip

lib = ctypes.CDLL(os.path.abspath("abso/libintra_prof.so"))
W, H, B = 1920, 1080, 8
enc = GpuH264Encoder(H264Params(width=W, height=H), slots=B)
y, u, v = synth_clip(B, 2, W, H, seed=5)
enc.encode(y, u, v)
torch.cuda.synchronize()
enc._prep(y, u, v, 0)
enc.qp.fill_(20)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
cur = enc.rec[0]
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
lib.mivc_launch_encode_intra(B, enc.wmb, enc.hmb, P(enc.src[0]), P(enc.src[1]), P(enc.src[2]), P(cur[0]), P(cur[1]),
                             P(cur[2]), P(enc.qp), 0, P(enc.hdr[0]), P(enc.coef[0]), P(enc.nz), None, None,
                             P(enc.err), 1, None, s, 1, None, 0, 0, 0, ctypes.c_float(1.0), None, ctypes.c_longlong(0))
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 256)()
lib.mivc_intra_prof_read(buf)
a = np.array(buf, dtype=np.int64).reshape(16, 16)
names = ["stage", "i16dec", "cdec", "i4+i8trial", "encode", "chroma", "tail", "publish"]
for mb in range(2, 10):
    d = np.diff(a[mb, :9])
    print(f"mb {mb}: " + " ".join(f"{n}={x}" for n, x in zip(names, d)) + f"  (i4={a[mb, 9] - a[mb, 3]} "
          f"i8={a[mb, 4] - a[mb, 9]})  total={a[mb, 8] - a[mb, 0]}  gap_from_prev={a[mb,0]-a[mb-1,8]}")

# inside the I4x4 trial, block 1 of each MB: 10 = its neighbours staged, 11 = DC value,
# 12 = mode ranked, 13 = transformed / quantised / reconstructed
for mb in range(2, 6):
    r = a[mb]
    print(f"mb {mb} i4 block 1: dc={r[11] - r[10]} rank={r[12] - r[11]} tq_recon={r[13] - r[12]} (block ~{r[13] - r[10]}+nb)")
