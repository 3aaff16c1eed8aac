"""Per-step phase timing of the deblock wavefront (variant built with MIVC_DEBLOCK_PROFILE,
see tools/build_ab.sh): wall_clock64 stamps of workgroup 0, lane 0 of every wave."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip  # noqa: E402

lib = ctypes.CDLL(os.path.abspath(sys.argv[1]))
B = 256
enc = GpuH264Encoder(H264Params(width=1920, height=1080, lookahead=False), slots=B)
y, u, v = synth_clip(B, 2, 1920, 1080, seed=5)
enc.encode(y, u, v, metrics=False, keep_recon=False)
torch.cuda.synchronize()
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
cur = enc.rec[0]
for _ in range(2):
    lib.mivc_launch_deblock(B, enc.wmb, enc.hmb, P(cur[0]), P(cur[1]), P(cur[2]), P(enc.hdr[1]), P(enc.nz),
                            enc.p.chroma_qp_offset, 0, 0, P(enc.err), s)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (16 * 512 * 6))()
lib.mivc_db_prof_read(buf)
a = np.array(buf, dtype=np.int64).reshape(16, 512, 6).astype(np.float64) * 10.0  # ns (100 MHz)
t0 = a[a[:, :, 0] > 0][:, 0].min()
for w in (0, 1, 8, 15):
    st = a[w]
    ok = (st[:, 0] > 0) & (st[:, 5] > 0) & (st[:, 1] > 0)
    d = st[ok]
    ph = np.diff(d[:, [0, 1, 2, 3, 4, 5]], axis=1)
    per = np.diff(st[st[:, 0] > 0][:, 0])
    print(f"wave {w}: steps {ok.sum()}, start {(st[st[:,0]>0][0,0]-t0)/1e3:.1f} us end {(st[st[:,5]>0][-1,5]-t0)/1e3:.1f} us; "
          f"median ns: wait {np.median(ph[:,0]):.0f} vert {np.median(ph[:,1]):.0f} horiz {np.median(ph[:,2]):.0f} "
          f"store+ring {np.median(ph[:,3]):.0f} save+pub {np.median(ph[:,4]):.0f} period {np.median(per):.0f}")
