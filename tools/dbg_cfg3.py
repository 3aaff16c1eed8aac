"""Debug driver for bench config 3 (4K transcode) with stage timings and a stack dump on stall."""
import faulthandler
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
faulthandler.dump_traceback_later(90, repeat=True)
import torch  # noqa: E402

from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip  # noqa: E402
from govideocompressor_amd.ops import native  # noqa: E402
from govideocompressor_amd.pipeline import encode_file  # noqa: E402

S, F = int(sys.argv[1]), int(sys.argv[2])
W, H = 3840, 2160
t = time.perf_counter()
enc = GpuH264Encoder(H264Params(width=W, height=H, crf=20), slots=S)
y, u, v = synth_clip(S, F, W, H, seed=3)
res = enc.encode(y, u, v, metrics=False)
torch.cuda.synchronize()
print("source encode", round(time.perf_counter() - t, 2), "s", flush=True)
enc.close()
tmp = tempfile.mkdtemp()
src = os.path.join(tmp, "in.264")
open(src, "wb").write(native.host().concat([r.bitstream for r in res]))
t = time.perf_counter()
r = encode_file(src, os.path.join(tmp, "out.264"), args="264", backend="gpu", slots=S, seg_frames=F,
                log=lambda s: print(s, flush=True))
print("transcode", round(time.perf_counter() - t, 2), "s", {k: r[k] for k in r if k != "decode_stats_rank"}, flush=True)
