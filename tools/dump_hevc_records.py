"""Capture the decision records the GPU HEVC encoder hands to the host CABAC writer
(one I and one P picture of a few slots) as raw files, for CPU profiling of
csrc/host/hevc_writer.cc (tools/bench_hevc_writer.cc).

    python tools/dump_hevc_records.py OUTDIR [B]
"""
import json
import os
import sys

import numpy as np
import torch

from govideocompressor_amd.models.h264_gpu import synth_clip
from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams


class _Spy:
    def __init__(self, host, out):
        self._h, self.out, self.n = host, out, 0
        self.meta = []

    def __getattr__(self, k):
        return getattr(self._h, k)

    def hevc_write_slices_packed(self, cfg, fps, ctu, cu, nz, off, lv, threads=1):
        return [self.hevc_write_slice_packed(cfg, fp, ctu[b], cu[b], nz[b], off[b], lv[b])[0]
                for b, fp in enumerate(fps)]

    def hevc_write_slice_packed(self, cfg, fp, ctu, cu, nz, off, lv):
        from govideocompressor_amd.utils.hevc_synth import unpack_levels
        W, H = -(-cfg["width"] // 32) * 32, -(-cfg["height"] // 32) * 32
        if fp["poc"] in (0, 1):
            self.hevc_write_slice(cfg, fp, ctu, cu, *unpack_levels(nz, off, lv, W, H), record_only=True)
        return self._h.hevc_write_slice_packed(cfg, fp, ctu, cu, nz, off, lv)

    def hevc_write_slice(self, cfg, fp, ctu, cu, cy, cb, cr, record_only=False):
        if fp["poc"] in (0, 1):
            i = self.n
            self.n += 1
            for name, a in (("ctu", ctu), ("cu", cu), ("cy", cy), ("cb", cb), ("cr", cr)):
                np.ascontiguousarray(a).tofile(os.path.join(self.out, f"{i}_{name}.bin"))
            self.meta.append(dict(cfg=cfg, fp=fp, cy=list(cy.shape), cb=list(cb.shape), ctu=list(ctu.shape),
                                  cu=list(cu.shape)))
        if record_only:
            return None
        return self._h.hevc_write_slice(cfg, fp, ctu, cu, cy, cb, cr)


def main():
    out = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    os.makedirs(out, exist_ok=True)
    enc = GpuHevcEncoder(HevcParams(width=1920, height=1080, crf=26), slots=B, entropy_threads=1)
    spy = _Spy(enc.host, out)
    enc.host = spy
    y, u, v = synth_clip(B, 2, 1920, 1080, seed=7)
    res = enc.encode(y, u, v, metrics=False)
    torch.cuda.synchronize()
    with open(os.path.join(out, "meta.txt"), "w") as f:
        for i, m in enumerate(spy.meta):
            c, fp = m["cfg"], m["fp"]
            f.write(f"{i} {c['width']} {c['height']} {c['bit_depth']} {c['sao']} {c['deblock']} {c['max_merge']} "
                    f"{fp['idr']} {fp['poc']} {fp['qp']} {fp['slice_type']}\n")
    with open(os.path.join(out, "meta.json"), "w") as f:
        json.dump(dict(records=spy.meta, bytes=[[len(n) for n in r.nals] for r in res]), f)
    print("dumped", spy.n, "pictures to", out)


if __name__ == "__main__":
    main()
