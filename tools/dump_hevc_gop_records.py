"""Capture everything the GPU HEVC encoder hands the host CABAC writer for a whole GOP (the
default tool set: B pictures, TMVP, several list-0 pictures, weightp, CTU 64, WPP, AQ), per
picture and slot, for CPU profiling of csrc/host/hevc_writer.cc with
tools/bench_hevc_writer_gop.cc (gprof-able):

    python tools/dump_hevc_gop_records.py OUTDIR [slots] [frames]     (on an MI355X)

OUTDIR/meta.txt: one line per written slice, "key value" tokens (lists as count + items);
OUTDIR/<n>_{ctu,cu,nz,off,lv}.bin: its packed records (hevc_write_slice_packed's inputs);
col_cu references the slice whose records are the collocated picture's (-1: none)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from govideocompressor_amd.models.h264_gpu import synth_clip  # noqa: E402
from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams  # noqa: E402

CFG_KEYS = ("width", "height", "bit_depth", "sao", "deblock", "max_merge", "wpp", "cu_qp_delta", "tu_inter_depth",
            "sdh", "level_idc", "bframes", "tmvp", "pyramid", "ctu64", "weightp", "refs")


class _Spy:
    def __init__(self, host, out):
        self._h, self.out, self.n, self.lines = host, out, 0, []
        self.by_cu = {}  # id of a CU record array -> slice index (collocated references)

    def __getattr__(self, k):
        return getattr(self._h, k)

    def hevc_write_slices_packed(self, cfg, fps, ctu, cu, nz, off, lv, threads=1, stats=False):
        for b, fp in enumerate(fps):
            i = self.n
            self.n += 1
            # only the level blocks the slice uses (the pinned buffer holds the whole capacity)
            nzb = np.asarray(nz[b]).reshape(-1, 2)
            cnt = np.array([bin(int(x)).count("1") for x in nzb[:, 0]]) + \
                np.array([bin(int(x) & 0xFFFFFFFF).count("1") for x in nzb[:, 1]])
            used = int((np.asarray(off[b]).astype(np.int64) + cnt).max()) if len(cnt) else 0
            for name, a in (("ctu", ctu[b]), ("cu", cu[b]), ("nz", nz[b]), ("off", off[b]),
                            ("lv", np.asarray(lv[b])[:used * 16])):
                np.ascontiguousarray(a).tofile(os.path.join(self.out, f"{i}_{name}.bin"))
            toks = [f"{k} {int(cfg.get(k, 0))}" for k in CFG_KEYS]
            col = -1
            for k, v in fp.items():
                if k == "col_cu":
                    col = -1 if v is None else self.by_cu.get((fp["col_poc"], b), -1)
                elif k in ("rps",):
                    toks.append(f"rps {len(v)} " + " ".join(f"{p} {u}" for p, u in v))
                elif isinstance(v, (list, tuple)):
                    toks.append(f"{k} {len(v)} " + " ".join(str(int(x)) for x in v))
                else:
                    toks.append(f"{k} {int(v)}")
            toks.append(f"col_cu {col}")
            self.lines.append(f"{i} " + " ".join(toks))
            self.by_cu[(fp["poc"], b)] = i
        return self._h.hevc_write_slices_packed(cfg, fps, ctu, cu, nz, off, lv, threads, stats) if stats else \
            self._h.hevc_write_slices_packed(cfg, fps, ctu, cu, nz, off, lv, threads)


def main():
    out = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    F = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    os.makedirs(out, exist_ok=True)
    enc = GpuHevcEncoder(HevcParams(width=1920, height=1080, crf=26), slots=B, entropy_threads=1)
    spy = _Spy(enc.host, out)
    enc.host = spy
    y, u, v = synth_clip(B, F, 1920, 1080, seed=7)
    res = enc.encode(y, u, v, metrics=False)
    torch.cuda.synchronize()
    with open(os.path.join(out, "meta.txt"), "w") as f:
        f.write("\n".join(spy.lines) + "\n")
    with open(os.path.join(out, "bytes.txt"), "w") as f:
        f.write(" ".join(str(len(n)) for r in res for n in r.nals) + "\n")
    print("dumped", spy.n, "slices to", out)


if __name__ == "__main__":
    main()
