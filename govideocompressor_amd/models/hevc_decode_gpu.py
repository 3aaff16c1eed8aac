"""Batched HEVC decode on MI355X: host CABAC parse (general Main / Main 10) + gfx950
reconstruction.

The reference worker decodes whatever its piece holds with ``ffmpeg -i <idx>.mp4``
(client.go:115) and its splitter stream-copies any codec (server.go:199-201).  Here an
HEVC transcode decodes many segments at once:

1. **parse** (``_host.hevc_parse``, csrc/host/hevc_dec.cc; one C++ thread per segment, GIL
   released): CABAC, merge / AMVP / TMVP, reference lists, weights, QPs, boundary
   strengths and SAO parameters resolved into flat records;
2. **pack + upload**: one picture step's records of every slot laid out by C++ in a pinned
   buffer (csrc/host/decode_batch.cc), copied on a side stream while the previous step
   reconstructs;
3. **reconstruct** (csrc/kernels/hevc_decode.hip): residuals (one wave per transform block),
   inter prediction (one wave per 8x8 block, from a per-slot decoded picture buffer), intra
   prediction in CTB wavefront order, deblocking, SAO, and an emit stage that writes each
   picture (cropped, converted) to its display position of the ``[segments, frames, H, W]``
   device tensors the encoder consumes.

Output frames land in display order (coded video sequence, then POC); pictures with
``pic_output_flag`` 0 and RASL pictures of a CRA that starts a segment are not output.
The CPU reconstruction of the same parse (``hevc_decode_full``) is the bit-exact oracle
of ``tests/test_gpu_hevc_decode.py``.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch

from ..ops import native
from .h264_decode_gpu import DecodedSegment

# meta columns of _host.hevc_parse (csrc/kernels/hevc_decode.h HevcMeta)
META = ("decode_idx", "poc", "cvs", "output", "irap", "idr", "slice_type", "slice_qp", "W", "H", "width", "height",
        "crop_x", "crop_y", "bd", "bdc", "log2_ctb", "constrained_intra", "strong_intra", "lf_across_tiles",
        "cb_qp_off", "cr_qp_off", "deblock_any", "sao_any")
HM = {k: i for i, k in enumerate(META)}
SCALING_BYTES = 8160


def hevc_dpb_schedule(ref_ids: np.ndarray, decode_idx: np.ndarray, max_buffers: int = 24):
    """Buffer plan of one segment (decoding order): (cur [P] buffer of each picture,
    reftab [P, 16] buffer of every ref_ids entry or -1, buffers used), or None when a
    reference is not held.  A picture keeps its buffer until the last picture that
    references it has been decoded (its output copy happens right after its own decode)."""
    P = len(decode_idx)
    last = {int(i): p for p, i in enumerate(decode_idx)}
    for p in range(P):
        for i in ref_ids[p]:
            if i >= 0:
                last[int(i)] = max(last.get(int(i), p), p)
    free = list(range(max_buffers))[::-1]
    held: dict[int, int] = {}
    cur = np.zeros(P, np.int8)
    reftab = np.full((P, 16), -1, np.int8)
    used = 0
    for p in range(P):
        for k, i in enumerate(ref_ids[p]):
            if i >= 0:
                if int(i) not in held:
                    return None
                reftab[p, k] = held[int(i)]
        if not free:
            return None
        b = free.pop()
        cur[p] = b
        held[int(decode_idx[p])] = b
        used = max(used, len(held))
        for i in [i for i, _ in held.items() if last.get(i, -1) <= p]:
            free.append(held.pop(i))
    return cur, reftab, max(used, 1)


class GpuHevcDecoder:
    """Decode lists of Annex-B HEVC segments into device tensors."""

    def __init__(self, device=None, threads: int | None = None):
        if not torch.cuda.is_available():
            raise RuntimeError("GpuHevcDecoder needs a GPU")
        self.dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.dev.index is None:
            self.dev = torch.device("cuda", torch.cuda.current_device())
        self.hip = native.hip()
        self.host = native.host()
        self.threads = threads or min(16, os.cpu_count() or 4)
        self.stats: dict[str, float] = {}

    # ------------------------------------------------------------------ public
    def decode(self, segments: list[bytes], fps: float = 30.0, out_dtype=None) -> list[DecodedSegment]:
        """``out_dtype``: torch.uint8 for 8-bit content (the default), int16 holding
        bit_depth-bit samples otherwise."""
        t0 = time.perf_counter()
        parsed = self.parse(segments)
        t1 = time.perf_counter()
        out = self.reconstruct(parsed, fps, out_dtype)
        self.stats = {"parse_s": t1 - t0, "gpu_s": time.perf_counter() - t1, "segments_gpu": len(segments)}
        return out

    def parse(self, segments: list[bytes]):
        """Host stage (GIL released, one C++ thread per segment): the GPU records, kept in a
        C++ ``HevcBatch`` (csrc/host/decode_batch.cc)."""
        return self.host.hevc_parse_batch(list(segments), self.threads)

    def reconstruct(self, batch, fps: float = 30.0, out_dtype=None) -> list[DecodedSegment]:
        """GPU stage: parsed segments -> device frames (display order)."""
        infos = [batch.info(i) for i in range(len(batch))]
        for i, s in enumerate(infos):
            if s.get("error"):
                raise ValueError(f"HEVC segment {i}: {s['error']}")
            if s["n"] == 0:
                raise ValueError(f"HEVC segment {i}: no pictures")
        out: list[DecodedSegment | None] = [None] * len(infos)
        groups: dict[tuple, list[int]] = {}
        for i, s in enumerate(infos):
            m = s["meta"][0]
            key = tuple(int(m[HM[k]]) for k in ("W", "H", "width", "height", "crop_x", "crop_y", "bd", "bdc", "log2_ctb"))
            groups.setdefault(key, []).append(i)
        for key, idxs in groups.items():
            for i, d in zip(idxs, self._decode_group(key, batch, idxs, [infos[i] for i in idxs], fps, out_dtype)):
                out[i] = d
        if len(groups) > 1:
            self.last_batch = None  # several geometries: no single [B, F] batch tensor
        return out  # type: ignore[return-value]

    # ------------------------------------------------------------------ internals
    def _staging(self, cap: int) -> list[tuple[torch.Tensor, torch.Tensor]]:
        """Two (pinned host, device) step buffers of at least ``cap`` bytes, kept across calls."""
        st = getattr(self, "_stage", None)
        if st is None or st[0][0].numel() < cap:
            cap = (cap + (1 << 20) - 1) // (1 << 20) * (1 << 20)
            st = [(torch.empty(cap, dtype=torch.uint8, pin_memory=True),
                   torch.empty(cap, dtype=torch.uint8, device=self.dev)) for _ in range(2)]
            self._stage = st
        return st

    _SECTIONS = ("meta", "tu_base", "coef_base", "op_base", "ref_base", "slice_base", "ctb_ops", "mvf", "mvf_sub", "bs", "ctbs",
                 "sao", "tus", "coefs", "ops", "refs", "slices")

    def _decode_group(self, key: tuple, batch, idxs: list[int], infos: list[dict], fps: float,
                      out_dtype) -> list[DecodedSegment]:
        """One batch of same-geometry segments.  Each picture step of every slot is packed by
        C++ into a pinned buffer (``HevcBatch.pack``) and copied on a side stream while the
        previous step reconstructs; the emit stage writes each picture (cropped, converted)
        to its display position of the output."""
        W, H, w, h, cx, cy, bd, bdc, log2_ctb = key
        dev = self.dev
        B = len(idxs)
        ctb = 1 << log2_ctb
        wctb, hctb = -(-W // ctb), -(-H // ctb)
        plans = []
        for s in infos:
            pl = hevc_dpb_schedule(s["ref_ids"], s["meta"][:, HM["decode_idx"]])
            if pl is None:
                raise ValueError("HEVC segment: a reference picture is not available in decoding order")
            plans.append(pl)
        D = max(pl[2] for pl in plans)
        ns = [int(s["n"]) for s in infos]
        F = max(ns)
        nout = [int(np.sum(s["display"] >= 0)) for s in infos]
        Fo = max(max(nout), 1)
        if out_dtype is None:
            out_dtype = torch.uint8 if bd == 8 else torch.int16
        if out_dtype == torch.uint8 and bd != 8:
            raise ValueError("uint8 output needs 8-bit content")
        # per-step slot tables, uploaded once: run, DPB buffer, reference buffers, output position
        run = np.zeros((F, B), np.int8)
        cur = np.zeros((F, B), np.int8)
        reftab = np.full((F, B, 16), -1, np.int8)
        disp = np.full((F, B), -1, np.int16)
        for j, s in enumerate(infos):
            n = ns[j]
            run[:n, j] = 1
            cur[:n, j] = plans[j][0]
            reftab[:n, j] = plans[j][1]
            disp[:n, j] = s["display"]
        d_run = torch.from_numpy(run).to(dev)
        d_cur = torch.from_numpy(cur).to(dev)
        d_reftab = torch.from_numpy(reftab).to(dev)
        d_disp = torch.from_numpy(disp).to(dev)
        slots = [[idxs[j] if t < ns[j] else -1 for j in range(B)] for t in range(F)]
        layouts = [batch.layout(t, slots[t]) for t in range(F)]
        stage = self._staging(max(L["total"] for L in layouts))
        cap = stage[0][0].numel()
        pdt = torch.int16  # samples (<= 10 bits) in int16 tensors, read as uint16 by the kernels
        dpb = [torch.empty((B, D, H, W), dtype=pdt, device=dev), torch.empty((B, D, H // 2, W // 2), dtype=pdt, device=dev),
               torch.empty((B, D, H // 2, W // 2), dtype=pdt, device=dev)]
        res = [torch.zeros((B, H, W), dtype=torch.int16, device=dev),
               torch.zeros((B, H // 2, W // 2), dtype=torch.int16, device=dev),
               torch.zeros((B, H // 2, W // 2), dtype=torch.int16, device=dev)]
        tmp = [torch.empty_like(r) for r in res]
        # display-size contiguous output: the encoder's [B, F, h, w] input
        y_out = torch.empty((B, Fo, h, w), dtype=out_dtype, device=dev)
        u_out = torch.empty((B, Fo, h // 2, w // 2), dtype=out_dtype, device=dev)
        v_out = torch.empty_like(u_out)
        err = torch.zeros((1,), dtype=torch.int32, device=dev)
        comp = torch.cuda.current_stream(dev)
        copy = getattr(self, "_copy_stream", None)
        if copy is None:
            copy = self._copy_stream = torch.cuda.Stream(dev)
        copied = [torch.cuda.Event(), torch.cuda.Event()]
        consumed = [torch.cuda.Event(), torch.cuda.Event()]
        for k in range(2):
            consumed[k].record(comp)
        s_ = comp.cuda_stream
        base_params = dict(B=B, W=W, H=H, D=D, bd=bd, bdc=bdc, log2_ctb=log2_ctb, wctb=wctb, hctb=hctb,
                           dpb=[x.data_ptr() for x in dpb], res=[x.data_ptr() for x in res],
                           tmp=[x.data_ptr() for x in tmp], err=err.data_ptr(),
                           out=[y_out.data_ptr(), u_out.data_ptr(), v_out.data_ptr()],
                           out_u8=int(out_dtype == torch.uint8), Fo=Fo, out_w=w, out_h=h, crop_x=cx, crop_y=cy)
        for t in range(F):
            k = t & 1
            host_buf, dev_buf = stage[k]
            L = layouts[t]
            copied[k].synchronize()            # the copy of step t - 2 has read host_buf
            batch.pack(t, slots[t], host_buf.data_ptr(), cap, 8)
            with torch.cuda.stream(copy):
                copy.wait_event(consumed[k])   # step t - 2's kernels are done with dev_buf
                dev_buf[:L["total"]].copy_(host_buf[:L["total"]], non_blocking=True)
                copied[k].record(copy)
            comp.wait_event(copied[k])
            base = dev_buf.data_ptr()
            params = dict(base_params, max_tus=int(L["max_tus"]), run=d_run[t].data_ptr(), cur=d_cur[t].data_ptr(),
                          reftab=d_reftab[t].data_ptr(), disp=d_disp[t].data_ptr(),
                          scaling=base + int(L["scaling"]) if L["scaling_on"] else 0,
                          **{n: base + int(L[n]) for n in self._SECTIONS})
            self.hip.hevc_decode_stage(params, 0, s_)
            self.hip.hevc_decode_stage(params, 1, s_)
            self.hip.hevc_decode_stage(params, 2, s_)
            if L["deblock_any"]:
                self.hip.hevc_decode_stage(params, 3, s_)
                self.hip.hevc_decode_stage(params, 4, s_)
            if L["sao_any"]:
                self.hip.hevc_decode_stage(params, 7, s_)
                self.hip.hevc_decode_stage(params, 5, s_)
            self.hip.hevc_decode_stage(params, 6, s_)
            consumed[k].record(comp)
            if t + 1 < F:
                for r in res:
                    r.zero_()
        e = int(err.item())
        if e != 0:
            raise RuntimeError(f"GPU HEVC decode failed (err={e:#x}: 16 = reference outside the DPB, "
                               "1 = wavefront progress timeout)")
        res_out = [DecodedSegment(y_out[j, :nout[j]], u_out[j, :nout[j]], v_out[j, :nout[j]], fps, "gpu")
                   for j in range(B)]
        self.last_batch = (y_out, u_out, v_out)
        return res_out
