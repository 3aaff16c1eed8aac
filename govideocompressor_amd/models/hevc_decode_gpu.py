"""Batched HEVC decode on MI355X: host CABAC parse (general Main / Main 10) + gfx950
reconstruction.

The reference worker decodes whatever its piece holds with ``ffmpeg -i <idx>.mp4``
(client.go:115) and its splitter stream-copies any codec (server.go:199-201).  Here an
HEVC transcode decodes many segments at once:

1. **parse** (``_host.hevc_parse``, csrc/host/hevc_dec.cc; one C++ thread per segment, GIL
   released): CABAC, merge / AMVP / TMVP, reference lists, weights, QPs, boundary
   strengths and SAO parameters resolved into flat records;
2. **upload**: one picture step's records of every slot packed into one pinned buffer, one
   host-to-device copy;
3. **reconstruct** (csrc/kernels/hevc_decode.hip): residuals (one wave per transform block),
   inter prediction (one wave per 8x8 block, from a per-slot decoded picture buffer), intra
   prediction in CTB wavefront order, deblocking, SAO -- writing straight into the
   ``[segments, frames, H, W]`` device tensors the encoder consumes.

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


class _Packer:
    """One picture step's records of every slot in one pinned buffer (16-byte aligned
    sections), uploaded with a single copy; ``ptr(name)`` gives each section's device address."""

    def __init__(self):
        self.parts: list[tuple[str, np.ndarray]] = []

    def add(self, name: str, arr: np.ndarray):
        self.parts.append((name, np.ascontiguousarray(arr)))

    def upload(self, dev, stream_pool: list) -> tuple[torch.Tensor, dict[str, int]]:
        offs, total = {}, 0
        for name, a in self.parts:
            offs[name] = total
            total += (a.nbytes + 15) // 16 * 16
        total = max(total, 16)
        host = torch.empty(total, dtype=torch.uint8).pin_memory()
        hn = host.numpy()
        for name, a in self.parts:
            o = offs[name]
            hn[o:o + a.nbytes] = a.view(np.uint8).reshape(-1)
        d = host.to(dev, non_blocking=True)
        stream_pool.append(host)  # keep the pinned source alive until the stream has read it
        base = d.data_ptr()
        return d, {k: base + v for k, v in offs.items()}


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

    def parse(self, segments: list[bytes]) -> list[dict]:
        """Host stage (GIL released, one C++ thread per segment): the GPU records."""
        return self.host.hevc_parse(list(segments), self.threads, False)

    def reconstruct(self, parsed: list[dict], fps: float = 30.0, out_dtype=None) -> list[DecodedSegment]:
        """GPU stage: parsed segments -> device frames (display order)."""
        for i, s in enumerate(parsed):
            if s.get("error"):
                raise ValueError(f"HEVC segment {i}: {s['error']}")
            if s["n"] == 0:
                raise ValueError(f"HEVC segment {i}: no pictures")
        out: list[DecodedSegment | None] = [None] * len(parsed)
        groups: dict[tuple, list[int]] = {}
        for i, s in enumerate(parsed):
            m = s["meta"][0]
            key = tuple(int(m[HM[k]]) for k in ("W", "H", "width", "height", "crop_x", "crop_y", "bd", "bdc", "log2_ctb"))
            groups.setdefault(key, []).append(i)
        for key, idxs in groups.items():
            for i, d in zip(idxs, self._decode_group(key, [parsed[i] for i in idxs], fps, out_dtype)):
                out[i] = d
        if len(groups) > 1:
            self.last_batch = None  # several geometries: no single [B, F] batch tensor
        return out  # type: ignore[return-value]

    # ------------------------------------------------------------------ internals
    def _decode_group(self, key: tuple, segs: list[dict], fps: float, out_dtype) -> list[DecodedSegment]:
        W, H, w, h, cx, cy, bd, bdc, log2_ctb = key
        dev = self.dev
        B = len(segs)
        ctb = 1 << log2_ctb
        wctb, hctb = -(-W // ctb), -(-H // ctb)
        nctb = wctb * hctb
        h4, w4 = H // 4, W // 4
        plans = []
        for s in segs:
            pl = hevc_dpb_schedule(s["ref_ids"], s["meta"][:, HM["decode_idx"]])
            if pl is None:
                raise ValueError("HEVC segment: a reference picture is not available in decoding order")
            plans.append(pl)
        D = max(pl[2] for pl in plans)
        F = max(int(s["n"]) for s in segs)
        nout = [int(np.sum(s["display"] >= 0)) for s in segs]
        Fo = max(max(nout), 1)
        if out_dtype is None:
            out_dtype = torch.uint8 if bd == 8 else torch.int16
        pdt = torch.int16  # samples (<= 10 bits) in int16 tensors, read as uint16 by the kernels
        dpb = [torch.zeros((B, D, H, W), dtype=pdt, device=dev), torch.zeros((B, D, H // 2, W // 2), dtype=pdt, device=dev),
               torch.zeros((B, D, H // 2, W // 2), dtype=pdt, device=dev)]
        res = [torch.zeros((B, H, W), dtype=torch.int16, device=dev),
               torch.zeros((B, H // 2, W // 2), dtype=torch.int16, device=dev),
               torch.zeros((B, H // 2, W // 2), dtype=torch.int16, device=dev)]
        tmp = [torch.empty_like(r) for r in res]
        # display-size contiguous output: the encoder's [B, F, h, w] input
        y_out = torch.empty((B, Fo, h, w), dtype=out_dtype, device=dev)
        u_out = torch.empty((B, Fo, h // 2, w // 2), dtype=out_dtype, device=dev)
        v_out = torch.empty_like(u_out)
        crop = ((cy, cy + h, cx, cx + w), (cy // 2, (cy + h) // 2, cx // 2, (cx + w) // 2))
        err = torch.zeros((1,), dtype=torch.int32, device=dev)
        stream = torch.cuda.current_stream(dev)
        s_ = stream.cuda_stream
        keep: list = []
        zmvf = np.zeros((h4, w4, 12), np.uint8)
        zbs = np.zeros((h4, w4), np.uint8)
        zctb = np.zeros((nctb, 8), np.uint8)
        zsao = np.zeros((nctb, 24), np.uint8)
        zmeta = np.zeros(24, np.int32)
        any_scaling = any(s["scaling"].size for s in segs)
        for t in range(F):
            act = [j for j, s in enumerate(segs) if t < int(s["n"])]
            run = np.zeros(B, np.int8)
            run[act] = 1
            cur = np.zeros(B, np.int8)
            reftab = np.full((B, 16), -1, np.int8)
            meta = np.zeros((B, 24), np.int32)
            tu_base = np.zeros(B + 1, np.int32)
            coef_base = np.zeros(B, np.int64)
            op_base = np.zeros(B, np.int32)
            ref_base = np.zeros(B, np.int32)
            slice_base = np.zeros(B, np.int32)
            ctb_ops = np.zeros((B, nctb + 1), np.uint32)
            mvfs, bss, ctbs, saos, tus, coefs, ops, refs, slices, scal = [], [], [], [], [], [], [], [], [], []
            ntu = ncoef = nop = nref = nsl = 0
            max_tus = 0
            for j, s in enumerate(segs):
                if run[j]:
                    cur[j] = plans[j][0][t]
                    reftab[j] = plans[j][1][t]
                    meta[j] = s["meta"][t]
                    mvfs.append(s["mvf"][t])
                    bss.append(s["bs"][t])
                    ctbs.append(s["ctbs"][t])
                    saos.append(s["sao"][t])
                    a, e = int(s["tu_off"][t]), int(s["tu_off"][t + 1])
                    tus.append(s["tus"][a:e])
                    c0, c1 = int(s["coef_off"][t]), int(s["coef_off"][t + 1])
                    coefs.append(s["coefs"][c0:c1])
                    o0, o1 = int(s["op_off"][t]), int(s["op_off"][t + 1])
                    ops.append(s["ops"][o0:o1])
                    r0, r1 = int(s["ref_off"][t]), int(s["ref_off"][t + 1])
                    refs.append(s["refs"][r0:r1])
                    s0, s1 = int(s["slice_off"][t]), int(s["slice_off"][t + 1])
                    slices.append(s["slices"][s0:s1])
                    ctb_ops[j] = s["ctb_ops"][t]
                    if any_scaling:
                        scal.append(s["scaling"][t] if s["scaling"].size else np.full(SCALING_BYTES, 16, np.uint8))
                    tu_base[j] = ntu
                    coef_base[j] = ncoef
                    op_base[j] = nop
                    ref_base[j] = nref
                    slice_base[j] = nsl
                    ntu += e - a
                    ncoef += c1 - c0
                    nop += o1 - o0
                    nref += r1 - r0
                    nsl += s1 - s0
                    max_tus = max(max_tus, e - a)
                else:
                    tu_base[j] = ntu
                    meta[j] = zmeta
                    mvfs.append(zmvf)
                    bss.append(zbs)
                    ctbs.append(zctb)
                    saos.append(zsao)
                    if any_scaling:
                        scal.append(np.full(SCALING_BYTES, 16, np.uint8))
            tu_base[B] = ntu
            pk = _Packer()
            for name, arr in (("run", run), ("cur", cur), ("reftab", reftab), ("meta", meta), ("tu_base", tu_base),
                              ("coef_base", coef_base), ("op_base", op_base), ("ref_base", ref_base),
                              ("slice_base", slice_base), ("ctb_ops", ctb_ops), ("mvf", np.stack(mvfs)),
                              ("bs", np.stack(bss)), ("ctbs", np.stack(ctbs)), ("sao", np.stack(saos)),
                              ("tus", np.concatenate(tus) if tus else np.zeros((0, 12), np.uint8)),
                              ("coefs", np.concatenate(coefs) if coefs else np.zeros(0, np.int16)),
                              ("ops", np.concatenate(ops) if ops else np.zeros((0, 12), np.uint8)),
                              ("refs", np.concatenate(refs) if refs else np.zeros((0, 16), np.uint8)),
                              ("slices", np.concatenate(slices) if slices else np.zeros((0, 8), np.uint8))):
                pk.add(name, arr)
            if any_scaling:
                pk.add("scaling", np.stack(scal))
            dbuf, ptr = pk.upload(dev, keep)
            keep.append(dbuf)
            params = dict(B=B, W=W, H=H, D=D, bd=bd, bdc=bdc, log2_ctb=log2_ctb, wctb=wctb, hctb=hctb,
                          dpb=[x.data_ptr() for x in dpb], res=[x.data_ptr() for x in res],
                          tmp=[x.data_ptr() for x in tmp], max_tus=max_tus, err=err.data_ptr(), **ptr)
            if not any_scaling:
                params["scaling"] = 0
            for r in res:
                r.zero_()
            self.hip.hevc_decode_stage(params, 0, s_)
            self.hip.hevc_decode_stage(params, 1, s_)
            self.hip.hevc_decode_stage(params, 2, s_)
            if np.any(meta[act, HM["deblock_any"]]):
                self.hip.hevc_decode_stage(params, 3, s_)
                self.hip.hevc_decode_stage(params, 4, s_)
            bi = torch.from_numpy(np.array(act, np.int64)).to(dev)
            ci = torch.from_numpy(cur[act].astype(np.int64)).to(dev)
            if np.any(meta[act, HM["sao_any"]]):
                for c in range(3):
                    tmp[c][bi] = dpb[c][bi, ci]
                self.hip.hevc_decode_stage(params, 5, s_)
            disp = np.array([int(segs[j]["display"][t]) for j in act], np.int64)
            sel = disp >= 0
            if np.any(sel):
                bo = bi[torch.from_numpy(sel).to(dev)]
                co = ci[torch.from_numpy(sel).to(dev)]
                do = torch.from_numpy(disp[sel]).to(dev)
                for k, (o_, p_) in enumerate(zip((y_out, u_out, v_out), dpb)):
                    r0, r1, c0, c1 = crop[min(k, 1)]
                    o_[bo, do] = p_[bo, co][:, r0:r1, c0:c1].to(out_dtype)
            if len(keep) > 64:  # bound the pinned staging held for in-flight copies
                stream.synchronize()
                keep.clear()
        e = int(err.item())
        if e != 0:
            raise RuntimeError(f"GPU HEVC decode failed (err={e:#x}: 16 = reference outside the DPB, "
                               "1 = wavefront progress timeout)")
        keep.clear()
        res_out = []
        for j in range(B):
            n = nout[j]
            res_out.append(DecodedSegment(y_out[j, :n], u_out[j, :n], v_out[j, :n], fps, "gpu"))
        self.last_batch = (y_out, u_out, v_out)
        return res_out
