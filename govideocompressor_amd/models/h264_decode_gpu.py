"""Batched H.264 decode on MI355X: host entropy decode (CAVLC / CABAC) + gfx950 reconstruction.

The reference worker decodes its piece with ffmpeg before re-encoding
(client.go:115-118 ``ffmpeg -i <idx>.mp4 <args> <out>``).  Here a transcode
decodes many closed-GOP segments at once:

1. **parse** (host C++, one thread per segment, GIL released): CAVLC -> per-MB
   ``MbHeader`` records + packed non-zero levels (``_host.parse``); this is the only
   inherently serial part of H.264 decoding (bit-serial entropy coding);
2. **upload**: all records of the batch in one host->device copy per array;
3. **reconstruct** (``decode.hip``): picture ``t`` of every segment in one launch
   pair -- inter MBs in parallel over (MB, segment), intra MBs in wavefront order,
   then the encoder's deblocking kernel -- writing straight into the
   ``[segments, frames, H, W]`` device tensors the encoder consumes, so decoded
   pixels never cross PCIe.

P and B pictures reconstruct from a per-slot decoded picture buffer ([B, D] pictures on
the device, :func:`dpb_schedule`): the parser hands over every 4x4 block's vectors and
reference indices (sub-8x8 partitions, B_8x8, spatial / temporal direct resolved),
the reference lists as picture ids, the weighted-prediction table (explicit or
implicit) and the deblocking boundary strengths; High-profile 8x8 transforms are
inverse-transformed on the GPU.  Output frames land in display (POC) order.

Segments the GPU path does not cover (I_PCM, Intra8x8, several slices, constrained intra
prediction, mmco 5, per-picture filter parameters that differ from the batch) are decoded
by the CPU decoder instead (``h264_decoder.cc``) and uploaded; the result is identical
either way (the CPU decoder is the bit-exact oracle of ``tests/test_gpu_decode.py``).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np
import torch

from ..ops import native


@dataclass
class DecodedSegment:
    """Decoded frames of one segment on the device: y [F, h, w], u/v [F, h/2, w/2]
    (display size, cropped views of the coded planes)."""
    y: torch.Tensor
    u: torch.Tensor
    v: torch.Tensor
    fps: float = 30.0
    path: str = "gpu"  # "gpu" or "cpu" (fallback decoder)

    @property
    def frames(self) -> int:
        return int(self.y.shape[0])

    @property
    def width(self) -> int:
        return int(self.y.shape[2])

    @property
    def height(self) -> int:
        return int(self.y.shape[1])


_META = ("pic_id", "ref_id", "nal_ref", "idr", "slice_type", "slice_qp", "alpha", "beta", "cqp", "deblock", "gpu_ok",
         "poc")
M = {k: i for i, k in enumerate(_META)}


def _gpu_plan(seg: dict) -> tuple[bool, str]:
    """Can the GPU path reconstruct this parsed segment?"""
    if seg.get("error"):
        return False, seg["error"]
    if seg["n"] == 0:
        return False, "no pictures"
    if not np.all(seg["meta"][:, M["gpu_ok"]] == 1):
        return False, "unsupported coding tools"
    return True, ""


def dpb_schedule(meta: np.ndarray, lists: np.ndarray, max_buffers: int = 32):
    """Decoded-picture-buffer plan of one segment (decode order).

    Returns (cur [P] buffer of each picture, reftab [P, 2, 32] buffer of RefPicListX[i]
    or -1, display [P] output position, buffers used) or None when a list names a picture
    that is not held.  A picture keeps its buffer until the last picture whose lists name
    it; the output copy happens right after its own decode."""
    P = meta.shape[0]
    ids = meta[:, M["pic_id"]].astype(np.int64)
    last = {int(i): p for p, i in enumerate(ids)}
    for p in range(P):
        for i in lists[p].reshape(-1):
            if i >= 0:
                last[int(i)] = max(last.get(int(i), p), p)
    free = list(range(max_buffers))[::-1]
    held: dict[int, int] = {}
    cur = np.zeros(P, np.int8)
    reftab = np.full((P, 2, 32), -1, np.int8)
    used = 0
    for p in range(P):
        for l in range(2):
            for k in range(32):
                i = int(lists[p, l, k])
                if i >= 0:
                    if i not in held:
                        return None
                    reftab[p, l, k] = held[i]
        if not free:
            return None
        b = free.pop()
        cur[p] = b
        held[int(ids[p])] = b
        used = max(used, len(held))
        for i in [i for i, _ in held.items() if last.get(i, -1) <= p]:
            free.append(held.pop(i))
    # display order: IDR epochs, then POC
    epoch = np.cumsum(meta[:, M["idr"]] != 0)
    order = np.lexsort((meta[:, M["poc"]], epoch))
    display = np.empty(P, np.int64)
    display[order] = np.arange(P)
    return cur, reftab, display, max(used, 1)


class GpuH264Decoder:
    """Decode lists of Annex-B segments into device tensors."""

    def __init__(self, device=None, threads: int | None = None):
        if not torch.cuda.is_available():
            raise RuntimeError("GpuH264Decoder needs a GPU")
        self.dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.dev.index is None:
            self.dev = torch.device("cuda", torch.cuda.current_device())
        self.hip = native.hip()
        self.host = native.host()
        self.threads = threads or min(16, os.cpu_count() or 4)
        self.stats: dict[str, float] = {}

    # ------------------------------------------------------------------ public
    def decode(self, segments: list[bytes], fps: float = 30.0) -> list[DecodedSegment]:
        import time
        t0 = time.perf_counter()
        parsed = self.parse(segments)
        t1 = time.perf_counter()
        out = self.reconstruct(parsed, fps)
        self.stats["parse_s"] = t1 - t0
        return out

    def parse(self, segments: list[bytes]):
        """Host stage (GIL released, one C++ thread per segment): entropy decode."""
        return list(segments), self.host.parse(list(segments), self.threads)

    def reconstruct(self, parsed_in, fps: float = 30.0) -> list[DecodedSegment]:
        """GPU stage (+ the CPU decoder for segments the GPU path does not cover)."""
        import time
        segments, parsed = parsed_in
        t1 = time.perf_counter()
        out: list[DecodedSegment | None] = [None] * len(segments)
        ok, fallback = [], []
        for i, seg in enumerate(parsed):
            good, why = _gpu_plan(seg)
            (ok if good else fallback).append(i)
        # one batch per coded geometry + filter parameters; the rest decode on the CPU
        groups: dict[tuple, list[int]] = {}
        for i in ok:
            s = parsed[i]
            m = s["meta"]
            params = {(int(r[M["alpha"]]), int(r[M["beta"]]), int(r[M["cqp"]]), int(r[M["deblock"]])) for r in m}
            if len(params) != 1:
                fallback.append(i)
                continue
            key = (s["coded_width"], s["coded_height"], s["width"], s["height"], s["crop_x"], s["crop_y"], params.pop())
            groups.setdefault(key, []).append(i)
        for key, idxs in groups.items():
            got = self._decode_group(key, [parsed[i] for i in idxs], fps)
            if got is None:
                fallback += idxs
                continue
            for i, d in zip(idxs, got):
                out[i] = d
        t2 = time.perf_counter()
        for i in fallback:
            out[i] = self._cpu_decode(segments[i], fps)
        self.stats = {"gpu_s": t2 - t1, "cpu_fallback_s": time.perf_counter() - t2,
                      "segments_gpu": len(segments) - len(fallback), "segments_cpu": len(fallback)}
        if fallback or len(groups) != 1:
            self.last_batch = None  # not one [B, F] batch tensor
        return out  # type: ignore[return-value]

    # ------------------------------------------------------------------ internals
    def _cpu_decode(self, data: bytes, fps: float) -> DecodedSegment:
        pics = self.host.decode(data)
        if not pics:
            raise ValueError("segment holds no pictures")
        w, h = pics[0]["width"], pics[0]["height"]
        buf = np.concatenate([p["i420"] for p in pics]).reshape(len(pics), -1)
        ys = w * h
        cs = (w // 2) * (h // 2)
        t = torch.from_numpy(buf).to(self.dev)
        y = t[:, :ys].reshape(len(pics), h, w)
        u = t[:, ys:ys + cs].reshape(len(pics), h // 2, w // 2)
        v = t[:, ys + cs:].reshape(len(pics), h // 2, w // 2)
        return DecodedSegment(y, u, v, fps, "cpu")

    def _decode_group(self, key: tuple, segs: list[dict], fps: float) -> list[DecodedSegment] | None:
        """Decode one batch of same-geometry segments; None if a DPB plan fails (CPU then)."""
        Wc, Hc, w, h, cx, cy, (alpha, beta, cqp, deblock) = key
        dev = self.dev
        wmb, hmb = Wc // 16, Hc // 16
        nmb = wmb * hmb
        B = len(segs)
        F = max(int(s["n"]) for s in segs)
        plans = [dpb_schedule(s["meta"], s["lists"]) for s in segs]
        if any(pl is None for pl in plans):
            return None
        D = max(pl[3] for pl in plans)
        # ---- per picture-step tables, [F, B, ...]
        hdr = np.zeros((F, B, nmb, 64), np.uint8)
        mask = np.zeros((F, B, nmb), np.uint32)
        off = np.zeros((F, B, nmb), np.uint32)
        run = np.zeros((F, B), np.int8)
        cur = np.zeros((F, B), np.int8)
        reftab = np.full((F, B, 2, 32), -1, np.int8)
        disp = np.zeros((F, B), np.int64)
        wp = np.zeros((F, B, 516), np.int16)
        base = 0
        coefs = []
        for j, s in enumerate(segs):
            Pn = int(s["n"])
            c_, r_, d_, _ = plans[j]
            hdr[:Pn, j] = s["hdr"]
            mask[:Pn, j] = s["mask"]
            off[:Pn, j] = s["off"] + (s["pic_off"][:Pn, None] + base).astype(np.uint32)
            st = s["meta"][:, M["slice_type"]] % 5
            run[:Pn, j] = np.where(st == 2, 1, 2)
            cur[:Pn, j] = c_
            reftab[:Pn, j] = r_
            disp[:Pn, j] = d_
            wp[:Pn, j] = s["wp"]
            coefs.append(s["coef"])
            base += int(s["pic_off"][Pn])
        if base >= 2 ** 32:
            raise ValueError("level array too large for 32-bit block offsets")
        coef = np.concatenate(coefs) if coefs else np.zeros(16, np.int16)
        if coef.size == 0:
            coef = np.zeros(16, np.int16)
        d_hdr = torch.from_numpy(hdr).to(dev)
        d_mask = torch.from_numpy(mask.view(np.int32)).to(dev)
        d_off = torch.from_numpy(off.view(np.int32)).to(dev)
        d_coef = torch.from_numpy(coef).to(dev)
        d_run = torch.from_numpy(run).to(dev)
        d_cur = torch.from_numpy(cur).to(dev)
        d_reftab = torch.from_numpy(reftab).to(dev)
        d_wp = torch.from_numpy(wp).to(dev)
        # ---- output tensors (display size, contiguous: the encoder's [B, F, h, w] input) and
        # the per-slot decoded picture buffers
        y_out = torch.empty((B, F, h, w), dtype=torch.uint8, device=dev)
        u_out = torch.empty((B, F, h // 2, w // 2), dtype=torch.uint8, device=dev)
        v_out = torch.empty_like(u_out)
        crop = ((cy, cy + h, cx, cx + w), (cy // 2, (cy + h) // 2, cx // 2, (cx + w) // 2))
        dpb = [torch.zeros((B, D, Hc, Wc), dtype=torch.uint8, device=dev),
               torch.zeros((B, D, Hc // 2, Wc // 2), dtype=torch.uint8, device=dev),
               torch.zeros((B, D, Hc // 2, Wc // 2), dtype=torch.uint8, device=dev)]
        nz = torch.zeros((B, nmb, 16), dtype=torch.uint8, device=dev)
        err = torch.zeros((1,), dtype=torch.int32, device=dev)
        s_ = torch.cuda.current_stream(dev).cuda_stream
        P_ = lambda t: t.data_ptr()  # noqa: E731
        zero_mv = np.zeros((2, nmb, 16, 2), np.int16)
        none_ref = np.full((2, nmb, 16), -1, np.int8)
        zero_bs = np.zeros((nmb, 32), np.uint8)
        for t in range(F):
            active = run[t] != 0
            any_inter = bool(np.any(run[t] == 2))
            mv_t = np.stack([sg["mv"][t] if t < int(sg["n"]) else zero_mv for sg in segs])
            ref_t = np.stack([sg["ref"][t] if t < int(sg["n"]) else none_ref for sg in segs])
            d_mv = torch.from_numpy(mv_t).to(dev)
            d_ref = torch.from_numpy(ref_t).to(dev)
            self.hip.decode_picture_dpb(B, wmb, hmb, D, P_(dpb[0]), P_(dpb[1]), P_(dpb[2]), P_(d_cur[t]),
                                        P_(d_reftab[t]), P_(d_wp[t]), P_(d_mv), P_(d_ref), P_(d_hdr[t]), P_(d_mask[t]),
                                        P_(d_off[t]), P_(d_coef), P_(d_run[t]), int(any_inter), cqp, P_(nz), P_(err), s_)
            if deblock:
                bs_t = np.stack([sg["bs"][t] if t < int(sg["n"]) else zero_bs for sg in segs])
                d_bs = torch.from_numpy(bs_t).to(dev)
                self.hip.deblock_dpb(B, wmb, hmb, D, P_(dpb[0]), P_(dpb[1]), P_(dpb[2]), P_(d_cur[t]), P_(d_hdr[t]),
                                     P_(nz), P_(d_bs), cqp, alpha, beta, P_(err), s_)
            sel = np.nonzero(active)[0]
            bi = torch.from_numpy(sel).to(dev)
            di = torch.from_numpy(disp[t, sel]).to(dev)
            ci = torch.from_numpy(cur[t, sel].astype(np.int64)).to(dev)
            for k, (o_, p_) in enumerate(zip((y_out, u_out, v_out), dpb)):
                r0, r1, c0, c1 = crop[min(k, 1)]
                o_[bi, di] = p_[bi, ci][:, r0:r1, c0:c1]
        if int(err.item()) != 0:
            raise RuntimeError(f"GPU decode failed (err={int(err.item()):#x}: 16 = reference outside the DPB, "
                               "else a wavefront progress timeout)")
        res = []
        for j, sg in enumerate(segs):
            Pn = int(sg["n"])
            res.append(DecodedSegment(y_out[j, :Pn], u_out[j, :Pn], v_out[j, :Pn], fps, "gpu"))
        self.last_batch = (y_out, u_out, v_out)
        return res
