"""Batched H.264 decode on MI355X: host entropy decode (CAVLC / CABAC) + gfx950 reconstruction.

The reference worker decodes its piece with ffmpeg before re-encoding
(client.go:115-118 ``ffmpeg -i <idx>.mp4 <args> <out>``).  Here a transcode
decodes many closed-GOP segments at once:

1. **parse** (host C++, one thread per segment, GIL released): CAVLC / CABAC -> per-MB
   ``MbHeader`` records (8x8-quadrant motion; a side-pool entry for partitions below 8x8),
   packed non-zero levels and 4-bit boundary strengths, kept in a C++ ``H264Batch``
   (csrc/host/decode_batch.cc); this is the only inherently serial part of H.264 decoding;
2. **pack + upload**: picture ``t`` of every slot is laid out by C++ straight into a pinned
   buffer and copied on a side stream while picture ``t - 1`` reconstructs;
3. **reconstruct** (``decode.hip``): inter MBs in parallel over (MB, segment), intra MBs
   in wavefront order, then the deblocking kernel with the parser's boundary strengths --
   each picture lands directly in its display position of the ``[segments, frames, H, W]``
   tensors the encoder consumes, and those same tensors are the reference store, so
   decoded pixels are neither copied nor cross PCIe.

P and B pictures (sub-8x8 partitions, B_8x8, spatial / temporal direct, explicit / implicit
weighted prediction, several references) reconstruct on the GPU; Intra 4x4 / 8x8 / 16x16
too, I_PCM macroblocks, constrained intra prediction, scaling matrices, and pictures of several
slices (the records carry each MB's slice for the intra neighbour availability).  Segments the
GPU path does not cover (High 10 and deeper streams -- the reconstruction kernels are 8-bit --,
mmco 5, implicit-weighted B slices with more than 8 references in a list, slices of one
picture with different reference lists or weights, per-picture filter parameters that differ
from the batch) are decoded by the CPU decoder instead (``h264_decoder.cc``) and uploaded; the
result is identical either way (the CPU decoder is the bit-exact oracle of
``tests/test_gpu_decode.py``).
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
    # High 10 streams (CPU decoder): int16 planes holding samples of this many bits -- the
    # layout of the encoders' 10-bit input (models/hevc_gpu.py Main 10)
    bit_depth: int = 8

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


def dpb_schedule(meta: np.ndarray, lists: np.ndarray):
    """Picture plan of one segment (decode order) when the decoded pictures themselves are
    the reference store: every picture is reconstructed straight into its display position
    of the segment's ``[F, H, W]`` output, and references are read from there.

    Returns (display [P] output position of each picture, reftab [P, 2, 32] output position
    of RefPicListX[i] or -1) or None when a list names a picture that is not decoded yet."""
    P = meta.shape[0]
    ids = meta[:, M["pic_id"]].astype(np.int64)
    # display order: IDR epochs, then POC
    epoch = np.cumsum(meta[:, M["idr"]] != 0)
    order = np.lexsort((meta[:, M["poc"]], epoch))
    display = np.empty(P, np.int64)
    display[order] = np.arange(P)
    pos: dict[int, int] = {}
    reftab = np.full((P, 2, 32), -1, np.int16)
    for p in range(P):
        for l in range(2):
            for k in range(32):
                i = int(lists[p, l, k])
                if i >= 0:
                    if i not in pos:
                        return None
                    reftab[p, l, k] = pos[i]
        pos[int(ids[p])] = int(display[p])
    return display, reftab


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
        """Host stage (GIL released, one C++ thread per segment): entropy decode into a
        C++-side batch (``_host.parse_batch``); nothing per-macroblock crosses into Python."""
        return list(segments), self.host.parse_batch(list(segments), self.threads)

    def reconstruct(self, parsed_in, fps: float = 30.0) -> list[DecodedSegment]:
        """GPU stage (+ the CPU decoder for segments the GPU path does not cover)."""
        import time
        segments, batch = parsed_in
        t1 = time.perf_counter()
        infos = [batch.info(i) for i in range(len(segments))]
        out: list[DecodedSegment | None] = [None] * len(segments)
        ok, fallback = [], []
        for i, seg in enumerate(infos):
            good, why = _gpu_plan(seg)
            (ok if good else fallback).append(i)
        # one batch per coded geometry + filter parameters; the rest decode on the CPU
        groups: dict[tuple, list[int]] = {}
        for i in ok:
            s = infos[i]
            m = s["meta"]
            params = {(int(r[M["alpha"]]), int(r[M["beta"]]), int(r[M["cqp"]]), int(r[M["deblock"]])) for r in m}
            if len(params) != 1:
                fallback.append(i)
                continue
            key = (s["coded_width"], s["coded_height"], s["width"], s["height"], s["crop_x"], s["crop_y"], params.pop())
            groups.setdefault(key, []).append(i)
        self.last_batch = None
        for key, idxs in groups.items():
            got = self._decode_group(key, batch, idxs, [infos[i] for i in idxs], fps)
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
        bd = int(pics[0].get("bit_depth", 8))
        if buf.dtype != np.uint8:
            buf = buf.astype(np.int16)  # <= 14-bit samples
        ys = w * h
        cs = (w // 2) * (h // 2)
        t = torch.from_numpy(buf).to(self.dev)
        y = t[:, :ys].reshape(len(pics), h, w)
        u = t[:, ys:ys + cs].reshape(len(pics), h // 2, w // 2)
        v = t[:, ys + cs:].reshape(len(pics), h // 2, w // 2)
        return DecodedSegment(y, u, v, fps, "cpu", bd)

    def _staging(self, cap: int) -> list[tuple[torch.Tensor, torch.Tensor]]:
        """Two (pinned host, device) step buffers of at least ``cap`` bytes, kept across calls."""
        st = getattr(self, "_stage", None)
        if st is None or st[0][0].numel() < cap:
            cap = (cap + (1 << 20) - 1) // (1 << 20) * (1 << 20)
            st = [(torch.empty(cap, dtype=torch.uint8, pin_memory=True),
                   torch.empty(cap, dtype=torch.uint8, device=self.dev)) for _ in range(2)]
            self._stage = st
        return st

    def _decode_group(self, key: tuple, batch, idxs: list[int], infos: list[dict],
                      fps: float) -> list[DecodedSegment] | None:
        """Decode one batch of same-geometry segments; None if a picture plan fails (CPU then).

        Each picture step of every slot is packed by C++ into a pinned buffer (``H264Batch.pack``)
        and copied on a side stream while the previous step reconstructs; pictures are
        reconstructed straight into their display positions of the output tensors, which are
        also the reference store (no separate decoded picture buffer, no output copy unless
        the stream crops)."""
        Wc, Hc, w, h, cx, cy, (alpha, beta, cqp, deblock) = key
        dev = self.dev
        wmb, hmb = Wc // 16, Hc // 16
        nmb = wmb * hmb
        B = len(idxs)
        ns = [int(s["n"]) for s in infos]
        F = max(ns)
        if F > 32767:
            return None
        plans = [dpb_schedule(s["meta"], s["lists"]) for s in infos]
        if any(pl is None for pl in plans):
            return None
        run = np.zeros((F, B), np.int8)
        nonref = np.ones((F,), bool)  # every active slot's picture of the step is a non-reference one
        cur = np.zeros((F, B), np.int16)
        reftab = np.full((F, B, 64), -1, np.int16)
        for j, s in enumerate(infos):
            Pn = ns[j]
            st = s["meta"][:, M["slice_type"]] % 5
            run[:Pn, j] = np.where(st == 2, 1, 2)
            nonref[:Pn] &= s["meta"][:, M["nal_ref"]] == 0
            cur[:Pn, j] = plans[j][0]
            reftab[:Pn, j] = plans[j][1].reshape(Pn, 64)
        d_run = torch.from_numpy(run).to(dev)
        d_cur = torch.from_numpy(cur).to(dev)
        d_reftab = torch.from_numpy(reftab).to(dev)
        slots = [[idxs[j] if t < ns[j] else -1 for j in range(B)] for t in range(F)]
        layouts = [batch.layout(t, slots[t], nmb) for t in range(F)]
        stage = self._staging(max(L["total"] for L in layouts))
        cap = stage[0][0].numel()
        # decoded pictures in display order: the output when the stream does not crop, else a
        # coded-size store cropped once at the end
        crop = (Hc, Wc) != (h, w)
        y_d = torch.empty((B, F, Hc, Wc), dtype=torch.uint8, device=dev)
        u_d = torch.empty((B, F, Hc // 2, Wc // 2), dtype=torch.uint8, device=dev)
        v_d = torch.empty_like(u_d)
        # per step parity: a non-reference step's deblocking (side stream) reads its nz while the
        # next step's reconstruction writes the other
        nzs = torch.zeros((2, B, nmb, 16), dtype=torch.uint8, device=dev)
        err = torch.zeros((1,), dtype=torch.int32, device=dev)
        comp = torch.cuda.current_stream(dev)
        copy = getattr(self, "_copy_stream", None)
        if copy is None:
            copy = self._copy_stream = torch.cuda.Stream(dev)
        copied = [torch.cuda.Event(), torch.cuda.Event()]
        consumed = [torch.cuda.Event(), torch.cuda.Event()]
        side = getattr(self, "_dbk_stream", None)
        if side is None:
            side = self._dbk_stream = torch.cuda.Stream(dev)
        side.wait_stream(comp)
        decoded = [torch.cuda.Event(), torch.cuda.Event()]
        for k in range(2):
            consumed[k].record(comp)
        s_ = comp.cuda_stream
        P_ = lambda t: t.data_ptr()  # noqa: E731
        for t in range(F):
            k = t & 1
            host_buf, dev_buf = stage[k]
            L = layouts[t]
            copied[k].synchronize()            # the copy of step t - 2 has read host_buf
            batch.pack(t, slots[t], nmb, host_buf.data_ptr(), cap, 8)
            with torch.cuda.stream(copy):
                copy.wait_event(consumed[k])   # step t - 2's kernels are done with dev_buf
                dev_buf[:L["total"]].copy_(host_buf[:L["total"]], non_blocking=True)
                copied[k].record(copy)
            comp.wait_event(copied[k])
            base = dev_buf.data_ptr()
            a = {n: base + int(L[n]) for n in ("hdr", "mask", "off", "bs", "wp", "coef", "sub")}
            any_inter = bool(np.any(run[t] == 2))
            nz = nzs[k]
            self.hip.decode_picture_dpb(B, wmb, hmb, F, P_(y_d), P_(u_d), P_(v_d), P_(d_cur[t]), P_(d_reftab[t]),
                                        a["wp"], a["sub"], a["hdr"], a["mask"], a["off"], a["coef"], P_(d_run[t]),
                                        int(any_inter), cqp, P_(nz), P_(err), s_)
            if deblock and nonref[t]:
                # nothing predicts from these pictures: their in-loop filter runs on a side stream
                # beside the next steps' reconstruction (the step's staging buffer and nz parity are
                # released after it)
                decoded[k].record(comp)
                side.wait_event(decoded[k])
                self.hip.deblock_dpb(B, wmb, hmb, F, P_(y_d), P_(u_d), P_(v_d), P_(d_cur[t]), a["hdr"], P_(nz),
                                     a["bs"], cqp, alpha, beta, P_(err), side.cuda_stream)
                consumed[k].record(side)
                continue
            if deblock:
                self.hip.deblock_dpb(B, wmb, hmb, F, P_(y_d), P_(u_d), P_(v_d), P_(d_cur[t]), a["hdr"], P_(nz),
                                     a["bs"], cqp, alpha, beta, P_(err), s_)
            consumed[k].record(comp)
        comp.wait_stream(side)  # the side-stream filters are part of the output
        if crop:
            y_out = y_d[:, :, cy:cy + h, cx:cx + w].contiguous()
            u_out = u_d[:, :, cy // 2:(cy + h) // 2, cx // 2:(cx + w) // 2].contiguous()
            v_out = v_d[:, :, cy // 2:(cy + h) // 2, cx // 2:(cx + w) // 2].contiguous()
            del y_d, u_d, v_d
        else:
            y_out, u_out, v_out = y_d, u_d, v_d
        if int(err.item()) != 0:
            raise RuntimeError(f"GPU decode failed (err={int(err.item()):#x}: 16 = reference outside the DPB, "
                               "else a wavefront progress timeout)")
        res = [DecodedSegment(y_out[j, :ns[j]], u_out[j, :ns[j]], v_out[j, :ns[j]], fps, "gpu") for j in range(B)]
        self.last_batch = (y_out, u_out, v_out)
        return res
