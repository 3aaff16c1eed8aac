"""Batched H.264 (CAVLC) decode on MI355X: host entropy decode + gfx950 reconstruction.

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

Segments the GPU path does not cover (sub-8x8 partitions, several reference
frames, I_PCM, several slices, per-picture filter parameters that differ from the
batch) are decoded by the CPU decoder instead (``h264_decoder.cc``) and uploaded;
the result is identical either way (the CPU decoder is the bit-exact oracle of
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

    @property
    def frames(self) -> int:
        return int(self.y.shape[0])

    @property
    def width(self) -> int:
        return int(self.y.shape[2])

    @property
    def height(self) -> int:
        return int(self.y.shape[1])


_META = ("pic_id", "ref_id", "nal_ref", "idr", "slice_type", "slice_qp", "alpha", "beta", "cqp", "deblock", "gpu_ok")
M = {k: i for i, k in enumerate(_META)}


def _gpu_plan(seg: dict) -> tuple[bool, str]:
    """Can the GPU path reconstruct this parsed segment?"""
    if seg.get("error"):
        return False, seg["error"]
    if seg["n"] == 0:
        return False, "no pictures"
    meta = seg["meta"]
    if not np.all(meta[:, M["gpu_ok"]] == 1):
        return False, "unsupported coding tools"
    last_ref = -1
    for r in meta:
        st = int(r[M["slice_type"]]) % 5
        if st == 0:
            if int(r[M["ref_id"]]) != last_ref or last_ref < 0:
                return False, "reference is not the previous reference picture"
        elif st != 2:
            return False, f"slice type {st}"
        if r[M["nal_ref"]]:
            last_ref = int(r[M["pic_id"]])
    return True, ""


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
        parsed = self.host.parse(list(segments), self.threads)
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
            for i, d in zip(idxs, self._decode_group(key, [parsed[i] for i in idxs], fps)):
                out[i] = d
        t2 = time.perf_counter()
        for i in fallback:
            out[i] = self._cpu_decode(segments[i], fps)
        self.stats = {"parse_s": t1 - t0, "gpu_s": t2 - t1, "cpu_fallback_s": time.perf_counter() - t2,
                      "segments_gpu": len(segments) - len(fallback), "segments_cpu": len(fallback)}
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

    def _decode_group(self, key: tuple, segs: list[dict], fps: float) -> list[DecodedSegment]:
        Wc, Hc, w, h, cx, cy, (alpha, beta, cqp, deblock) = key
        dev = self.dev
        wmb, hmb = Wc // 16, Hc // 16
        nmb = wmb * hmb
        B = len(segs)
        F = max(int(s["n"]) for s in segs)
        # ---- pack the batch: [F, B, nmb, ...] records, one flat level array
        hdr = np.zeros((F, B, nmb, 64), np.uint8)
        mask = np.zeros((F, B, nmb), np.uint32)
        off = np.zeros((F, B, nmb), np.uint32)
        run = np.zeros((F, B), np.int8)
        nal_ref = np.zeros((F, B), bool)
        base = 0
        coefs = []
        for j, s in enumerate(segs):
            P = int(s["n"])
            hdr[:P, j] = s["hdr"]
            mask[:P, j] = s["mask"]
            off[:P, j] = s["off"] + (s["pic_off"][:P, None] + base).astype(np.uint32)
            st = s["meta"][:, M["slice_type"]] % 5
            run[:P, j] = np.where(st == 2, 1, 2)
            nal_ref[:P, j] = s["meta"][:, M["nal_ref"]] != 0
            coefs.append(s["coef"])
            base += int(s["pic_off"][P])
        if base >= 2 ** 32:
            raise ValueError("level array too large for 32-bit block offsets")
        coef = np.concatenate(coefs) if coefs else np.zeros(16, np.int16)
        if coef.size == 0:
            coef = np.zeros(16, np.int16)
        d_hdr = torch.from_numpy(hdr).to(dev, non_blocking=False)
        d_mask = torch.from_numpy(mask.view(np.int32)).to(dev)
        d_off = torch.from_numpy(off.view(np.int32)).to(dev)
        d_coef = torch.from_numpy(coef).to(dev)
        d_run = torch.from_numpy(run).to(dev)
        # ---- output tensors and the per-slot working pictures
        y_out = torch.empty((B, F, Hc, Wc), dtype=torch.uint8, device=dev)
        u_out = torch.empty((B, F, Hc // 2, Wc // 2), dtype=torch.uint8, device=dev)
        v_out = torch.empty_like(u_out)
        cur = [torch.zeros((B, Hc, Wc), dtype=torch.uint8, device=dev),
               torch.zeros((B, Hc // 2, Wc // 2), dtype=torch.uint8, device=dev),
               torch.zeros((B, Hc // 2, Wc // 2), dtype=torch.uint8, device=dev)]
        ref = [torch.zeros_like(x) for x in cur]
        nz = torch.zeros((B, nmb, 16), dtype=torch.uint8, device=dev)
        err = torch.zeros((1,), dtype=torch.int32, device=dev)
        s = torch.cuda.current_stream(dev).cuda_stream
        P_ = lambda t: t.data_ptr()  # noqa: E731
        for t in range(F):
            active = run[t] != 0
            any_p = bool(np.any(run[t] == 2))
            self.hip.decode_picture(B, wmb, hmb, P_(ref[0]), P_(ref[1]), P_(ref[2]), P_(cur[0]), P_(cur[1]),
                                    P_(cur[2]), P_(d_hdr[t]), P_(d_mask[t]), P_(d_off[t]), P_(d_coef), P_(d_run[t]),
                                    int(any_p), cqp, P_(nz), P_(err), s)
            if deblock:
                self.hip.deblock(B, wmb, hmb, P_(cur[0]), P_(cur[1]), P_(cur[2]), P_(d_hdr[t]), P_(nz), cqp, alpha,
                                 beta, P_(err), s)
            y_out[:, t].copy_(cur[0])
            u_out[:, t].copy_(cur[1])
            v_out[:, t].copy_(cur[2])
            upd = nal_ref[t] & active
            if (upd == active).all():  # inactive slots have ended: their buffers are free
                cur, ref = ref, cur
            elif upd.any():
                sel = torch.from_numpy(np.nonzero(upd)[0]).to(dev)
                for k in range(3):
                    ref[k].index_copy_(0, sel, cur[k].index_select(0, sel))
        if int(err.item()) != 0:
            raise RuntimeError("GPU decode: wavefront progress timeout")
        res = []
        for j, sg in enumerate(segs):
            P = int(sg["n"])
            res.append(DecodedSegment(y_out[j, :P, cy:cy + h, cx:cx + w], u_out[j, :P, cy // 2:(cy + h) // 2, cx // 2:(cx + w) // 2],
                                      v_out[j, :P, cy // 2:(cy + h) // 2, cx // 2:(cx + w) // 2], fps, "gpu"))
        return res
