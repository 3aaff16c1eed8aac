"""gfx950 backend: a batch of pieces -> one batched GPU encode.

The reference worker runs one ``ffmpeg`` process per lease (client.go:101-130).
An MI355X worker holds several leases at once (worker ``--leases K``) and feeds
every closed-GOP unit of every piece into ONE :class:`GpuH264Encoder` call: the
wavefront kernels then see ``units x MB-rows`` independent waves instead of one
segment's worth, which is what fills 256 CUs.

Units of unequal length are padded to the longest by repeating their last frame;
the padded frames' NALs are dropped (P frames only reference earlier frames, so
truncating a closed GOP leaves a conformant stream).
"""
from __future__ import annotations

import concurrent.futures as cf
import time

import numpy as np

from ..jobs.ffargs import EncoderConfig
from ..utils import yuv  # noqa: F401  (type of encode_clips items)
from .common import (BackendError, PieceJob, PieceResult, Timer, idr_id, load_clip, output_size, unit_plan,
                     write_log, write_output)


class GpuBackend:
    name = "gpu"

    def __init__(self, device: str = "cuda", entropy: str = "gpu", max_slots: int = 256):
        import torch
        if not torch.cuda.is_available():
            raise BackendError("gpu backend requested but no GPU is visible")
        from ..ops import native
        native.hip()  # fail loudly if the gfx950 extension is missing
        self.torch = torch
        self.device = torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.entropy = entropy
        self.max_slots = max_slots
        from ..models.h264_gpu import GpuH264Encoder
        from ..models.hevc_gpu import GpuHevcEncoder, HevcParams
        from ..runtime import EncoderPool, StageStreams

        def make(p, b):
            if isinstance(p, HevcParams):
                return GpuHevcEncoder(p, slots=b, device=self.device)
            return GpuH264Encoder(p, slots=b, device=self.device, entropy=self.entropy)

        self._pool = EncoderPool(make, max_resident=1)
        self._streams = StageStreams(self.device)
        self._io = cf.ThreadPoolExecutor(max_workers=8)
        self._decoder = None

    def _encoder(self, params, slots: int):
        key = (type(params).__name__, params.width, params.height, params.fps, params.crf, params.qp,
               getattr(params, "bit_depth", 8), slots)
        return self._pool.get(key, params, slots)

    def encode_clips(self, items: list[tuple[str, "yuv.Clip"]], cfg: EncoderConfig,
                     tm: Timer | None = None) -> dict[str, tuple[bytes, dict]]:
        """Encode several clips (pieces/segments) together.  ``items``: (index token, clip).
        Returns token -> (Annex-B stream, stats).  Raises on failure."""
        from ..models.h264_gpu import H264Params
        from ..models.hevc_gpu import HevcParams
        from ..ops import native
        if cfg.codec not in ("h264", "hevc"):
            raise BackendError(f"codec {cfg.codec} is not available in the gpu backend")
        if cfg.bit_depth != 8 and cfg.codec == "h264":
            raise BackendError("10-bit H.264 output needs High 10; not supported")
        tm = tm or Timer()
        host = native.host()
        out: dict[str, tuple[bytes, dict]] = {}
        clips = dict(items)
        groups: dict[tuple, list[str]] = {}
        for key, c in items:
            groups.setdefault((c.width, c.height, output_size(cfg, c)), []).append(key)
        for (w, h, (ow, oh)), keys in groups.items():
            units = []  # (key, unit_no, start, count)
            for key in keys:
                for u, (s, c) in enumerate(unit_plan(clips[key].frames, cfg.keyint)):
                    units.append((key, u, s, c))
            fps = cfg.fps or clips[keys[0]].fps
            if cfg.codec == "hevc":
                if (ow, oh) != (w, h):
                    raise BackendError("scaling is not available in the HEVC path")
                params = HevcParams(width=ow, height=oh, fps=fps, crf=cfg.crf, qp=cfg.qp if cfg.qp is not None else 30,
                                    bit_depth=cfg.bit_depth)
            else:
                params = H264Params(width=ow, height=oh, fps=fps, crf=cfg.crf, qp=cfg.qp if cfg.qp is not None else 26)
            unit_out = []
            for b0 in range(0, len(units), self.max_slots):
                unit_out += self._encode_chunk(units[b0:b0 + self.max_slots], clips, params, w, h, tm)
            for key in keys:
                parts = sorted((x for x in unit_out if x[0] == key), key=lambda x: x[1])
                stream = host.concat([p[2] for p in parts])
                st = {"backend": "gpu", "codec": cfg.codec, "idx": key, "frames": clips[key].frames, "units": len(parts),
                      "width": ow, "height": oh, "fps": fps, "stream_bytes": len(stream),
                      "psnr_y": float(np.mean([p[3] for p in parts])), "ssim_y": float(np.mean([p[4] for p in parts])),
                      "config": cfg.as_dict()}
                out[key] = (stream, st)
        return out

    def decoder(self):
        """The batched GPU H.264 decoder (host CAVLC parse + gfx950 reconstruction)."""
        if self._decoder is None:
            from ..models.h264_decode_gpu import GpuH264Decoder
            self._decoder = GpuH264Decoder(self.device)
        return self._decoder

    def decode_streams(self, streams: list[bytes], fps: float = 30.0):
        """Annex-B segments -> device-resident clips (``DecodedSegment``), one batched call."""
        return self.decoder().decode(streams, fps)

    def _load_compressed(self, jobs: list[PieceJob]) -> dict[str, object]:
        """Compressed pieces (.264/.mp4, CAVLC) decode together on the GPU."""
        from ..ops import native
        from ..segment.probe import annexb_of, kind_of
        host = native.host()
        streams, keys, fps = [], [], 30.0
        for j in jobs:
            st = annexb_of(j.in_path, kind_of(j.in_path))
            info = host.stream_info(st)
            if info["entropy"] == "cabac":
                raise BackendError("input uses CABAC; this build decodes CAVLC H.264 only")
            fps = info["fps"] or fps
            streams.append(st)
            keys.append(j.idx)
        return dict(zip(keys, self.decode_streams(streams, fps)))

    def transcode(self, jobs: list[PieceJob], cfg: EncoderConfig) -> list[PieceResult]:
        from ..segment.probe import kind_of
        tm = Timer()
        t0 = time.perf_counter()
        results: dict[str, PieceResult] = {}
        items = []
        comp = [j for j in jobs if kind_of(j.in_path) in ("h264", "mp4")]
        raw = [j for j in jobs if j not in comp]
        futs = {j.idx: self._io.submit(load_clip, j.in_path) for j in raw}
        if comp:
            try:
                dec = self._load_compressed(comp)
                items += [(j.idx, dec[j.idx]) for j in comp]
            except Exception as e:  # noqa: BLE001 - reported to the coordinator
                for j in comp:
                    results[j.idx] = PieceResult(j.idx, False, f"decode: {e}")
        for j in raw:
            try:
                items.append((j.idx, futs[j.idx].result()))
            except Exception as e:  # noqa: BLE001 - reported to the coordinator
                results[j.idx] = PieceResult(j.idx, False, f"load: {e}")
        tm.add("load_s", time.perf_counter() - t0)
        if items:
            try:
                enc = self.encode_clips(items, cfg, tm)
            except Exception as e:  # noqa: BLE001
                for key, _ in items:
                    results[key] = PieceResult(key, False, f"encode: {e}")
                enc = {}
            for j in jobs:
                if j.idx in enc:
                    stream, st = enc[j.idx]
                    st["bytes"] = write_output(j, stream, st["fps"], cfg.codec)
                    st["timings"] = dict(tm.t)
                    write_log(j, st)
                    results[j.idx] = PieceResult(j.idx, True, stats=st)
        return [results[j.idx] for j in jobs]

    def _encode_chunk(self, chunk, clips, params, w: int, h: int, tm: Timer):
        torch = self.torch
        B = len(chunk)
        F = max(c for *_, c in chunk)
        t0 = time.perf_counter()
        if isinstance(clips[chunk[0][0]].y, torch.Tensor):  # device-resident (GPU-decoded) clips
            dy = torch.empty((B, F, h, w), dtype=torch.uint8, device=self.device)
            du = torch.empty((B, F, h // 2, w // 2), dtype=torch.uint8, device=self.device)
            dv = torch.empty_like(du)
            for b, (key, _, s, c) in enumerate(chunk):
                cl = clips[key]
                for dst, src in ((dy, cl.y), (du, cl.u), (dv, cl.v)):
                    dst[b, :c].copy_(src[s:s + c])
                    if c < F:
                        dst[b, c:].copy_(src[s + c - 1].expand(F - c, *src.shape[1:]))
            tm.add("upload_s", time.perf_counter() - t0)
            return self._run_encoder(chunk, params, dy, du, dv, tm)
        y = torch.empty((B, F, h, w), dtype=torch.uint8).pin_memory()
        u = torch.empty((B, F, h // 2, w // 2), dtype=torch.uint8).pin_memory()
        v = torch.empty_like(u).pin_memory()
        yn, un, vn = y.numpy(), u.numpy(), v.numpy()
        for b, (key, _, s, c) in enumerate(chunk):
            cl = clips[key]
            yn[b, :c], un[b, :c], vn[b, :c] = cl.y[s:s + c], cl.u[s:s + c], cl.v[s:s + c]
            if c < F:
                yn[b, c:], un[b, c:], vn[b, c:] = cl.y[s + c - 1], cl.u[s + c - 1], cl.v[s + c - 1]
        (dy, du, dv), ev = self._streams.upload([y, u, v], self.device)
        self._streams.wait(ev)
        tm.add("upload_s", time.perf_counter() - t0)
        return self._run_encoder(chunk, params, dy, du, dv, tm)

    def _run_encoder(self, chunk, params, dy, du, dv, tm: Timer):
        B = len(chunk)
        t1 = time.perf_counter()
        enc = self._encoder(params, B)
        if hasattr(enc, "encode") and type(params).__name__ == "HevcParams":
            res = enc.encode(dy, du, dv)
        else:
            # a short segment (padded to F frames) must end on an anchor to be cut there
            res = enc.encode(dy, du, dv, idr_ids=[idr_id(key, un_) for key, un_, _, _ in chunk],
                             anchors_at=sorted({c - 1 for _, _, _, c in chunk}))
        tm.add("encode_s", time.perf_counter() - t1)
        ps = enc.parameter_sets()
        return [(key, un_, ps + b"".join(res[b].display_prefix(c)), res[b].psnr_y, getattr(res[b], "ssim_y", 0.0))
                for b, (key, un_, s, c) in enumerate(chunk)]

    def close(self):
        self._pool.close()
        self._io.shutdown(wait=False)
