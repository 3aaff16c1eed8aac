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
import os
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
        from ..runtime.device import device_info
        from ..runtime.pool import PinnedPool
        self._pinned = PinnedPool(max_cached=6)
        self._info = device_info(self.device.index)
        self._streams = StageStreams(self.device)
        self._io = cf.ThreadPoolExecutor(max_workers=8)
        self._decoder = None

    def _encoder(self, params, slots: int):
        import dataclasses
        key = (type(params).__name__, dataclasses.astuple(params), slots)
        return self._pool.get(key, params, slots)

    def encode_clips(self, items: list[tuple[str, "yuv.Clip"]], cfg: EncoderConfig,
                     tm: Timer | None = None, rate_stats: dict | None = None,
                     qp_offsets: dict[str, float] | None = None) -> dict[str, tuple[bytes, dict]]:
        """Encode several clips (pieces/segments) together.  ``items``: (index token, clip).
        Returns token -> (Annex-B stream, stats).  Raises on failure.

        Rate control: CRF / QP as given; with ``cfg.bitrate`` every clip is one rate group
        whose QP offset is solved by re-encoding the batch (:mod:`..rc.abr`), ``rate_stats``
        carries the ``-pass 1`` statistics in (pass 2) or out (pass 1), and ``qp_offsets``
        pins the offsets instead (the global two-pass of ``mivc encode``)."""
        from ..models.h264_gpu import H264Params
        from ..models.hevc_gpu import HevcParams
        from ..ops import native
        from ..rc import presets
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
            crf = cfg.crf if cfg.bitrate is None else 23.0  # ABR searches an offset from CRF 23
            if cfg.codec == "hevc":
                params = HevcParams(width=ow, height=oh, fps=fps, crf=crf if cfg.qp is None else None,
                                    qp=cfg.qp if cfg.qp is not None else 30, bit_depth=cfg.bit_depth)
            else:
                params = H264Params(width=ow, height=oh, fps=fps, crf=crf if cfg.qp is None else None,
                                    qp=cfg.qp if cfg.qp is not None else 26)
            params = presets.apply(params, cfg.preset)
            try:
                params = cfg.apply_opts(params)  # -profile:v / -tune / -level / -x26x-params
            except ValueError as e:
                raise BackendError(str(e)) from None
            # batch width: every unit at once up to what HBM holds (runtime.device.slots_for)
            from ..runtime.device import slots_for
            cap = min(self.max_slots, slots_for(ow, oh, max(c for *_, c in units), self._info, cap=self.max_slots))
            chunks = [units[b0:b0 + cap] for b0 in range(0, len(units), cap)]

            def prepare(ch, w=w, h=h, ow=ow, oh=oh):
                dev = self._prepare_chunk(ch, clips, w, h, tm)
                if (ow, oh) != (w, h):  # -s WxH: bicubic resample on the device (ops/scale.py)
                    if getattr(self, "_scaler", None) is None:
                        from ..ops.scale import GpuScaler
                        self._scaler = GpuScaler(self.device)
                    dev = self._scaler.clip(*dev, ow, oh)
                return dev

            rate_info: dict[str, dict] = {}
            if cfg.bitrate is None and qp_offsets is None:
                # one chunk resident at a time: `cap` sizes ONE chunk to the HBM budget
                unit_out = []
                for ch in chunks:
                    dev = prepare(ch)
                    unit_out += self._run_encoder(ch, params, *dev, tm)
                    del dev
            else:
                # the rate search re-encodes the batch: a single chunk stays resident between
                # passes, several chunks are re-prepared for every pass (only one fits)
                if len(chunks) == 1:
                    held = prepare(chunks[0])
                    prepared = [lambda: held]
                else:
                    prepared = [lambda ch=ch: prepare(ch) for ch in chunks]
                unit_out, rate_info = self._encode_rate(keys, chunks, prepared, clips, params, cfg, fps, tm,
                                                        rate_stats, qp_offsets)
            for key in keys:
                parts = sorted((x for x in unit_out if x["key"] == key), key=lambda x: x["unit"])
                stream = host.concat([p["stream"] for p in parts])
                st = {"backend": "gpu", "codec": cfg.codec, "idx": key, "frames": clips[key].frames, "units": len(parts),
                      "width": ow, "height": oh, "fps": fps, "stream_bytes": len(stream),
                      "psnr_y": float(np.mean([p["psnr"] for p in parts])),
                      "ssim_y": float(np.mean([p["ssim"] for p in parts])),
                      "frame_bits": [b for p in parts for b in p["frame_bits"]],
                      "timings": dict(tm.t), "config": cfg.as_dict(), **rate_info.get(key, {})}
                out[key] = (stream, st)
        return out

    def _encode_rate(self, keys, chunks, prepared, clips, params, cfg: EncoderConfig, fps: float, tm: Timer,
                     rate_stats: dict | None, qp_offsets: dict[str, float] | None):
        """ABR / two-pass / VBV over one geometry group: every key is a rate group."""
        from ..rc import abr
        frames = np.array([clips[k].frames for k in keys], dtype=np.float64)
        kidx = {k: i for i, k in enumerate(keys)}

        def encode_all(offsets: np.ndarray, vbv: dict[tuple, np.ndarray] | None = None):
            outs = []
            for ch, get_dev in zip(chunks, prepared):
                dev = get_dev()
                F = max(c for *_, c in ch)
                delta = np.zeros((len(ch), F))
                for b, (key, un_, _, c) in enumerate(ch):
                    delta[b] = offsets[kidx[key]]
                    if vbv and (key, un_) in vbv:
                        delta[b, :len(vbv[(key, un_)])] += vbv[(key, un_)]
                outs += self._run_encoder(ch, params, *dev, tm, qp_delta=delta)
            bits = np.zeros(len(keys))
            for o in outs:
                bits[kidx[o["key"]]] += 8 * len(o["stream"])
            return outs, bits

        if qp_offsets is not None:  # pinned offsets (global two-pass of mivc encode)
            offs = np.array([float(qp_offsets.get(k, 0.0)) for k in keys])
            outs, bits = encode_all(offs)
            return outs, {k: {"qp_offset": float(offs[i]), "rate_passes": 1} for i, k in enumerate(keys)}
        targets = float(cfg.bitrate) * frames / fps
        search = abr.OffsetSearch(targets, max_passes=4 if cfg.two_pass != 1 else 1)
        hist = []
        offsets = np.zeros(len(keys))
        seeded = cfg.two_pass == 2 and rate_stats is not None and all(k in rate_stats for k in keys)
        if seeded:
            search.observe([rate_stats[k]["offset"] for k in keys], [rate_stats[k]["bits"] for k in keys])
            hist.append(None)
            offsets = search.propose()
        while True:
            outs, bits = encode_all(offsets)
            search.observe(offsets, bits)
            hist.append(outs)
            if search.done():
                break
            offsets = search.propose()
        pick = search.best_per_group()
        if seeded:  # the seed entry has no encode behind it
            errs = np.stack([np.abs(b / np.maximum(targets, 1) - 1) for _, b in search.hist[1:]])
            pick = np.argmin(errs, axis=0) + 1
        best_off = np.array([search.hist[pick[i]][0][i] for i in range(len(keys))])
        chosen = []
        for i, k in enumerate(keys):
            chosen += [o for o in hist[pick[i]] if o["key"] == k]
        if cfg.two_pass == 1 and rate_stats is not None:
            for i, k in enumerate(keys):
                rate_stats[k] = {"offset": float(search.hist[-1][0][i]), "bits": float(search.hist[-1][1][i]),
                                 "frames": int(frames[i])}
        npass = len(search.hist) - (1 if seeded else 0)
        vbv_passes = 0
        if cfg.maxrate and cfg.bufsize and cfg.two_pass != 1:
            vbv: dict[tuple, np.ndarray] = {}
            for _ in range(2):
                fixes = 0
                for k in keys:
                    parts = sorted((o for o in chosen if o["key"] == k), key=lambda o: o["unit"])
                    fb = [b for p in parts for b in p["frame_bits"]]
                    if abr.vbv_fill(fb, cfg.maxrate, cfg.bufsize, fps).min() >= 0:
                        continue
                    dq = abr.vbv_deltas(fb, cfg.maxrate, cfg.bufsize, fps)
                    pos = 0
                    for p in parts:
                        n = len(p["frame_bits"])
                        disp = np.zeros(n)
                        disp[np.asarray(p["order"][:n])] = dq[pos:pos + n]  # coding -> display order
                        key2 = (k, p["unit"])
                        vbv[key2] = vbv.get(key2, np.zeros(n)) + disp
                        pos += n
                    fixes += 1
                if not fixes:
                    break
                chosen, _ = encode_all(best_off, vbv)
                vbv_passes += 1
        info = {}
        for i, k in enumerate(keys):
            got = sum(8 * len(o["stream"]) for o in chosen if o["key"] == k)
            info[k] = {"target_bits": float(targets[i]), "bits": float(got), "qp_offset": float(best_off[i]),
                       "rate_passes": int(npass), "vbv_passes": vbv_passes}
        return chosen, info

    def decoder(self, codec: str = "h264"):
        """The batched GPU decoder of ``codec``: host entropy parse + gfx950 reconstruction
        (H.264: h264_decode_gpu, HEVC: hevc_decode_gpu)."""
        if self._decoder is None:
            self._decoder = {}
        if codec not in self._decoder:
            if codec == "hevc":
                from ..models.hevc_decode_gpu import GpuHevcDecoder
                self._decoder[codec] = GpuHevcDecoder(self.device)
            else:
                from ..models.h264_decode_gpu import GpuH264Decoder
                self._decoder[codec] = GpuH264Decoder(self.device)
        return self._decoder[codec]

    def decode_streams(self, streams: list[bytes], fps: float = 30.0, keep_high_bit: bool = False):
        """Annex-B segments (H.264 and / or HEVC) -> device-resident clips (``DecodedSegment``),
        one batched call per codec.  Main 10 pictures are rounded to 8 bits (yuv.to_8bit) unless
        ``keep_high_bit`` (a Main 10 output: the HEVC encoder takes the 10-bit samples as they are)."""
        from ..segment.probe import codec_of
        import torch
        out = [None] * len(streams)
        by: dict[str, list[int]] = {}
        for i, s in enumerate(streams):
            by.setdefault(codec_of(s), []).append(i)
        self.decode_stats = {}
        for codec, idxs in by.items():
            dec = self.decoder(codec)
            got = dec.decode([streams[i] for i in idxs], fps)
            for k, v in dec.stats.items():
                self.decode_stats[k] = self.decode_stats.get(k, 0) + v
            for i, d in zip(idxs, got):
                if d.y.dtype != torch.uint8:
                    from ..models.h264_decode_gpu import DecodedSegment
                    bd = d.bit_depth if d.bit_depth > 8 else 10  # (the HEVC decoder's segments: Main 10)
                    if not keep_high_bit:  # Main 10 / High 10 input, 8-bit output
                        d = DecodedSegment(yuv.to_8bit(d.y, bd), yuv.to_8bit(d.u, bd), yuv.to_8bit(d.v, bd),
                                           d.fps, d.path)
                    elif bd != 10:  # 9/12/14-bit High 10-family input, Main 10 output: rescale to 10 bits
                        d = DecodedSegment(yuv.rescale_bits(d.y, bd), yuv.rescale_bits(d.u, bd),
                                           yuv.rescale_bits(d.v, bd), d.fps, d.path, bit_depth=10)
                out[i] = d
        return out

    def _load_compressed(self, jobs: list[PieceJob], keep_high_bit: bool = False) -> dict[str, object]:
        """Compressed pieces (.264 / .265 / .mp4: H.264 CAVLC or CABAC I/P/B High, HEVC Main /
        Main 10) decode together on the GPU."""
        from ..ops import native
        from ..segment.probe import annexb_of, codec_of, kind_of
        host = native.host()
        streams, keys, fps = [], [], 30.0
        for j in jobs:
            st = annexb_of(j.in_path, kind_of(j.in_path))
            info = host.hevc_stream_info(st) if codec_of(st) == "hevc" else host.stream_info(st)
            fps = info["fps"] or fps
            streams.append(st)
            keys.append(j.idx)
        return dict(zip(keys, self.decode_streams(streams, fps, keep_high_bit)))

    def _decode_group(self, jobs: list[PieceJob], keep_high_bit: bool):
        """Decode thread of :meth:`transcode`: one group of compressed pieces on the decode
        stream; returns (idx -> DecodedSegment, completion event)."""
        torch = self.torch
        if getattr(self, "_dec_stream", None) is None:
            self._dec_stream = torch.cuda.Stream(self.device)
        with torch.cuda.stream(self._dec_stream):
            dec = self._load_compressed(jobs, keep_high_bit)
            ev = torch.cuda.Event()
            ev.record(self._dec_stream)
        return dec, ev

    def transcode(self, jobs: list[PieceJob], cfg: EncoderConfig) -> list[PieceResult]:
        """Compressed pieces are decoded and encoded in groups of up to ``max_slots`` pieces, as
        a two-stage pipeline (the layout of models/transcode.GpuTranscoder): the GPU decode of
        group k+1 runs on its own stream, issued from a worker thread, while group k encodes
        on the main stream -- the decode kernels fill the CUs the encoder's wavefront and
        entropy stages leave idle.  Raw pieces load on the I/O pool and join the first group."""
        from ..segment.probe import kind_of
        torch = self.torch
        tm = Timer()
        t0 = time.perf_counter()
        results: dict[str, PieceResult] = {}
        comp = [j for j in jobs if kind_of(j.in_path) in ("h264", "hevc", "mp4", "ts", "mkv")]
        raw = [j for j in jobs if j not in comp]
        futs = {j.idx: self._io.submit(load_clip, j.in_path) for j in raw}
        # -pix_fmt yuv420p10le with libx265: Main 10 in, Main 10 out (no 8-bit detour)
        keep = cfg.codec == "hevc" and cfg.bit_depth == 10
        gsize = max(1, int(os.environ.get("MIVC_TRANSCODE_GROUP", self.max_slots)))
        groups = [comp[i:i + gsize] for i in range(0, len(comp), gsize)] or [[]]
        if getattr(self, "_dec_pool", None) is None:
            self._dec_pool = cf.ThreadPoolExecutor(max_workers=1)
        main = torch.cuda.current_stream(self.device)
        if comp:
            if getattr(self, "_dec_stream", None) is None:
                self._dec_stream = torch.cuda.Stream(self.device)
            self._dec_stream.wait_stream(main)
        nxt = self._dec_pool.submit(self._decode_group, groups[0], keep) if comp else None
        from ..rc import abr
        rate_stats = None
        paths = {j.idx: abr.stats_path_for(j.out_path, cfg.passlogfile) for j in jobs}
        if cfg.two_pass == 1:
            rate_stats = {}
        elif cfg.two_pass == 2:
            rate_stats = {}
            for j in jobs:
                if os.path.exists(paths[j.idx]):
                    rate_stats.update(abr.load_stats(paths[j.idx]))
        for g, group in enumerate(groups):
            items = []
            tw = time.perf_counter()
            if nxt is not None:
                try:
                    dec, ev = nxt.result()
                    main.wait_event(ev)
                    for d in dec.values():
                        for x in (d.y, d.u, d.v):
                            x.record_stream(main)
                    items += [(j.idx, dec[j.idx]) for j in group]
                except Exception as e:  # noqa: BLE001 - reported to the coordinator
                    for j in group:
                        results[j.idx] = PieceResult(j.idx, False, f"decode: {e}")
                nxt = None
            tm.add("decode_wait_s", time.perf_counter() - tw)
            if g + 1 < len(groups):  # decode of the next group overlaps this group's encode
                nxt = self._dec_pool.submit(self._decode_group, groups[g + 1], keep)
            if g == 0:
                for j in raw:
                    try:
                        items.append((j.idx, futs[j.idx].result()))
                    except Exception as e:  # noqa: BLE001 - reported to the coordinator
                        results[j.idx] = PieceResult(j.idx, False, f"load: {e}")
                tm.add("load_s", time.perf_counter() - t0)
            if not items:
                continue
            try:
                enc = self.encode_clips(items, cfg, tm, rate_stats=rate_stats)
            except Exception as e:  # noqa: BLE001
                for key, _ in items:
                    results[key] = PieceResult(key, False, f"encode: {e}")
                enc = {}
            del items
            for key, (stream, st) in enc.items():
                j = next(x for x in jobs if x.idx == key)
                st["bytes"] = write_output(j, stream, st["fps"], cfg.codec, cfg.audio)
                st["timings"] = dict(tm.t)
                write_log(j, st)
                results[key] = PieceResult(key, True, stats=st)
        if cfg.two_pass == 1 and rate_stats is not None:
            for j in jobs:
                if j.idx in rate_stats:
                    abr.save_stats(paths[j.idx], {j.idx: rate_stats[j.idx]})
        return [results[j.idx] for j in jobs]

    def _prepare_chunk(self, chunk, clips, w: int, h: int, tm: Timer):
        """One chunk's frames as [B, F, h, w] device planes (short units padded with their last frame)."""
        torch = self.torch
        B = len(chunk)
        F = max(c for *_, c in chunk)
        t0 = time.perf_counter()
        if isinstance(clips[chunk[0][0]].y, torch.Tensor):  # device-resident (GPU-decoded) clips
            dt = clips[chunk[0][0]].y.dtype  # uint8, or int16 Main 10 samples kept for a Main 10 encode
            dy = torch.empty((B, F, h, w), dtype=dt, device=self.device)
            du = torch.empty((B, F, h // 2, w // 2), dtype=dt, device=self.device)
            dv = torch.empty_like(du)
            for b, (key, _, s, c) in enumerate(chunk):
                cl = clips[key]
                for dst, src in ((dy, cl.y), (du, cl.u), (dv, cl.v)):
                    dst[b, :c].copy_(src[s:s + c])
                    if c < F:
                        dst[b, c:].copy_(src[s + c - 1].expand(F - c, *src.shape[1:]))
            tm.add("upload_s", time.perf_counter() - t0)
            return dy, du, dv
        # staging in recycled page-locked buffers (non_blocking H2D needs pinned memory;
        # pinning fresh pages per batch costs more than the copy)
        y = self._pinned.get(B * F * h * w).view(B, F, h, w)
        u = self._pinned.get(B * F * (h // 2) * (w // 2)).view(B, F, h // 2, w // 2)
        v = self._pinned.get(B * F * (h // 2) * (w // 2)).view(B, F, h // 2, w // 2)
        yn, un, vn = y.numpy(), u.numpy(), v.numpy()
        for b, (key, _, s, c) in enumerate(chunk):
            cl = clips[key]
            yn[b, :c], un[b, :c], vn[b, :c] = cl.y[s:s + c], cl.u[s:s + c], cl.v[s:s + c]
            if c < F:
                yn[b, c:], un[b, c:], vn[b, c:] = cl.y[s + c - 1], cl.u[s + c - 1], cl.v[s + c - 1]
        (dy, du, dv), ev = self._streams.upload([y, u, v], self.device)
        self._streams.wait(ev)
        if ev is not None:
            ev.synchronize()  # the staging buffers go back to the pool
        for t in (y, u, v):
            self._pinned.put(t)
        tm.add("upload_s", time.perf_counter() - t0)
        return dy, du, dv

    def _run_encoder(self, chunk, params, dy, du, dv, tm: Timer, qp_delta=None):
        t1 = time.perf_counter()
        enc = self._encoder(params, len(chunk))
        if type(params).__name__ == "HevcParams":
            res = enc.encode(dy, du, dv, qp_delta=qp_delta, anchors_at=sorted({c - 1 for _, _, _, c in chunk}))
        else:
            # a short segment (padded to F frames) must end on an anchor to be cut there
            res = enc.encode(dy, du, dv, idr_ids=[idr_id(key, un_) for key, un_, _, _ in chunk],
                             anchors_at=sorted({c - 1 for _, _, _, c in chunk}), qp_delta=qp_delta)
        tm.add("encode_s", time.perf_counter() - t1)
        ps = enc.parameter_sets()
        out = []
        for b, (key, un_, s, c) in enumerate(chunk):
            nals = res[b].display_prefix(c)
            order = list(getattr(res[b], "order", range(len(nals))))[:len(nals)]
            out.append(dict(key=key, unit=un_, stream=ps + b"".join(nals), psnr=res[b].psnr_y,
                            ssim=getattr(res[b], "ssim_y", 0.0), frame_bits=[8 * len(n) for n in nals], order=order))
        return out

    def close(self):
        self._pool.close()
        self._io.shutdown(wait=False)
        if getattr(self, "_dec_pool", None) is not None:
            self._dec_pool.shutdown(wait=True)
