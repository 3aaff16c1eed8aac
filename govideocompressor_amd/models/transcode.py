"""Segment-batched transcode on one MI355X: compressed pieces -> GPU decode -> GPU encode.

The reference worker transcodes one piece per process: ``ffmpeg -i <idx>.mp4 <args>
c<idx>.mp4`` (client.go:101-130), decode and encode inside ffmpeg.  Here a batch of
pieces goes through the GPU together, as a three-stage pipeline:

* **host parse** of batch k+2 (H.264: CAVLC / CABAC entropy decode, csrc/host/h264_decoder.cc;
  HEVC: CABAC + motion derivation, csrc/host/hevc_dec.cc; C++ threads, GIL released) on a
  worker thread;
* **GPU decode** of batch k+1 on its own HIP stream, issued from a second worker thread
  (h264_decode_gpu / hevc_decode_gpu), writing display-size frames straight into the
  ``[B, F, h, w]`` tensors the encoder reads -- equal-length pieces are encoded from the
  decoder's output without another copy;
* **GPU encode** of batch k on the main thread's stream, with an encoder constructed once,
  before the first batch.  The decode kernels of batch k+1 fill the CUs the encoder's
  wavefront / entropy stages leave idle.

``run`` returns one Annex-B stream per piece plus stage timings.
"""
from __future__ import annotations

import concurrent.futures as cf
import time

import torch


class GpuTranscoder:
    def __init__(self, params, slots: int, device=None, threads: int | None = None):
        """``params``: H264Params or HevcParams of the output; ``slots``: pieces per GPU batch."""
        from .h264_decode_gpu import GpuH264Decoder
        from .h264_gpu import GpuH264Encoder
        from .hevc_decode_gpu import GpuHevcDecoder
        from .hevc_gpu import GpuHevcEncoder, HevcParams
        self.dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.dev.index is None:
            self.dev = torch.device("cuda", torch.cuda.current_device())
        self.p = params
        self.slots = int(slots)
        self.hevc_out = isinstance(params, HevcParams)
        self.enc = (GpuHevcEncoder(params, slots=self.slots, device=self.dev) if self.hevc_out
                    else GpuH264Encoder(params, slots=self.slots, device=self.dev))
        self.dec = {"h264": GpuH264Decoder(self.dev, threads), "hevc": GpuHevcDecoder(self.dev, threads)}
        self.pool = cf.ThreadPoolExecutor(max_workers=1)
        self.timings: dict[str, float] = {}

    def close(self):
        self.pool.shutdown(wait=True)
        if getattr(self, "dec_pool", None) is not None:
            self.dec_pool.shutdown(wait=True)
        self.enc.close()

    # ------------------------------------------------------------------ stages
    def _parse(self, pieces: list[bytes]):
        from ..segment.probe import codec_of
        t0 = time.perf_counter()
        codecs = {codec_of(p) for p in pieces}
        if len(codecs) != 1:
            raise ValueError("a transcode batch mixes H.264 and HEVC pieces")
        codec = codecs.pop()
        parsed = self.dec[codec].parse(pieces)
        return codec, parsed, time.perf_counter() - t0

    def _frames(self, codec: str, parsed, fps: float):
        """GPU decode -> (y, u, v [B, F, h, w] uint8, frames per piece)."""
        dec = self.dec[codec]
        segs = dec.reconstruct(parsed, fps)
        counts = [s.frames for s in segs]
        batch = getattr(dec, "last_batch", None)
        F = max(counts)
        if batch is not None and all(c == F for c in counts) and batch[0].shape[1] == F and batch[0].dtype == torch.uint8:
            return batch[0], batch[1], batch[2], counts
        # unequal pieces (or 10-bit / several geometries): pad with each piece's last frame
        B = len(segs)
        h, w = segs[0].height, segs[0].width
        y = torch.empty((B, F, h, w), dtype=torch.uint8, device=self.dev)
        u = torch.empty((B, F, h // 2, w // 2), dtype=torch.uint8, device=self.dev)
        v = torch.empty_like(u)
        for b, s in enumerate(segs):
            for dst, src in ((y, s.y), (u, s.u), (v, s.v)):
                if src.dtype != torch.uint8:  # Main 10 / High 10 input -> 8-bit encoder input (rounded)
                    from ..utils.yuv import to_8bit
                    src = to_8bit(src, s.bit_depth if s.bit_depth > 8 else 10)
                c = src.shape[0]
                dst[b, :c].copy_(src)
                if c < F:
                    dst[b, c:].copy_(src[c - 1].expand(F - c, *src.shape[1:]))
        return y, u, v, counts

    def _encode(self, y, u, v, counts: list[int], first: int = 0) -> list[bytes]:
        """``first``: global index of the batch's first piece -- each piece's idr_pic_id derives
        from its own index, so a piece codes the same bytes whatever batch or rank it lands in
        (and neighbouring pieces of a merged stream still alternate)."""
        B = y.shape[0]
        if B < self.slots:  # a short last batch: repeat the first piece in the spare slots
            pad = self.slots - B
            y, u, v = (torch.cat([t, t[:1].expand(pad, *t.shape[1:])]) for t in (y, u, v))
        ps = self.enc.parameter_sets()
        if self.hevc_out:
            res = self.enc.encode(y, u, v, metrics=False)
        else:
            res = self.enc.encode(y, u, v, idr_ids=[(first + b) & 0xFFFF for b in range(self.slots)],
                                  anchors_at=sorted({c - 1 for c in counts}),
                                  metrics=False)
        return [ps + b"".join(res[b].display_prefix(counts[b])) for b in range(B)]

    # ------------------------------------------------------------------ public
    def _decode_batch(self, fut):
        """Decode thread: wait for the batch's parse, reconstruct it on the decode stream."""
        codec, parsed, dt = fut.result()
        with torch.cuda.stream(self.dec_stream):
            t0 = time.perf_counter()
            y, u, v, counts = self._frames(codec, parsed, self._fps)
            del parsed
            ev = torch.cuda.Event()
            ev.record(self.dec_stream)
            ev.synchronize()
            return y, u, v, counts, ev, dt, time.perf_counter() - t0

    def run(self, pieces: list[bytes], fps: float = 30.0, first_index: int = 0) -> list[bytes]:
        """``first_index``: global index of pieces[0] (a rank's share of a larger job)."""
        batches = [pieces[i:i + self.slots] for i in range(0, len(pieces), self.slots)]
        out: list[bytes] = []
        t = dict(parse_s=0.0, decode_s=0.0, encode_s=0.0, decode_wait_s=0.0)
        if not batches:
            self.timings = t
            return out
        self._fps = fps
        if getattr(self, "dec_stream", None) is None:
            self.dec_stream = torch.cuda.Stream(self.dev)
            self.dec_pool = cf.ThreadPoolExecutor(max_workers=1)
        main = torch.cuda.current_stream(self.dev)
        # the decode stream starts after whatever the caller queued on the main stream
        self.dec_stream.wait_stream(main)
        pf = {k: self.pool.submit(self._parse, batches[k]) for k in range(min(2, len(batches)))}
        df = {0: self.dec_pool.submit(self._decode_batch, pf.pop(0))}
        for k in range(len(batches)):
            tw = time.perf_counter()
            y, u, v, counts, ev, dt_parse, dt_dec = df.pop(k).result()
            t["decode_wait_s"] += time.perf_counter() - tw
            t["parse_s"] += dt_parse
            t["decode_s"] += dt_dec
            if k + 1 < len(batches):   # GPU decode of k + 1 overlaps this batch's encode
                df[k + 1] = self.dec_pool.submit(self._decode_batch, pf.pop(k + 1))
            if k + 2 < len(batches):   # host parse two batches ahead
                pf[k + 2] = self.pool.submit(self._parse, batches[k + 2])
            main.wait_event(ev)
            for x in (y, u, v):
                x.record_stream(main)
            te = time.perf_counter()
            out += self._encode(y, u, v, counts, first_index + k * self.slots)
            main.synchronize()
            t["encode_s"] += time.perf_counter() - te
            del y, u, v
        self.timings = t
        return out
