"""Single-node, multi-GPU file encode: ``mivc encode`` (SURVEY.md 2.5 / CS-6 collapsed).

The reference's operator workflow is split -> coordinate -> N workers ->
concat.sh (CS-6).  On one MI355X node the same data flow runs as one process per
GPU with no files in between:

1. every rank probes the input and builds the same segment plan (closed GOPs;
   rank 0's plan is broadcast as a consistency check, CC-4);
2. segments are assigned statically (cost-balanced) or claimed dynamically in
   batch-sized chunks from the TCPStore ticket counter (the pull scheduling of
   server.go:175-189);
3. each rank reads/decodes only its own segments, encodes them as one batched GPU
   call per chunk and keeps the bitstreams;
4. the bitstreams go point-to-point to rank 0 (CC-2 sizes all-gather + CC-3 RCCL
   isend/irecv) and rank 0 concatenates them in segment order into the output (the
   concat.sh step, server.go:349-361).
"""
from __future__ import annotations

import json
import os
import time

import numpy as np

from .backends import get_backend
from .jobs import ffargs
from .parallel import dist as D
from .parallel.tickets import TicketDispenser
from .segment import plan as P
from .segment.probe import annexb_of, probe
from .utils import yuv


def _segments(path: str, info, world: int, slots: int, seg_frames: int | None, gop: int | None):
    """Returns (kind, segment list).  Raw: frame ranges; compressed: IDR-aligned pieces."""
    if info.kind in ("h264", "hevc", "mp4", "ts", "mkv"):
        from .segment.probe import split_stream
        target = seg_frames or max(1, info.frames // max(1, world * slots))
        pieces = split_stream(annexb_of(path, info.kind), target)
        return "pieces", pieces
    if seg_frames:
        pl = P.fixed_plan(info.frames, seg_frames)
    else:
        pl = P.balanced_plan(info.frames, world=world, per_rank=slots, min_frames=max(8, gop or 8), gop=gop)
    return "ranges", pl


def _load_segment(path: str, info, kind: str, segs, i: int) -> yuv.Clip:
    if kind == "pieces":
        from .backends.common import decode_stream_cpu
        return decode_stream_cpu(segs[i], info.fps)
    s, c, _ = (int(x) for x in segs[i])
    if info.kind == "y4m":
        return yuv.read_y4m(path, s, c)
    return yuv.read_yuv(path, info.width, info.height, info.fps, info.bit_depth, s, c)


class SegmentCheckpoint:
    """Per-segment checkpoint of ``encode_file(resume=True)``: every encoded
    segment is written to ``<work_dir>/<idx>.seg`` (atomic rename) and recorded in this
    rank's ``manifest.rank<r>.json`` (size + CRC32); a restarted run with the same input
    plan and arguments skips the segments every manifest already holds, and rank 0
    concatenates the finished parts.  A plan or argument change invalidates the checkpoint."""

    def __init__(self, work_dir: str, rank: int, sig: dict):
        self.dir = work_dir
        self.rank = rank
        self.sig = sig
        os.makedirs(work_dir, exist_ok=True)
        self.mine: dict[str, dict] = {}

    def _manifests(self):
        return sorted(f for f in os.listdir(self.dir) if f.startswith("manifest.rank") and f.endswith(".json"))

    def done(self) -> dict[int, dict]:
        """Segments finished by any rank of an earlier run with the same plan (file checked)."""
        import zlib
        out = {}
        for f in self._manifests():
            try:
                with open(os.path.join(self.dir, f)) as fh:
                    m = json.load(fh)
            except (OSError, ValueError):
                continue
            if m.get("sig") != self.sig:
                continue
            for k, v in m.get("done", {}).items():
                pth = os.path.join(self.dir, f"{int(k)}.seg")
                try:
                    with open(pth, "rb") as fh:
                        data = fh.read()
                except OSError:
                    continue
                if len(data) == v["bytes"] and zlib.crc32(data) == v["crc"]:
                    out[int(k)] = v
        return out

    def put(self, idx: int, data: bytes) -> None:
        import zlib
        pth = os.path.join(self.dir, f"{idx}.seg")
        with open(pth + ".part", "wb") as fh:
            fh.write(data)
        os.replace(pth + ".part", pth)
        self.mine[str(idx)] = {"bytes": len(data), "crc": zlib.crc32(data)}
        mpath = os.path.join(self.dir, f"manifest.rank{self.rank}.json")
        try:
            with open(mpath) as fh:
                old = json.load(fh)
            if old.get("sig") == self.sig:
                merged = {**old.get("done", {}), **self.mine}
            else:
                merged = dict(self.mine)
        except (OSError, ValueError):
            merged = dict(self.mine)
        with open(mpath + ".part", "w") as fh:
            json.dump({"sig": self.sig, "done": merged}, fh)
        os.replace(mpath + ".part", mpath)

    def read(self, idx: int) -> bytes:
        with open(os.path.join(self.dir, f"{idx}.seg"), "rb") as fh:
            return fh.read()


def content_digest(path: str, sample: int = 1 << 20, points: int = 16) -> str:
    """Identity of an input's *content* for the resume checkpoint: a hash of the first and
    last MiB plus ``points`` evenly spaced 1 MiB samples (raw clips of one geometry all have
    the same size, so size + path alone would splice an old run's segments into a new clip)."""
    import hashlib
    h = hashlib.blake2b(digest_size=16)
    n = os.path.getsize(path)
    with open(path, "rb") as f:
        offs = sorted({0, max(0, n - sample), *(k * max(0, n - sample) // max(1, points - 1) for k in range(points))})
        for o in offs:
            f.seek(o)
            h.update(f.read(sample))
    h.update(str(n).encode())
    return h.hexdigest()


def encode_file(path: str, output: str, args: str = "264", backend: str = "auto", slots: int = 16,
                seg_frames: int | None = None, schedule: str = "static", raw_size: tuple[int, int] | None = None,
                fps: float = 30.0, log=print, resume: bool = False, work_dir: str | None = None) -> dict:
    """Encode one file on this node's ranks.  ``resume``: keep a per-segment checkpoint in
    ``work_dir`` (default ``<output>.parts``) and skip the segments it already holds."""
    env = D.init(prefer_gpu=(backend in ("auto", "gpu")))
    cfg = ffargs.parse(args)
    w, h = raw_size or (0, 0)
    info = probe(path, w, h, fps)
    kind, segs = _segments(path, info, env.world, slots, seg_frames, cfg.keyint)
    n = len(segs)
    sig = (kind, n, int(np.sum([len(x) for x in segs])) if kind == "pieces" else int(np.sum(segs[:, 1])))
    sig0 = D.broadcast_object(env, sig)
    if sig0 != sig:
        raise RuntimeError(f"rank {env.rank}: segment plan differs from rank 0 ({sig} vs {sig0})")
    ckpt = None
    skip: set[int] = set()
    if resume:
        if cfg.bitrate is not None:
            raise ValueError("resume is for CRF / QP encodes: -b:v solves one offset over the whole file")
        plan_sig = {"input": os.path.abspath(path), "size": os.path.getsize(path),
                    "mtime_ns": os.stat(path).st_mtime_ns, "content": content_digest(path), "args": args,
                    "plan": list(sig), "seg_frames": seg_frames, "world": env.world, "slots": slots}
        ckpt = SegmentCheckpoint(work_dir or output + ".parts", env.rank, plan_sig)
        D.barrier(env)
        skip = set(ckpt.done())
    be = get_backend(backend, **({"device": str(env.device)} if backend in ("gpu",) or
                                 (backend == "auto" and env.device.type == "cuda") else {}))
    impl = be.impl
    t0 = time.perf_counter()
    mine: dict[int, bytes] = {}
    stats: list[dict] = []

    import concurrent.futures as cf
    loader = cf.ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4))  # native decode releases the GIL

    gpu_decode = kind == "pieces" and hasattr(impl, "decode_streams")
    dec_stats: dict[str, float] = {}

    from .obs.log import JsonLogger
    jlog = JsonLogger(os.environ.get("MIVC_LOG_JSON"), rank=env.rank, component="encode")

    def run(idxs: list[int], offset: float | None = None, into: dict | None = None):
        if gpu_decode:  # compressed input on a GPU rank: batched GPU decode, frames stay on the device
            clips = impl.decode_streams([segs[i] for i in idxs], info.fps)
            for k, v in getattr(impl, "decode_stats", {}).items():
                dec_stats[k] = dec_stats.get(k, 0) + v
        else:
            clips = list(loader.map(lambda i: _load_segment(path, info, kind, segs, i), idxs))
        items = [(str(i), c) for i, c in zip(idxs, clips)]
        tb = time.perf_counter()
        if offset is None:
            res = impl.encode_clips(items, cfg)
        else:
            res = impl.encode_clips(items, cfg, qp_offsets={str(i): offset for i in idxs})
        dt = time.perf_counter() - tb
        if jlog.enabled:  # per-segment metrics: frames, bits, PSNR / SSIM, batch timing
            for i in idxs:
                st = res[str(i)][1]
                jlog.event("segment", segment=i, frames=st.get("frames"), bits=8 * st.get("stream_bytes", 0),
                           psnr_y=st.get("psnr_y"), ssim_y=st.get("ssim_y"), qp_offset=st.get("qp_offset"),
                           batch_segments=len(idxs), batch_s=round(dt, 4),
                           batch_fps=round(sum(c.frames for c in clips) / dt, 2) if dt > 0 else None,
                           stages={k: round(v, 4) for k, v in st.get("timings", {}).items()})
        for i in idxs:
            stream, st = res[str(i)]
            (mine if into is None else into)[i] = stream
            stats.append(st)
            if ckpt is not None:
                ckpt.put(i, stream)

    rate = None
    if cfg.bitrate is not None and hasattr(impl, "decode_streams"):
        # global rate control over the whole file (x264 two-pass semantics): one QP offset
        # for every segment of every rank, solved on all-reduced bit totals (CC-1)
        from .rc.abr import OffsetSearch
        schedule = "static"
        if kind == "ranges":
            my = P.shard(segs, env.rank, env.world, by_cost=True)
        else:
            my = list(range(env.rank, n, env.world))
        target = float(cfg.bitrate) * info.frames / (cfg.fps or info.fps)
        search = OffsetSearch(np.array([target]), max_passes=4)
        passes: list[dict] = []
        off = 0.0
        while True:
            got: dict[int, bytes] = {}
            stats.clear()
            for b in range(0, len(my), slots):
                run(my[b:b + slots], off, got)
            total = D.sum_over_ranks(env, float(sum(8 * len(x) for x in got.values())))
            search.observe([off], [total])
            passes.append(got)
            if search.done():
                break
            off = float(search.propose()[0])
        best = search.best()
        mine.update(passes[best])
        rate = {"target_bits": target, "bits": float(search.hist[best][1][0]), "qp_offset": float(search.hist[best][0][0]),
                "rate_passes": len(passes)}
    elif schedule == "dynamic":
        td = TicketDispenser(n)
        while True:
            got = td.claim(slots)
            if not got:
                break
            got = [i for i in got if i not in skip]
            if got:
                run(got)
    elif rate is None:
        if kind == "ranges":
            my = P.shard(segs, env.rank, env.world, by_cost=True)
        else:
            my = list(range(env.rank, n, env.world))
        my = [i for i in my if i not in skip]
        for b in range(0, len(my), slots):
            run(my[b:b + slots])
    t_enc = time.perf_counter() - t0
    order = sorted(mine)
    # CC-2/CC-3: bitstreams + their segment indices to rank 0
    idx_blob = json.dumps(order).encode()
    g = D.BitstreamGather(env, [idx_blob] + [mine[i] for i in order]).start()
    gathered = g.wait()
    out = {"segments": n, "world": env.world, "encode_s_rank": t_enc, "rate": rate, "resumed_segments": len(skip),
           "decode": ("gpu" if gpu_decode else "cpu"), "decode_stats_rank": dec_stats}
    if env.is_main:
        by_idx: dict[int, bytes] = {}
        for rank_pieces in gathered:
            ids = json.loads(rank_pieces[0].decode())
            for i, pc in zip(ids, rank_pieces[1:]):
                by_idx[i] = pc
        for i in skip:  # finished by an earlier (interrupted) run
            if i not in by_idx:
                by_idx[i] = ckpt.read(i)
        missing = [i for i in range(n) if i not in by_idx]
        if missing:
            raise RuntimeError(f"segments never encoded: {missing[:8]}")
        from .ops import native
        hst = native.host()
        stream = hst.concat([by_idx[i] for i in range(n)])
        out_fps = cfg.fps or info.fps
        if output.lower().endswith(".mp4"):
            from .segment import mp4
            extra = []
            if info.kind == "mp4" and cfg.audio == "copy":  # the input's audio, stream-copied
                with open(path, "rb") as f:
                    extra = mp4.file_audio(f.read())
            elif info.kind in ("ts", "mkv") and cfg.audio == "copy":  # its AAC tracks (containers.py)
                from .segment.containers import demux
                extra = demux(path, info.kind).audio
            data = mp4.mux_video(stream, out_fps, cfg.codec, extra)
        else:
            data = stream
        with open(output + ".part", "wb") as f:
            f.write(data)
        os.replace(output + ".part", output)
        frames = info.frames
        out.update(output=output, bytes=len(data), frames=frames,
                   psnr_y_rank0=float(np.mean([s["psnr_y"] for s in stats])) if stats else 0.0)
    wall = D.max_over_ranks(env, time.perf_counter() - t0)
    out["wall_s"] = wall
    if env.is_main:
        out["fps"] = info.frames / wall if wall > 0 else 0.0
        log(json.dumps(out))
    jlog.event("done", wall_s=round(wall, 4), segments=n, encoded_here=len(mine))
    jlog.close()
    loader.shutdown(wait=False)
    be.close()
    D.shutdown(env)
    return out
