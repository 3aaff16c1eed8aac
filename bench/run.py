#!/usr/bin/env python3
"""Benchmark harness for the five BASELINE.json configurations (SURVEY.md 4.2 tier T7).

    python bench/run.py --config 2 [--gpus N]        # one JSON line per run
    python bench/run.py --all                         # every config this build supports

1. 640x360 10 s synthetic YUV -> H.264 through the job API on localhost
   (coordinator + workers over TCP).  The reference's worker shells out to ffmpeg;
   this image has no ffmpeg binary, so the ffmpeg-subprocess variant reports
   "n/a (no ffmpeg)" and the run uses the native CPU reference backend (and the
   GPU backend when a GPU is visible).
2. 1080p30 synthetic YUV -> H.264 CRF23 on MI355X: delegates to ``bench.py``
   (the driver's headline metric).
3. 4K30 H.264 -> H.264 (and HEVC -> H.264) transcode, segment-parallel: 4K pieces (High
   CABAC + 3 B pictures, or HEVC Main) are made (untimed) with the GPU encoders, then decode
   (host parse of the next batch overlapping the GPU work: gfx950 DPB reconstruction) +
   re-encode is timed end to end, next to the encode-only rate of the same batch.
4. 1080p30 synthetic YUV -> HEVC CRF26 (the reference's "265" preset) on MI355X:
   batched GPU HEVC encoder (CTU intra analysis/reconstruction, P pictures, deblock,
   SAO) + host CABAC.
5. 8K60 synthetic 10-bit YUV -> HEVC Main 10, two-pass average bitrate: pass 1 at the
   CRF QPs, per-frame statistics summed over ranks with one all-reduce (CC-1; RCCL
   over xGMI on a multi-GPU node), global rate solve, pass 2 at the solved QPs; both
   passes are timed.

Multi-GPU runs (``--gpus N``, N > 1) are launched one process per GPU with
``torch.distributed.run``; this harness never starts them itself on a 1-GPU box.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

METRIC = "encoded frames/sec (whole node)"


def emit(rec: dict, out: str | None):
    line = json.dumps(rec)
    print(line, flush=True)
    if out:
        with open(out, "a") as f:
            f.write(line + "\n")


def config1(args) -> list[dict]:
    """Job API plumbing on localhost: split -> coordinator -> workers -> merge."""
    from govideocompressor_amd.backends import get_backend
    from govideocompressor_amd.jobs import transport as T
    from govideocompressor_amd.jobs.coordinator import Coordinator
    from govideocompressor_amd.jobs.worker import Worker
    from govideocompressor_amd.segment.split import split
    from govideocompressor_amd.utils import yuv
    import torch

    recs = []
    frames = int(10 * 30)
    backends = ["cpu"] + (["gpu"] if torch.cuda.is_available() else [])
    if shutil.which("ffmpeg") is None:
        recs.append({"config": 1, "variant": "ffmpeg-subprocess", "value": None,
                     "note": "n/a (no ffmpeg binary in this image)"})
    else:
        backends.insert(0, "ffmpeg")
    for be_name in backends:
        tmp = tempfile.mkdtemp(prefix="mivc_cfg1_")
        try:
            clip = yuv.synth_clip_cpu(frames, 640, 360, seed=1)
            src = os.path.join(tmp, "clip.y4m")
            yuv.write_y4m(src, clip)
            d, n = split(src, seconds=1.0, out_root=tmp, log=lambda s: None)
            logs = []
            co = Coordinator(d, "264", port=0, host="127.0.0.1", out_root=os.path.join(tmp, "out"),
                             log=logs.append, src_root=tmp, merge=True)
            ready = threading.Event()
            orig = co.listening
            co.listening = lambda: (orig(), ready.set())
            rc = {}
            th = threading.Thread(target=lambda: rc.setdefault("rc", co.run()), daemon=True)
            t0 = time.perf_counter()
            th.start()
            ready.wait(30)
            workers = []
            nw = args.workers if be_name != "gpu" else 1
            for i in range(nw):
                kw = {"binary": shutil.which("ffmpeg")} if be_name == "ffmpeg" else {}
                be = get_backend(be_name, **kw)
                w = Worker("127.0.0.1", co.port, be, T.LocalFs(tmp, os.path.join(tmp, "out")),
                           leases=(n if be_name == "gpu" else 1), retry_s=0.1, idle_exit_s=2.0, batch_wait_s=0.5)
                wt = threading.Thread(target=w.run, daemon=True)
                wt.start()
                workers.append(wt)
            th.join(600)
            wall = time.perf_counter() - t0
            for wt in workers:
                wt.join(10)
            recs.append({"config": 1, "variant": f"job-api/{be_name}", "metric": METRIC, "value": round(frames / wall, 2),
                         "unit": "frames/s", "n_gpus": 1 if be_name == "gpu" else 0, "frames": frames, "pieces": n,
                         "workers": nw, "wall_s": round(wall, 3), "rc": rc.get("rc"),
                         "data": "synthetic 640x360 10 s Y4M"})
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
    return recs


def config2(args) -> list[dict]:
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(args.steps), "--warmup", str(args.warmup)]
    if args.gpus > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr=127.0.0.1", "--master-port=29511", os.path.join(ROOT, "bench.py"), "--gpus",
               str(args.gpus), "--steps", str(args.steps), "--warmup", str(args.warmup)]
    out = subprocess.run(cmd, capture_output=True, text=True, check=True).stdout.strip().splitlines()[-1]
    rec = json.loads(out)
    rec["config"] = 2
    return [rec]


def transcode_batch(n: int, max_slots: int, min_batches: int = 3) -> int:
    """Pieces per GPU batch for a rank holding ``n`` pieces: the largest batch <= max_slots that
    divides ``n`` into >= min_batches equal batches (the parse / decode / encode pipeline of
    models/transcode.py needs several batches to overlap, and an uneven last batch encodes
    padding), else the largest divisor of n <= max_slots, else max_slots."""
    n, max_slots = max(1, int(n)), max(1, int(max_slots))
    divs = [b for b in range(1, min(n, max_slots) + 1) if n % b == 0]
    good = [b for b in divs if n // b >= min_batches]
    return max(good) if good else (max(divs) if divs else max_slots)


def config3(args) -> list[dict]:
    """4K30 H.264 (or HEVC) -> H.264, segment-parallel over the ranks of one node: each rank
    (one process per GPU, torch.distributed.run) transcodes its contiguous share of the
    pieces -- batched GPU decode (host parse of batch k+1 overlapping the GPU work of batch k)
    + GPU re-encode (models/transcode.py) -- and the per-rank outputs are merged into ONE
    Annex-B stream on rank 0 in piece order (parallel/dist.py SegmentMerge: sizes all-gather,
    point-to-point payload over xGMI).  The reference's equivalent is pull dispatch of pieces to
    workers and concat.sh (server.go:161-191, client.go:37-80, server.go:349-361).  Timed:
    barrier + sync, transcode of this rank's pieces, merge; the time is the max over ranks."""
    import torch
    if not torch.cuda.is_available():
        return [{"config": 3, "value": None, "note": "needs a GPU"}]
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip
    from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams
    from govideocompressor_amd.models.transcode import GpuTranscoder
    from govideocompressor_amd.parallel import dist as D
    env = D.init(prefer_gpu=True)
    W, H = (int(x) for x in args.size3.split("x"))
    F, S = args.frames3, args.segments3
    # this rank's contiguous share of the global pieces (rank-major = piece order when merged)
    lo, hi = env.rank * S // env.world, (env.rank + 1) * S // env.world
    # batches sized from the share: >= 3 per rank (parse / decode / encode overlap), no padded slots
    B = transcode_batch(hi - lo, args.slots3)
    threads = args.threads3 or None
    recs = []
    for codec in args.codec3.split(","):
        # untimed: the input pieces (closed GOPs of F frames) made by this framework's
        # encoders; piece i's content depends on i only, not on the split over ranks
        pieces = []
        mk = (GpuHevcEncoder(_params(HevcParams, width=W, height=H, crf=22.0), slots=B, device=env.device) if codec == "hevc"
              else GpuH264Encoder(_params(H264Params, width=W, height=H, crf=20), slots=B, device=env.device))
        for b0 in range(lo, hi, B):
            y, u, v = synth_clip(B, F, W, H, seed=3, slot0=b0, device=env.device)
            pieces += [r.bitstream for r in mk.encode(y, u, v, metrics=False)][:hi - b0]
            del y, u, v
        mk.close()
        del mk
        torch.cuda.empty_cache()
        tc = GpuTranscoder(_params(H264Params, width=W, height=H, crf=23.0), slots=B, device=env.device, threads=threads)
        if args.warmup:
            tc.run(pieces[:B], 30.0)  # warmup batch
        merger = D.SegmentMerge(env)
        torch.cuda.synchronize()
        D.barrier(env)
        t0 = time.perf_counter()
        outs = tc.run(pieces, 30.0, first_index=lo)
        merged = merger.run(outs)
        torch.cuda.synchronize()
        D.barrier(env)
        wall = D.max_over_ranks(env, time.perf_counter() - t0)
        tm = dict(tc.timings)
        enc_fps = None
        if args.encode_only3:
            # encode-only reference on the same batch width: the decoded frames of one batch
            codec_in, parsed, _ = tc._parse(pieces[:B])
            y, u, v, counts = tc._frames(codec_in, parsed, 30.0)
            del parsed
            torch.cuda.synchronize()
            te = time.perf_counter()
            for _ in range(2):
                tc._encode(y, u, v, counts)
            torch.cuda.synchronize()
            enc_fps = 2 * B * F / (time.perf_counter() - te)
            del y, u, v
        tc.close()
        fps = S * F / wall
        if env.is_main:
            if args.merged_out3:
                with open(f"{args.merged_out3}.{codec}", "wb") as f:
                    f.write(memoryview(merged))
            recs.append({"config": 3, "metric": f"transcoded frames/sec (whole node), {args.size3} {codec.upper()}->H.264",
                         "value": round(fps, 2), "unit": "frames/s", "n_gpus": env.world, "frames": S * F,
                         "segments": S, "segments_per_gpu": hi - lo, "segments_per_batch": B,
                         "batches_per_gpu": -(-(hi - lo) // B), "parse_threads": tc.dec["h264"].threads,
                         "parallelism": f"dp{env.world} (segment-parallel, merged on rank 0)",
                         "wall_s": round(wall, 3), "merged_bytes": int(len(merged)),
                         "encode_only_fps_same_batch_rank0": round(enc_fps, 1) if enc_fps else None,
                         "transcode_vs_encode_only": round(fps / env.world / enc_fps, 3) if enc_fps else None,
                         "stage_s_rank0": {k: round(v, 3) for k, v in tm.items()},
                         "data": f"synthetic {codec.upper()} pieces made by this framework's encoder "
                                 "(no reference clips available)"})
        del pieces, outs
        torch.cuda.empty_cache()
    D.shutdown(env)
    return recs


def _hevc_run(args, W, H, B, F, bd, crf, two_pass_kbps=None, fps=30.0, resident=False):
    """Encode B segments x F frames of synthetic W x H content with the GPU HEVC encoder;
    returns (frames/s over the timed steps, details).

    bd 10 content is rendered at 10-bit precision by the synth kernel (not 8-bit x 4).
    resident: the clip is generated once into HBM before the warmup and every step
    encodes that same resident clip (config 5: a 10 s 8K clip held on the GPU)."""
    import numpy as np
    import torch

    from govideocompressor_amd.models.h264_gpu import synth_clip
    from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams
    from govideocompressor_amd.parallel import dist as D
    from govideocompressor_amd.rc import GlobalStats, TwoPassFeedback, abr_solve

    env = D.init(prefer_gpu=True)
    # MIVC_ENTROPY_THREADS (a runtime knob): host CABAC threads of this rank (a rank of an 8-GPU
    # node gets cores / 8; tools/gpu/r6_hevc_rehearse.sh)
    threads = int(os.environ["MIVC_ENTROPY_THREADS"]) if os.environ.get("MIVC_ENTROPY_THREADS") else None
    enc = GpuHevcEncoder(_params(HevcParams, width=W, height=H, fps=fps, crf=crf, bit_depth=bd), slots=B, device=env.device,
                         entropy_threads=threads)

    held = None
    if resident:
        held = synth_clip(B, F, W, H, seed=500 + env.rank * 131, device=env.device, bit_depth=bd)

    def clip(step):
        if held is not None:
            return held
        return synth_clip(B, F, W, H, seed=500 + step * 7 + env.rank * 131, device=env.device, bit_depth=bd)

    def step(k, quality=False):
        y, u, v = clip(k)
        if two_pass_kbps is None:
            return enc.encode(y, u, v, metrics=quality), None
        r1 = enc.encode(y, u, v, metrics=False)                       # pass 1: CRF QPs from the GPU lookahead
        # pass-1 bits are per NAL (coding order): pair them with the QPs in coding order too
        q1 = np.ascontiguousarray(enc.last_qps[:, enc.last_order])
        n = B * F
        gs = GlobalStats(n * env.world, env)
        st = np.zeros((n, 4))
        st[:, 2] = [b for r in r1 for b in r.bits]
        st[:, 3] = q1.reshape(-1)
        gs.put(env.rank * n, st)
        glob = gs.reduce()                                             # CC-1 all-reduce
        target = two_pass_kbps * 1000.0 * (n * env.world) / fps
        # the global solve (CC-1 totals) sets this rank's share of the budget: the frames
        # of every rank at one common offset; pass 2 then steers its share with feedback
        d0 = abr_solve(glob, target)
        p1 = glob[:, 2] * 2.0 ** (-d0 / 6.0)
        share = target * float(np.sum(p1[env.rank * n:(env.rank + 1) * n])) / max(float(np.sum(p1)), 1.0)
        fb = TwoPassFeedback(st[:, 2].reshape(B, F), q1, share)
        r2 = enc.encode(y, u, v, metrics=quality, rate_fb=fb)          # pass 2
        got = float(sum(sum(r.bits) for r in r2))
        return r2, dict(pass1_bits=float(np.sum(st[:, 2])), target_bits=share, pass2_bits=got,
                        pass2_vs_target=round(got / share, 4), exponent=round(fb.e, 3),
                        feedback_updates=len(fb.history))

    synth_stream = torch.cuda.Stream(device=env.device)

    def run_pipelined(first, n, quality=False):
        """n CRF steps pipelined like bench.py: step k + 1's synthesis and lookahead on a side
        stream while step k encodes, step k's CABAC tail (host entropy jobs) beside step k + 1's
        GPU work (encode_async); the last step is collected before returning."""
        def synth_async(k):
            with torch.cuda.stream(synth_stream):
                c = clip(k)
                ev = torch.cuda.Event()
                ev.record(synth_stream)
            return c, ev
        c, ev = synth_async(first)
        ana = enc.analyse_async(c[0], stream=synth_stream)
        prev = res = None
        for k in range(n):
            (y, u, v), cur_ev, cur_ana = c, ev, ana
            if k + 1 < n:
                c, ev = synth_async(first + k + 1)
                ana = enc.analyse_async(c[0], stream=synth_stream)
            torch.cuda.current_stream().wait_event(cur_ev)
            pend = enc.encode_async(y, u, v, metrics=quality and k == 0, analysis=cur_ana)
            del y, u, v
            if prev is not None:
                r = prev.result()
                res = r if res is None or not quality else res
            prev = pend
        r = prev.result()
        return (res if (quality and res is not None) else r), None

    pipelined = two_pass_kbps is None and held is None
    enc.stage_timer.enabled = True                                     # HIP-event stage times, warmup only
    res, info = run_pipelined(-1, 1, quality=True) if pipelined else step(-1, quality=True)  # warmup (+ PSNR)
    stage_ms = {k: round(v["s"] * 1000.0, 1) for k, v in enc.stage_timer.summary().items()}
    enc.stage_timer.enabled = False
    psnr = float(np.mean([r.psnr_y for r in res]))
    torch.cuda.synchronize()
    D.barrier(env)
    t0 = time.perf_counter()
    if pipelined:
        res, info = run_pipelined(0, args.steps)
    else:
        for k in range(args.steps):
            res, info = step(k)
    torch.cuda.synchronize()
    D.barrier(env)
    dt = D.max_over_ranks(env, time.perf_counter() - t0)
    bits = sum(sum(r.bits) for r in res)
    enc.close()
    clip_gb = (B * F * W * H * 3 // 2 * (2 if bd > 8 else 1)) / 1e9
    fps_out = B * F * args.steps * env.world / dt
    return fps_out, dict(psnr_y_warmup=round(psnr, 2), kbps_per_stream=round(bits / (B * F) * fps / 1000, 1),
                         ms_per_step=round(dt / args.steps * 1000, 1), timings=enc.timings, rc=info, world=env.world,
                         stage_device_ms_warmup=stage_ms, encoder_stats={k: round(v, 4) for k, v in enc.stats.items()},
                         resident_clip_gb=round(clip_gb, 1) if resident else None,
                         model=(f"HEVC Main{'10' if bd == 10 else ''} CTU {64 if enc.p.ctu64 else 32}, "
                                f"{enc.p.eff_bframes()}B{' pyramid' if enc.p.pyramid else ''}"
                                f"{' TMVP' if enc.p.tmvp else ''}, AQ + cutree, max-merge {enc.p.max_merge}, "
                                f"SAO, WPP{', sign hiding' if enc.p.sdh else ''}"))


def config4(args) -> list[dict]:
    import torch
    if not torch.cuda.is_available():
        return [{"config": 4, "value": None, "note": "needs a GPU"}]
    B, F = args.slots4, args.frames4
    v, d = _hevc_run(args, 1920, 1080, B, F, 8, 26.0)
    return [{"config": 4, "metric": "encoded frames/sec (whole node), 1080p30 -> HEVC CRF26", "value": round(v, 2),
             "unit": "frames/s", "n_gpus": d["world"], "segments_per_gpu": B, "frames_per_segment": F,
             "dtype": "int (8-bit video)", "data": "synthetic 1080p30 YUV", **d}]


def config5(args) -> list[dict]:
    import torch
    if not torch.cuda.is_available():
        return [{"config": 5, "value": None, "note": "needs a GPU"}]
    B, F = args.slots5, args.frames5
    v, d = _hevc_run(args, 7680, 4320, B, F, 10, 26.0, two_pass_kbps=args.kbps5, fps=60.0, resident=True)
    return [{"config": 5, "metric": "encoded frames/sec (whole node), 8K60 10-bit HEVC two-pass", "value": round(v, 2),
             "unit": "frames/s", "n_gpus": d["world"], "segments_per_gpu": B, "frames_per_segment": F,
             "target_kbps": args.kbps5, "data": "synthetic 8K60 10-bit YUV (10-bit synth kernel), resident in HBM",
             **d}]


_ALLOW_KNOBS = False


def _params(cls, **kw):
    """Encoder parameters of a config: its own settings, plus the MIVC_* encoder knobs of the
    environment when --allow-knobs was given (models/knobs.py)."""
    from govideocompressor_amd.models import knobs as K
    return cls(**{**kw, **(K.encoder_overrides(cls) if _ALLOW_KNOBS else {})})


def config_na(n: int, what: str) -> list[dict]:
    return [{"config": n, "value": None, "note": f"not implemented in this build: {what}"}]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--all", action="store_true")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--frames3", type=int, default=30)
    ap.add_argument("--segments3", type=int, default=256)
    ap.add_argument("--slots3", type=int, default=64, help="largest transcode batch (sized down per rank share)")
    ap.add_argument("--threads3", type=int, default=0, help="host parse threads per rank (0: decoder default)")
    ap.add_argument("--codec3", default="h264,hevc")
    ap.add_argument("--size3", default="3840x2160")
    ap.add_argument("--merged-out3", default=None, help="rank 0 writes the merged stream to <path>.<codec>")
    ap.add_argument("--no-encode-only3", dest="encode_only3", action="store_false",
                    help="skip the encode-only reference rate of config 3")
    ap.add_argument("--slots4", type=int, default=256, help="config 4 batch width (sweep 64 / 128 / 256: 2304 / 2408 / 2469 fps, profiles/r6_hevc_rank_rehearsal.md)")
    ap.add_argument("--frames4", type=int, default=30)
    # 10 segments x 60 frames = a 10 s 8K60 clip (~60 GB of 10-bit samples) resident in HBM
    ap.add_argument("--slots5", type=int, default=10)
    ap.add_argument("--frames5", type=int, default=60)
    ap.add_argument("--kbps5", type=float, default=80000.0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--allow-knobs", action="store_true", help="apply MIVC_* encoder knobs (models/knobs.py)")
    a = ap.parse_args()
    global _ALLOW_KNOBS
    from govideocompressor_amd.models import knobs as K
    K.check_environment(a.allow_knobs)
    _ALLOW_KNOBS = a.allow_knobs
    todo = [1, 2, 3, 4, 5] if a.all else [a.config]
    for c in todo:
        if c == 1:
            recs = config1(a)
        elif c == 2:
            recs = config2(a)
        elif c == 3:
            recs = config3(a)
        elif c == 4:
            recs = config4(a)
        else:
            recs = config5(a)
        for r in recs:
            emit(r, a.out)


if __name__ == "__main__":
    main()
