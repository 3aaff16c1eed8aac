#!/usr/bin/env python3
"""Headline benchmark: whole-node encoded frames/sec, 1080p30 synthetic YUV -> H.264 CRF23.

Metric/config from BASELINE.json ("encoded frames/sec (whole node), 1080p30->H.264
CRF23, at 1/2/4/8 MI355X").  One process per GPU (torch.distributed.run), weak
scaling: every rank encodes B closed-GOP segments of F frames per step.  A timed step is

    synthesize B*F new 1080p frames in HBM (new content every step)
    -> GPU lookahead over all B*F frames (lowres search + MFMA Hadamard SATD) -> CRF QPs
    -> batched GPU encode (ME, TQ, intra/deblock wavefronts, CAVLC)
    -> merge: piece sizes + packed bitstreams all-gathered over xGMI (RCCL), rank 0
       copies every rank's bytes back to back into ONE Annex-B stream in segment order
       (the reference's concat.sh); runs on a side stream/thread, overlapping the next
       step's encode, and the next step's input synthesis is queued before it

bracketed by barrier + torch.cuda.synchronize(); the step time is the max over ranks.
The reference publishes no numbers, so vs_baseline is null.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import dataclasses
import hashlib
import json
import os
import sys
import time

# eight hardware queues (HIP's default is 4), before anything can load the HIP runtime: the
# encoder's compute, binarisation and arithmetic-coding streams plus the next step's input /
# lookahead stream must not share queues (govideocompressor_amd/__init__.py)
if not os.environ.get("GPU_MAX_HW_QUEUES", "").isdigit() or int(os.environ["GPU_MAX_HW_QUEUES"]) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def _knob_env() -> bool:
    """--allow-knobs, read before argparse so the MIVC_BENCH_* shape defaults below only apply
    with it (models/knobs.py)."""
    return "--allow-knobs" in sys.argv


def _memory(env, merged) -> dict:
    """Per-rank memory footprint (rank 0): HBM peak, host RSS, the pinned budget of one of
    the ranks sharing this host, and the merge's host buffer (rank 0 only, world x bytes)."""
    import torch

    from govideocompressor_amd.runtime.device import pinned_budget
    try:
        import psutil
        rss = psutil.Process().memory_info().rss
    except Exception:  # pragma: no cover
        rss = 0
    return {"hbm_peak_gb": round(torch.cuda.max_memory_allocated(env.device) / 1e9, 2),
            "hbm_reserved_gb": round(torch.cuda.max_memory_reserved(env.device) / 1e9, 2),
            "host_rss_gb": round(rss / 1e9, 2), "pinned_budget_gb": round(pinned_budget() / 1e9, 2),
            "merge_bytes_per_step": int(len(merged)) if merged is not None else 0}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    knobs = _knob_env()
    env_ = os.environ if knobs else {}
    ap.add_argument("--slots", type=int, default=int(env_.get("MIVC_BENCH_SLOTS", "256")),
                    help="segments encoded concurrently per GPU")
    ap.add_argument("--frames", type=int, default=int(env_.get("MIVC_BENCH_FRAMES", "60")),
                    help="frames per segment (GOP length)")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--crf", type=float, default=23.0)
    ap.add_argument("--bframes", type=int, default=int(env_.get("MIVC_BENCH_BFRAMES", "3")),
                    help="B pictures between anchors (x264 default 3)")
    ap.add_argument("--cavlc", action="store_true",
                    help="Constrained Baseline CAVLC (the round-1 encoder) instead of Main CABAC")
    ap.add_argument("--no-8x8dct", dest="t8x8", action="store_false",
                    help="Main profile (no High-profile 8x8 transform)")
    ap.add_argument("--no-partitions", dest="partitions", action="store_false",
                    help="P macroblocks 16x16 only (no P_8x8 / P_16x8 / P_8x16)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--merged-out", default=None,
                    help="rank 0 writes the last timed step's merged Annex-B stream here")
    ap.add_argument("--no-quality", dest="quality", action="store_false",
                    help="skip the PSNR/SSIM measurement of the first warmup step")
    ap.add_argument("--allow-knobs", action="store_true",
                    help="apply MIVC_* encoder / bench knobs from the environment (refused otherwise); "
                         "every applied value is reported under config.env")
    a = ap.parse_args()
    from govideocompressor_amd.models import knobs as K
    env_knobs = K.check_environment(a.allow_knobs)

    import torch

    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip
    from govideocompressor_amd.parallel import dist as D

    env = D.init(prefer_gpu=True)
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    if env.world != a.gpus:
        if env.is_main:
            print(f"warning: --gpus {a.gpus} but WORLD_SIZE {env.world}", file=sys.stderr)
    overrides = K.encoder_overrides(H264Params) if a.allow_knobs else {}
    p = H264Params(**{**dict(width=a.width, height=a.height, fps=30.0, crf=a.crf, bframes=a.bframes, cabac=not a.cavlc,
                             t8x8=a.t8x8, partitions=a.partitions), **overrides})
    enc = GpuH264Encoder(p, slots=a.slots, device=env.device,
                         entropy_threads=int(os.environ.get("MIVC_ENTROPY_THREADS", "16")))
    B, F = a.slots, a.frames

    merger = D.SegmentMerge(env)
    merge_stream = torch.cuda.Stream(device=env.device)
    merge_pool = cf.ThreadPoolExecutor(max_workers=1)

    def synth(step: int):
        # rank r renders global slots [r * B, (r + 1) * B): the content (and so the merged
        # stream) does not depend on how the global batch is split over ranks
        seed = 1000 + step * 7919
        return synth_clip(B, F, a.width, a.height, seed=seed, device=env.device, slot0=env.rank * B)

    def merge(res):
        # CC-2/CC-3 + concat on a side stream: overlaps the next batch's encode
        with torch.cuda.device(env.device), torch.cuda.stream(merge_stream):
            return merger.run([r.parts() for r in res])

    synth_stream = torch.cuda.Stream(device=env.device)
    step_wall: list[float] = []  # host time at which each step's results were complete

    def synth_async(step: int):
        """Input of a later step on a side stream (it overlaps the current step's encode the way
        a decoder feeding the encoder would), with the event that ends it."""
        with torch.cuda.stream(synth_stream):
            clip = synth(step)
            ev = torch.cuda.Event()
            ev.record(synth_stream)
        return clip, ev

    def run_steps(first: int, n: int, metrics_first: bool = False):
        """n steps: synthesize (new content) -> lookahead + encode -> merge on rank 0.
        Step k + 1's input synthesis and lookahead run on a side stream while step k encodes,
        step k's entropy tail overlaps step k + 1's first kernels (encode_async), and the
        merge of step k overlaps the encode of step k + 1 -- all inside the n steps: nothing is
        prepared beyond the last step, and the last step is collected before the clock stops."""
        clip, ev = synth_async(first)
        ana = enc.analyse_async(clip[0], stream=synth_stream)
        fut = prev = first_res = res = None

        def collect(pend):
            # step k - 1's results once step k is issued: its last coder groups and NAL
            # wrapping ran beside step k's first kernels (encode_async)
            nonlocal fut, first_res, res
            res = pend.result()
            step_wall.append(time.perf_counter())
            if fut is not None:
                fut.result()
            fut = merge_pool.submit(merge, res)
            if first_res is None:
                first_res = res

        for k in range(n):
            (y, u, v), cur_ev, cur_ana = clip, ev, ana
            if k + 1 < n:
                clip, ev = synth_async(first + k + 1)
                ana = enc.analyse_async(clip[0], stream=synth_stream)
            torch.cuda.current_stream().wait_event(cur_ev)
            pend = enc.encode_async(y, u, v, idr_base=env.rank * B, metrics=(metrics_first and k == 0),
                                    analysis=cur_ana)
            del y, u, v
            if prev is not None:
                collect(prev)
            prev = pend
        collect(prev)
        merged = fut.result()
        return first_res, res, merged

    # PSNR/SSIM are measured on the (untimed) first warmup step: quality measurement is not
    # part of encoding (an ffmpeg/x264 encode computes none unless asked); the timed steps
    # encode the same content distribution (new seed per step).
    qres = None
    stage_ms = {}
    if a.warmup:
        # per-stage device time (HIP events + roctx ranges) on the untimed warmup only
        enc.stage_timer.enabled = True
        qres, _, _ = run_steps(-100, a.warmup, metrics_first=a.quality)
        stage_ms = {k: round(v["s"] * 1000.0 / a.warmup, 2) for k, v in enc.stage_timer.summary().items()}
        enc.stage_timer.enabled = False
        # the timed loop keeps two input batches alive (step k encodes while k + 1 is
        # synthesized): let the caching allocator map the second one (on the synthesis
        # stream, whose pool it comes from) before the clock starts
        spare = synth_async(-99)
        torch.cuda.synchronize()
        del spare
    D.barrier(env)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step_wall.clear()
    step_wall.append(time.perf_counter())
    _, res, merged = run_steps(0, a.steps)
    torch.cuda.synchronize()
    D.barrier(env)
    t1 = time.perf_counter()
    elapsed = D.max_over_ranks(env, t1 - t0)
    merge_pool.shutdown()
    total_frames = env.world * B * F * a.steps
    fps = total_frames / elapsed
    # quality of the warmup step, rate of the last timed step (this rank), averaged over ranks
    q = qres if (qres is not None and a.quality) else None
    psnr = D.sum_over_ranks(env, sum(r.psnr_y for r in q) / len(q) if q else 0.0) / env.world
    ssim = D.sum_over_ranks(env, sum(r.ssim_y for r in q) / len(q) if q else 0.0) / env.world
    nbytes = D.sum_over_ranks(env, float(sum(r.nbytes() for r in res)))
    kbps = nbytes * 8 / (env.world * B * F / p.fps) / 1000.0
    if env.is_main:
        out = {
            "metric": "encoded frames/sec (whole node), 1080p30->H.264 CRF23",
            "value": round(fps, 2),
            "unit": "frames/s",
            "n_gpus": env.world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1000.0, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "uint8 (8-bit 4:2:0 samples, int32 transforms)",
            "data": "synthetic (GPU-generated moving-texture YUV, new content every step)",
            "config": {
                "model": f"H.264 {p.profile_name()}, gfx950 batched encoder, CRF from GPU lookahead",
                "resolution": f"{a.width}x{a.height}",
                "fps": 30,
                "crf": a.crf,
                "global_batch": env.world * B * F,
                "seq_len": F,
                "segments_per_gpu": B,
                "parallelism": f"dp{env.world} (segment-parallel)",
                # every effective encoder setting (H264Params), environment knobs included
                "encoder": dataclasses.asdict(p),
                "slices_per_picture": p.eff_slices(),
                "env": {"allow_knobs": a.allow_knobs, "encoder_overrides": overrides, **{
                    k: v for k, v in env_knobs.items() if k != "unknown" and v}},
                "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                "entropy_threads": enc.entropy_threads,
            },
            "quality": {"psnr_y_db": round(psnr, 3), "ssim_y": round(ssim, 4), "bitrate_kbps": round(kbps, 1),
                        "measured_on": "first warmup step (untimed)" if q else "n/a (no warmup step)",
                        "merged_bytes": len(merged) if merged is not None else 0,
                        # identity of the last timed step's merged stream (same seed: byte-identity
                        # check of kernel changes, tools/gpu/ab_steps.sh)
                        "merged_sha256_16": hashlib.sha256(memoryview(merged)).hexdigest()[:16]
                        if merged is not None else None},
            "timings_rank0_s": {k: round(v, 3) for k, v in enc.timings.items()},
            # interval between consecutive timed steps' completion on rank 0 (the first includes
            # the first input's synthesis and lookahead; the last is not shortened by the merge)
            "step_wall_ms_rank0": [round(1000.0 * (b - a_), 1) for a_, b in zip(step_wall, step_wall[1:])],
            "stage_device_ms_per_step_rank0": {"measured_on": "warmup steps (untimed)", **stage_ms},
            "encoder_stats_rank0": {k: round(v, 4) for k, v in enc.stats.items()},
            "memory_rank0": _memory(env, merged),
        }
        if a.merged_out and merged is not None:
            with open(a.merged_out, "wb") as f:
                f.write(memoryview(merged))
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    enc.close()
    D.shutdown(env)


if __name__ == "__main__":
    main()
