"""MI355X H.264 encoder: B closed-GOP segments encoded concurrently on one GPU.

This is the MI355X-native replacement of the reference worker's codec call
(``ffmpeg -i <idx>.mp4 -threads 4 -vcodec libx264 c<idx>.mp4``, client.go:101-130;
preset expansion at server.go:67-71).  Where the reference runs one segment per
3-vCPU droplet, here a *batch* of segments shares one GPU: every kernel launch
covers all B slots, so the serial wavefront stages (intra coding, deblocking)
still expose B x (MB rows) independent waves.

Per frame step t (frame t of every slot):
  prep (pad/scale) -> [P: me -> encode_inter] -> encode_intra (wavefront)
  -> deblock (wavefront) -> metrics, then the decision records (MbHeader +
  coefficients) are copied to pinned host memory on a side stream and CAVLC
  coded by a host thread pool while the GPU runs step t+1.
"""
from __future__ import annotations

import concurrent.futures as cf
import math
import os
import time
from dataclasses import dataclass

import numpy as np
import torch

from ..ops import native
from .gop import PicPlan, dpb_frames, fixed_types, gop_plan, h264_plan  # noqa: F401  (re-exported)

MB_HDR_BYTES = 64
NO_COST = 0x3FFFFFFF  # me.hip kNoCost
# csrc/kernels/route.h SlotRoute (32 bytes): one per slot and coding step
ROUTE_DTYPE = np.dtype([("kind", "i1"), ("cur", "i1"), ("n0", "i1"), ("l1", "i1"), ("l0", "i1", (4,)),
                        ("w1", "<i2", (4,)), ("dsf", "<i2", (4,)), ("dcopy", "i1", (4,)), ("flags", "u1"),
                        ("col_l1", "i1"), ("disp", "<i2")])
assert ROUTE_DTYPE.itemsize == 32
SK = {"P": 0, "B": 1, "I": 2}
SF_REF, SF_DEBLOCK = 1, 2
WP_LOG2 = 6  # luma / chroma log2 weight denominators of explicit weighted prediction
COEF_PER_MB = 408


@dataclass
class H264Params:
    width: int
    height: int
    fps: float = 30.0
    crf: float | None = 23.0       # CRF (None -> fixed qp)
    qp: int = 26                    # used when crf is None
    ip_offset: int = 3              # I-frame QP = P QP - ip_offset (ipratio 1.4)
    me_range: int = 8              # integer full-search radius around the best predictor
    subpel: int = 2
    i4x4: bool = True
    # x264 --partitions i8x8 (its default with --8x8dct): Intra8x8 MBs (High profile) tried where
    # Intra4x4 is (I pictures, scene cuts), closed loop with the 8x8 transform, sa8d ranking
    i8x8: bool = True
    # Intra4x4 trial for the (rare) intra MBs of P frames.  Off by default: a P-frame
    # intra MB is coded by the wavefront kernel, whose latency (x chain length) is
    # dominated by the 16 serial I4x4 block trials; these MBs are ~0.1-1% of a P frame.
    i4x4_in_p: bool = False
    deblock: bool = True
    chroma_qp_offset: int = 0
    vui: bool = True
    # CRF per-frame QPs from the GPU lookahead (rc/lookahead.py); False = flat CRF QP
    lookahead: bool = True
    # lowres search range around the quarter-resolution seed (rc/lookahead.py RANGES): +-4 and
    # +-6 are BD-rate-identical on the content suite (-0.01 %, profiles/r4_la_range_rd.json),
    # +-4 searches 81 positions instead of 169
    la_range: int = 4
    # lowres weighted prediction in the lookahead (rc/lookahead.py GpuLookahead(weighted=True)):
    # P candidates of fades / flashes priced with the weights the encoder's weightp will use
    la_weights: bool = True
    # x264 --scenecut: a P frame whose lowres inter cost saves less than this percent of
    # its intra cost is coded all-intra (I4x4/I16x16 MBs) at the I-frame QP; 0 disables
    scenecut: int = 40
    # x264 --aq-mode 1 (variance AQ): per-MB QP offset strength * 1.0397 * (log2(AC energy)
    # - 14.427); 0 disables (every MB at the frame QP)
    aq_strength: float = 1.0
    # x264 --mbtree (default on): lookahead propagation of inter-frame references -> per-MB
    # QP offsets (csrc/kernels/mbtree.hip), with x264's CRF compensation; needs the lookahead
    mbtree: bool = True
    # entropy coder: CABAC (x264's default; Main profile) or CAVLC (Constrained Baseline)
    cabac: bool = True
    # x264 --bframes 3: B pictures between P anchors (non-reference, temporal direct); CABAC
    # only (the Baseline CAVLC path has no B slices).  b_qp_offset: x264 --pbratio 1.3 as a QP
    # offset (6 log2 1.3 = 2.27) over the distance-weighted QP of the B picture's references
    bframes: int = 3
    b_qp_offset: float = 6.0 * math.log2(1.3)
    # x264 --b-adapt: 1 ("fast", x264's default) places B pictures per slot from the lookahead's
    # lowres costs (rc/badapt.py, lookahead.hip la_multi); 0 = the fixed pattern.  Round 4
    # measured +10 % BD-rate against the fixed pattern (profiles/r4_content_rd.md: the
    # unweighted integer-pel lowres costs made fades look like new content and the rule placed
    # too few of this encoder's cheap B pictures).  With lowres weighting (la_weights) and
    # --b-bias 100, one pattern per batch: -1.85 % BD-rate on the suite mean, but -3.2 % fps at
    # the headline (profiles/r5_badapt_rd.md) -- the default keeps the fixed pattern's
    # throughput, -preset slow and up place B pictures adaptively
    b_adapt: int = 0
    # x264 --b-bias: > 0 places more B pictures (B costs * 100 / (120 + bias), run thresholds)
    b_bias: int = 0
    # x264's intra-MB guards on the b-adapt decision (rc/badapt.py): P(i+2 | i) more than half
    # intra keeps both pictures P, a closing P more than a third intra ends the B run.  Off:
    # measured +4 % BD-rate on top of b-adapt's own loss (profiles/r5_content_rd.md -- they
    # force P pictures where this encoder's B pictures are cheap, fades above all)
    badapt_guard: bool = False
    # b-adapt decides ONE pattern for the batch from the lowres costs summed over its slots (each
    # slot still anchors at its own cuts / forced positions): per-slot patterns mix P and B
    # pictures in every coding step, so each step runs both the P and the B kernels at partial
    # width (same-box A/B: 9.9k vs 13.0k fps at the headline config, profiles/r5_badapt_ab.md)
    badapt_shared: bool = True
    # radius of the lowres refinement around the distance-scaled vector in la_multi (the P
    # costs at distance >= 2 and the list-1 search of the B cost): 2 = +-2 lowres pixels
    badapt_range: int = 2
    # x264 seeds its motion search from the lookahead's lowres motion: the P search and both B
    # searches get one more candidate, the picture's lowres vector x 2 scaled to its reference
    # distance (when the lookahead ran on the coded MB grid)
    lowres_seed: bool = True
    # integer search radius of the two B-picture searches (their predictors are the scaled
    # co-located vectors of temporal direct, so a small window suffices)
    b_me_range: int = 4
    # Jacobi passes of the P_Skip-aware vector choice after ME (csrc/kernels/bframe.hip
    # p_mv_refine): 0 disables.  Each pass settles the field one MB further: 2 -> 4 passes is
    # -2.55 % BD-rate on the content suite for -1.3 % headline fps (profiles/r4_knob_sweep.md)
    skip_refine: int = 4
    # skip-refine passes after the first re-evaluate only MBs next to an MB the previous pass
    # moved (exact: the others derive the same predictor at the same cost); False = every MB
    # every pass (A/B switch)
    refine_skip: bool = True
    # x264 --8x8dct (default on): High profile, the 8x8 transform chosen per inter MB where
    # its sa8d beats the 4x4 satd; CABAC only (the CAVLC path stays Constrained Baseline)
    t8x8: bool = True
    # x264 --weightb (default on): implicit weighted bi-prediction in B pictures
    # (weighted_bipred_idc 2: list weights from the POC distances, 8.4.2.3.1)
    weightb: bool = True
    # x264 --partitions p8x8 (default): P macroblocks may split into 8x8 quadrants with their
    # own vectors (coded as P_8x8 / P_16x8 / P_8x16); CABAC only.  part_overhead: bits
    # charged to a split beyond its mvds; part_min_satd: 16x16 SATD at or below which the
    # split is not searched
    partitions: bool = True
    # x264 --partitions b8x8: B macroblocks split into quadrants that pick their own candidate
    # (direct, L0, L1, bi of the MB's two searched vectors): B_16x8 / B_8x16 / B_8x8
    bpartitions: bool = True
    # (1080p CRF23 sweep, profiles/r2_partition_sweep.txt: 8 / 2000 -> -0.5% bits at equal
    # PSNR for ~1% of the step time; a threshold of 0 searches every MB for the same bits)
    part_overhead: int = 8
    part_min_satd: int = 2000
    # x264-style ME early termination: a search whose best candidate (the predictors and
    # their neighbours) already has SAD <= this skips the window and the integer search
    # (B pictures: the temporal-direct predictor); 0 disables
    p_early_sad: int = 0
    b_early_sad: int = 1024
    # B macroblocks whose temporal-direct cost (SATD + lambda, a b_decide pre-pass) is <= b_gate
    # (< 0: -b_gate lambdas) skip both list searches and take direct (x264's early B_Skip /
    # direct termination); 0 disables.  1080p RD sweep (profiles/r3_b_gate_rd.md): 2400 ->
    # -8.8 % BD-rate (PSNR-Y) and +7..20 % fps against no gate
    b_gate: int = 2400
    # x264 --trellis 1 (default): rate-distortion choice of the levels of inter MBs
    # (encode_inter.hip trellis_lite4x4 / trellis_lite8_chunk); 1 = the 4x4 luma blocks only,
    # 2 = also the 8x8 luma and the chroma AC blocks; trellis_lambda scales its SSD lambda
    trellis: int = 2
    # x264 --direct: "temporal" (co-located motion scaled by POC distances: every MB decides in
    # parallel) or "spatial" (the neighbours' motion: b_decide keeps each searched MB's best
    # explicit candidate, then bframe.hip b_spatial_decide derives the exact spatial motion in
    # an MB wavefront and takes direct where its SATD + lambda is not dearer; RD in
    # profiles/r3_direct_rd.md)
    direct: str = "temporal"
    # spatial direct: direct is taken when its cost <= the explicit candidate's + direct_bias * lambda
    direct_bias: int = 8
    # spatial direct: the B gate skips the searches of MBs with static co-located motion only
    # (wavefront decision) / of MBs whose estimated spatial direct cost passes b_gate (fast path)
    spatial_gate: bool = True
    # spatial direct decision: False (fast, default) = priced in parallel from an estimate of the
    # neighbours' motion, then made exact by an integer-only decoding-order pass
    # (b_spatial_exact) and re-predicted where the estimate was off (b_spatial_fixup); True =
    # the exact derivation priced MB by MB inside the wavefront (b_spatial_decide, ~3.7 ms per
    # picture of serial chain)
    spatial_wavefront: bool = False
    # fast path: a direct quadrant whose exact motion lies further than this many quarter
    # samples from the priced estimate keeps the estimate as explicit motion (B_L0 / L1 / Bi
    # partitions, explicit 8x8 sub-blocks: the priced prediction, plus mvd bits) instead of being
    # re-predicted with motion nobody priced.  Content suite (profiles/r4_content_rd.md), BD-rate
    # vs temporal direct: -1 (always re-predict) +111 %, 0 (always explicit) +68 %, 4 +25 %.
    # The exact direct field follows the *sequential* decisions (the first MBs of a picture
    # derive zero motion and spread it unless they are coded explicitly), which no parallel
    # estimate reproduces -- temporal direct stays the default
    spatial_fix_tol: int = 4
    # temporal direct: B_Direct_16x16 preferred by tdirect_bias * lambda in b_decide's choice
    # (-0.36 % BD-rate at 8, profiles/r3_direct_rd.md)
    tdirect_bias: int = 8
    # x264 --b-pyramid normal: in a run of two or more B pictures the middle one is a reference
    # picture (coded first, predicted from the two anchors, then a reference of the others and of
    # the next P); needs spatial direct (temporal direct's co-located motion would come from a B)
    pyramid: bool = False
    trellis_lambda: float = 1.0
    # the same rate-distortion levels on the intra MBs' final encode (encode_intra.hip,
    # lane-parallel h264_trellis.h grp_trellis4x4; x264 applies --trellis 1 to every MB):
    # -1 = follow `trellis`, 0 = dead-zone quantisation (rounding 1/3), 1 / 2 as `trellis`.
    # Off by default: on the content suite (profiles/r5_content_rd.md) intra trellis at the
    # inter lambda is +1.1 % BD-rate (worse on 6 of 7 classes: the coarser intra pictures cost
    # the pictures predicted from them more than the levels save) and -0.7 % fps
    intra_trellis: int = 0
    # deblock non-reference B pictures even when neither metrics nor the reconstruction
    # are requested (x264 --full-recon); the bitstream does not depend on it
    full_recon: bool = False
    # level_idc written in the SPS (-level); 0 = the lowest level the size / rate fits
    level_idc: int = 0
    # x264 --ref 3 (its default): P macroblocks choose among the 3 latest anchors (ref_idx in
    # the records; searches of the farther pictures seeded by the distance-scaled list-0[0]
    # vector, radius ref_range); B pictures' temporal direct follows the co-located block's
    # reference.  CABAC only (the Baseline CAVLC path keeps one reference).  ref_gate: MBs
    # whose list-0[0] cost (SATD + lambda * bits) is <= ref_gate are not searched in the farther pictures
    refs: int = 3
    # x264 --weightp (default 2 outside Baseline): explicit weighted prediction of a P picture's
    # RefPicList0[0] (luma and chroma weight / offset, denominator 2^6) where the source
    # statistics say the brightness or contrast changed (fades, flashes): the weights come from
    # the means and variances of the two source pictures (wp_min_mean: mean change in luma
    # levels, wp_min_scale: contrast change, either one turns weighting on).  CABAC only.
    weightp: bool = True
    wp_min_mean: float = 2.0
    wp_min_scale: float = 0.08
    ref_range: int = 4
    # content suite (profiles/r4_knob_sweep.md): 3000 is -0.67 % BD-rate and +1.5 % fps vs 1500
    ref_gate: int = 3000
    # slices per picture (x264 --slices): whole MB rows each.  The GPU arithmetic coder codes
    # one slice per lane, so S slices give S times the independent serial chains per picture
    # (and the intra wavefront restarts at every slice); each slice costs a header and the
    # prediction across its top edge.  CABAC only (spatial direct: the fast path).
    # 0 = auto: one slice up to 68 MB rows (1080p), else one per 34 rows (4K: 4, 8K: 8) --
    # a 4K picture in one slice is a 4x longer serial chain for the arithmetic coder at a
    # quarter of the slots per batch (4K encode-only, 64 x 30 frames: 1105 fps with 1 slice,
    # 1693 with 4, 1742 with 8; at 1080p 4 slices cost +2.3 % BD-rate for +2 % fps)
    slices: int = 0

    def slice_count(self) -> int:
        hmb = (self.height + 15) // 16
        n = int(self.slices)
        if n <= 0:
            wavefront_spatial = self.direct == "spatial" and self.spatial_wavefront  # one slice only
            n = 1 if (hmb <= 68 or wavefront_spatial) else -(-hmb // 34)
        return n

    def slice_rows(self) -> int:
        """MB rows per slice (0: one slice per picture)."""
        hmb = (self.height + 15) // 16
        n = self.slice_count()
        if n <= 1 or not self.cabac:
            return 0
        return max(1, -(-hmb // n))

    def eff_slices(self) -> int:
        r = self.slice_rows()
        return 1 if r == 0 else -(-((self.height + 15) // 16) // r)

    def eff_bframes(self) -> int:
        return max(0, int(self.bframes)) if self.cabac else 0

    def eff_pyramid(self) -> bool:
        return bool(self.pyramid and self.eff_bframes() >= 2)

    def eff_refs(self) -> int:
        return max(1, min(4, int(self.refs))) if self.cabac else 1

    def eff_weightp(self) -> bool:
        return bool(self.weightp and self.cabac)

    def eff_t8x8(self) -> bool:
        return bool(self.t8x8 and self.cabac)

    def eff_intra_trellis(self) -> int:
        return int(self.trellis if self.intra_trellis < 0 else self.intra_trellis)

    def eff_partitions(self) -> bool:
        return bool(self.partitions and self.cabac)

    def host_cfg(self) -> dict:
        return dict(width=self.width, height=self.height, fps=self.fps, qp=self.qp,
                    deblock=int(self.deblock), chroma_qp_offset=self.chroma_qp_offset,
                    vui=int(self.vui), cabac=int(self.cabac), bframes=self.eff_bframes(), t8x8=int(self.eff_t8x8()),
                    weighted_bipred=2 if self.weightb else 0, refs=self.eff_refs(), weightp=int(self.eff_weightp()),
                    level_idc=int(self.level_idc), pyramid=int(self.eff_pyramid()))

    def profile_name(self) -> str:
        if not self.cabac:
            return "Constrained Baseline CAVLC"
        nb = self.eff_bframes()
        return (("High CABAC 8x8dct" if self.eff_t8x8() else "Main CABAC") + (" i8x8" if self.eff_t8x8() and self.i8x8 else "")
                + (" p8x8" if self.eff_partitions() else "") + (" b8x8" if self.eff_partitions() and self.bpartitions and self.eff_bframes() else "") + (f" ref{self.eff_refs()}" if self.eff_refs() > 1 else "")
                + (" weightp" if self.eff_weightp() else "")
                + (f" {nb}B" + (" b-adapt" if self.b_adapt else "") + (" b-pyramid" if self.eff_pyramid() else "")
                   + f" {self.direct}-direct" if nb else "")
                + (" weightb" if nb and self.weightb else "")
                + (f" slices{self.eff_slices()}" if self.eff_slices() > 1 else ""))

    def frame_qps(self) -> tuple[int, int]:
        """(qp_I, qp_P).  CRF maps to the P-frame QP (x264 scale without MB-tree);
        per-frame adaptation is done by :mod:`govideocompressor_amd.rc`."""
        qp_p = int(round(self.crf)) if self.crf is not None else int(self.qp)
        qp_p = max(0, min(51, qp_p))
        return max(0, qp_p - self.ip_offset), qp_p


class SegmentResult:
    """One encoded closed-GOP segment: parameter sets + one slice NAL per frame.

    ``bitstream`` (the Annex-B piece) is joined on first access; the segment merge
    packs ``parts()`` straight into its staging buffer instead."""

    __slots__ = ("frames", "nals", "bits", "header", "psnr_y", "psnr_u", "psnr_v", "ssim_y", "_bs", "order")

    def __init__(self, frames: int, nals: list[bytes] | None = None, bits: list[int] | None = None,
                 header: bytes = b"", bitstream: bytes | None = None, order: list[int] | None = None):
        self.frames = frames
        self.nals = list(nals or [])
        self.bits = list(bits or [])
        self.header = header
        self._bs = bitstream
        # display index of each NAL (coding order); identity without B pictures
        self.order = list(order) if order is not None else list(range(len(self.nals)))
        self.psnr_y = self.psnr_u = self.psnr_v = self.ssim_y = 0.0

    @property
    def bitstream(self) -> bytes:
        if self._bs is None:
            self._bs = self.header + b"".join(self.nals)
        return self._bs

    def display_prefix(self, c: int) -> list[bytes]:
        """The slice NALs of display pictures 0..c-1 (a coding-order prefix when c-1 was an
        anchor: encode(anchors_at=...))."""
        out = [n for n, d in zip(self.nals, self.order) if d < c]
        if any(d >= c for d in self.order[:len(out)]):
            raise ValueError(f"pictures 0..{c - 1} are not a coding-order prefix (encode with anchors_at)")
        return out

    def parts(self) -> list[bytes]:
        return [self._bs] if self._bs is not None else [self.header, *self.nals]

    def nbytes(self) -> int:
        return len(self._bs) if self._bs is not None else len(self.header) + sum(len(n) for n in self.nals)


def _resolve(device) -> torch.device:
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


class CabacPoolExhausted(RuntimeError):
    """The batch's CABAC symbols outgrew the pool (very low QPs); encode() grows it and retries."""


class PendingEncode:
    """A batch issued by :meth:`GpuH264Encoder.encode_async`."""

    def __init__(self, enc, finish, planes, kw, results=None):
        self._enc, self._finish, self._planes, self._kw = enc, finish, planes, kw
        self._res = results
        self._exc: BaseException | None = None
        self._done = finish is None

    def done(self) -> bool:
        return self._done

    def _complete(self) -> None:
        """Run the batch's finish once; a pool overflow is kept for result() to redo."""
        if self._done:
            return
        try:
            self._res = self._finish()
        except BaseException as e:  # noqa: BLE001
            self._exc = e
        self._done = True
        self._finish = None
        if self in self._enc._inflight:
            self._enc._inflight.remove(self)

    def result(self) -> list:
        self._complete()
        if isinstance(self._exc, CabacPoolExhausted):
            # drain the other batch in flight (its copy threads read the pools), grow, redo
            enc = self._enc
            for other in list(enc._inflight):
                other._complete()
            torch.cuda.synchronize(enc.dev)
            enc._alloc_cabac(enc.cab_G, grow=enc.cab_grow * 4)
            enc.stats["cabac_pool_regrow"] = enc.stats.get("cabac_pool_regrow", 0) + 1
            self._exc = None
            self._res = enc.encode(*self._planes, **self._kw)
        if self._exc is not None:
            raise self._exc
        self._planes = None
        return self._res


class GpuH264Encoder:
    """Batched gfx950 H.264 encoder: Main profile with GPU CABAC (default) or Constrained
    Baseline with GPU CAVLC; ``entropy="cpu"`` codes the slices with the host writers."""

    def __init__(self, params: H264Params, slots: int, device: str | torch.device = "cuda",
                 entropy_threads: int | None = None, entropy: str = "gpu", cabac_group: int | None = None):
        """cabac_group: frame steps whose slices the GPU CABAC arithmetic coder runs at once
        (default 20; its serial stage runs one slice per lane, so throughput scales with it).
        The symbol pool budget per MB is MIVC_CABAC_SYMS_PER_MB (default 128 per frame step,
        shared by the steps of a group)."""
        if params.width % 2 or params.height % 2:
            raise ValueError("width and height must be even")
        if params.direct not in ("temporal", "spatial"):
            raise ValueError("direct must be 'temporal' or 'spatial'")
        if params.eff_pyramid() and params.direct != "spatial":
            # temporal direct scales the co-located block's motion by its own list-0 picture,
            # which is the current list 0 only while RefPicList1[0] is a P anchor
            raise ValueError("b-pyramid needs spatial direct prediction (direct='spatial')")
        if entropy not in ("gpu", "cpu"):
            raise ValueError("entropy must be 'gpu' or 'cpu'")
        if params.eff_slices() > 1 and params.direct == "spatial" and params.eff_bframes() and params.spatial_wavefront:
            raise ValueError("slices > 1: spatial direct needs the fast path (spatial_wavefront=False)")
        self.entropy = entropy
        self.p = params
        self.slice_rows = params.slice_rows()
        self.S = params.eff_slices()
        self.B = int(slots)
        self.dev = _resolve(device)
        self.hip = native.hip()
        self.host = native.host()
        self.wmb = (params.width + 15) // 16
        self.hmb = (params.height + 15) // 16
        self.W, self.H = self.wmb * 16, self.hmb * 16
        self.nmb = self.wmb * self.hmb
        self._mbtree = None  # [B, F, nmb] MB-tree QP offsets of the batch being encoded
        self._wp = self._wp_steps = None  # explicit weights of the batch's P pictures (see _weights)
        B, H, W, nmb, dev = self.B, self.H, self.W, self.nmb, self.dev
        u8, i16, i32 = torch.uint8, torch.int16, torch.int32

        def planes():
            return (torch.zeros((B, H, W), dtype=u8, device=dev),
                    torch.zeros((B, H // 2, W // 2), dtype=u8, device=dev),
                    torch.zeros((B, H // 2, W // 2), dtype=u8, device=dev))

        # padded source pictures of the current step.  (Preparing step t + 1's on a side stream
        # while step t encodes was measured 3-4 % slower: the copy then competes with the step's
        # first kernels for memory bandwidth instead of running alone between them.)
        self.src = planes()
        self.nb = params.eff_bframes()
        self.nref = params.eff_refs()
        # Every slot follows its own GOP plan (models/gop.py h264_plan): its reference pictures
        # live in a per-slot pool of reconstruction buffers [B, nbuf, plane] (the DPB's
        # max_num_ref_frames, one more for the picture being coded, one scratch buffer for
        # non-reference B pictures), with the half-sample planes of every reference picture
        # (built once, shared by all pictures predicting from it) and, for B pictures, the
        # decision records of the co-located candidates.  One SlotRoute per slot and coding
        # step (csrc/kernels/route.h) tells the kernels which buffer plays which role.
        self.nref_frames = dpb_frames(self.nref, params.eff_pyramid(), self.nb)
        self.nbuf = self.nref_frames + 2
        NB = self.nbuf
        self.rec_pool = (torch.zeros((B, NB, H, W), dtype=u8, device=dev),
                         torch.zeros((B, NB, H // 2, W // 2), dtype=u8, device=dev),
                         torch.zeros((B, NB, H // 2, W // 2), dtype=u8, device=dev))
        self.rec = [tuple(p[:, i] for p in self.rec_pool) for i in range(NB)]  # per-buffer views (tools)
        self.hp_bytes = 3 * (H + 8) * (W + 8)
        self.hp_pool = torch.empty(B * NB * self.hp_bytes + 64, dtype=u8, device=dev)
        self.hdr = [torch.zeros((B, nmb, MB_HDR_BYTES), dtype=u8, device=dev) for _ in range(2)]
        self.coef = [torch.zeros((B, nmb, COEF_PER_MB), dtype=i16, device=dev) for _ in range(2)]
        self.nz = torch.zeros((B, nmb, 16), dtype=u8, device=dev)
        self.mv = torch.zeros((B, nmb, 2), dtype=i16, device=dev)
        self.mv_tmp = torch.zeros((B, nmb, 2), dtype=i16, device=dev)
        self.mv8 = torch.zeros((B, nmb, 4, 2), dtype=i16, device=dev)   # P partition vectors
        self.prev_mv = torch.zeros((B, nmb, 2), dtype=i16, device=dev)
        self.me_cost = torch.zeros((B, nmb), dtype=i32, device=dev)
        self.intra_cost = torch.zeros((B, nmb), dtype=i32, device=dev)
        self.pred = torch.zeros((B, nmb, 256), dtype=u8, device=dev)
        self.mref = torch.zeros((B, nmb), dtype=torch.int8, device=dev)
        self.dref = torch.zeros((B, nmb, 4), dtype=torch.int8, device=dev)
        self.seed = [torch.zeros((B, nmb, 2), dtype=i16, device=dev) for _ in range(2)]  # lowres search seeds L0 / L1
        self._slot_ar = torch.arange(B, device=dev)
        if self.nref > 1:
            # searches of RefPicList0[1 ..] (P pictures) and the reference choice per MB
            K = self.nref - 1
            self.xmv = torch.zeros((K, B, nmb, 2), dtype=i16, device=dev)
            self.xcost = torch.zeros((K, B, nmb), dtype=i32, device=dev)
            self.xpred = torch.zeros((K, B, nmb, 256), dtype=u8, device=dev)
            self.xpm = torch.zeros((B, nmb, 2), dtype=i16, device=dev)
        if self.nb:
            # B pictures: the list-1 search, temporal direct vectors and the mode decision
            self.mv1 = torch.zeros((B, nmb, 2), dtype=i16, device=dev)
            self.me_cost1 = torch.zeros((B, nmb), dtype=i32, device=dev)
            self.pred1 = torch.zeros((B, nmb, 256), dtype=u8, device=dev)
            self.pred_b = torch.zeros((B, nmb, 256), dtype=u8, device=dev)
            self.cost_b = torch.zeros((B, nmb), dtype=i32, device=dev)
            self.pm0 = torch.zeros((B, nmb, 2), dtype=i16, device=dev)
            self.pm1 = torch.zeros((B, nmb, 2), dtype=i16, device=dev)
            self.dmv = torch.zeros((B, nmb, 16), dtype=i16, device=dev)
            self.czero = torch.zeros((B, nmb), dtype=u8, device=dev)  # colZeroFlag bits (spatial direct)
            self.sfix = torch.zeros((B, nmb), dtype=u8, device=dev)   # direct MBs re-predicted after the exact pass
            # records of every reference picture (the co-located candidates of B pictures)
            self.col_pool = torch.zeros((B, NB, nmb, MB_HDR_BYTES), dtype=u8, device=dev)
        if params.eff_weightp():
            self.src_me = torch.zeros((B, H, W), dtype=u8, device=dev)  # inverse-weighted luma for ME
        self.intra_flag = torch.zeros((B, nmb), dtype=u8, device=dev)
        self.aq = torch.zeros((B, nmb), dtype=torch.int8, device=dev)     # per-MB QP offsets (AQ)
        self.qp_flags = torch.zeros((B, nmb), dtype=u8, device=dev)       # MB carries mb_qp_delta
        self.intra_count = torch.zeros((B,), dtype=i32, device=dev)
        self.qp = torch.zeros((B,), dtype=i32, device=dev)
        # error flags, one buffer per batch in flight (encode_async: the next batch zeroes its own
        # while the previous one's coder may still report); pinned host copies of them
        self.err_bufs = [torch.zeros((1,), dtype=i32, device=dev) for _ in range(2)]
        self.err = self.err_bufs[0]
        self.h_err = [torch.zeros((1,), dtype=i32).pin_memory() for _ in range(2)]
        self._batch_no = 0
        self._ring_last: list = [None, None]  # per CABAC ring: (copied event, future, wrap futures) of its last group
        self._inflight: list = []             # encode_async batches not yet finished (oldest first)
        self.p_intra_mbs = torch.zeros((), dtype=torch.int64, device=dev)  # intra MBs coded in P frames
        self.far_ref_mbs = torch.zeros((), dtype=torch.int64, device=dev)  # P MBs choosing RefPicList0[1 ..]
        self.sfix_mbs = torch.zeros((), dtype=torch.int64, device=dev)  # fast spatial direct: MBs re-predicted
        self.sconv_mbs = torch.zeros((), dtype=torch.int64, device=dev)  # ... and MBs made explicit
        # pinned staging for the entropy stage (double-buffered)
        if entropy == "cpu":
            self.h_hdr = [torch.empty((B, nmb, MB_HDR_BYTES), dtype=u8).pin_memory() for _ in range(2)]
            self.h_coef = [torch.empty((B, nmb, COEF_PER_MB), dtype=i16).pin_memory() for _ in range(2)]
        elif params.cabac:
            self._alloc_cabac(cabac_group)
        else:
            i64 = torch.int64
            mbb = int(self.hip.cavlc_mb_bytes())
            # worst case ~3.3 kbit per MB (I_PCM-like); 4 kbit per MB + header slack
            self.cap_words = nmb * 128 + 64
            self.cav_mbs = torch.zeros((B, nmb, mbb), dtype=u8, device=dev)
            self.cav_len = torch.zeros((B, nmb), dtype=i32, device=dev)
            self.cav_off = torch.zeros((B, nmb), dtype=i64, device=dev)
            self.cav_trail = torch.zeros((B,), dtype=i32, device=dev)
            self.cav_total = torch.zeros((B,), dtype=i64, device=dev)
            self.cav_words = torch.zeros((B, self.cap_words), dtype=torch.int32, device=dev)
            self.cav_out_off = torch.zeros((B,), dtype=i64, device=dev)
            self.cav_hdr_bits = [torch.zeros((B, 16), dtype=i32, device=dev) for _ in range(2)]
            self.cav_hdr_nbits = [torch.zeros((B,), dtype=i32, device=dev) for _ in range(2)]
            self.h_hdr_bits = [torch.zeros((B, 16), dtype=i32).pin_memory() for _ in range(2)]
            self.h_hdr_nbits = [torch.zeros((B,), dtype=i32).pin_memory() for _ in range(2)]
            self.cav_sizes = [torch.zeros((B,), dtype=i32, device=dev) for _ in range(2)]
            self.h_sizes = [torch.zeros((B,), dtype=i32).pin_memory() for _ in range(2)]
            self.cav_out = [torch.zeros((B * self.cap_words * 4,), dtype=u8, device=dev) for _ in range(2)]
            # compressed bytes land in one of 3 pinned host buffers (grown on demand): frame t's
            # NAL wrapping may still read buffer t%3 while frames t+1, t+2 are copied out
            self.h_out: list = [None, None, None]
            self.out_done = [torch.cuda.Event() for _ in range(2)]
            self.copy_pool = cf.ThreadPoolExecutor(max_workers=1)
        self.copy_stream = torch.cuda.Stream(device=dev)
        self.copy_done = [torch.cuda.Event() for _ in range(2)]
        self.compute_done = [torch.cuda.Event() for _ in range(2)]
        nthreads = entropy_threads or min(16, max(2, (os.cpu_count() or 4)))
        self.entropy_threads = nthreads
        self.pool = cf.ThreadPoolExecutor(max_workers=nthreads)
        self.cfg = params.host_cfg()
        self.timings: dict[str, float] = {}
        self.stats: dict[str, float] = {}
        # per-stage device time (HIP events on the encode stream, resolved lazily) and roctx
        # ranges; off unless MIVC_STAGE_TIMING=1 or enabled by the caller (bench.py warmup)
        from ..obs.timers import EventTimer
        self.stage_timer = EventTimer(enabled=os.environ.get("MIVC_STAGE_TIMING", "0") == "1")

    def _alloc_cabac(self, group: int | None, grow: int = 1):
        """GPU CABAC buffers.  Per frame step (copy stream): block masks, per-MB coding state
        and symbol counts.  Per group of G steps, double-buffered (group g binarises into
        ring g % 2 while the arithmetic coder drains ring (g - 1) % 2 on the entropy stream):
        the symbol pool (slice outputs are written over their consumed symbols), slice
        regions / symbol totals, slice headers, output sizes and the compacted bytes."""
        B, nmb, dev = self.B, self.nmb, self.dev
        u8, i32, i64 = torch.uint8, torch.int32, torch.int64
        G = int(group or os.environ.get("MIVC_CABAC_GROUP", 20))
        if not 1 <= G <= 64:
            raise ValueError("cabac_group must be in 1..64")
        self.cab_G = G
        # pool budget: an average per MB and frame step plus one picture's worth of intra-heavy
        # headroom per group (IDR / scene cuts / low QPs run to several hundred symbols per MB)
        per_mb = int(os.environ.get("MIVC_CABAC_SYMS_PER_MB", 96)) * grow
        peak_mb = int(os.environ.get("MIVC_CABAC_PEAK_SYMS_PER_MB", 768)) * grow
        self.cab_grow = grow
        gap = int(self.hip.cabac_gap())
        L = G * B * self.S  # one lane per slice: G steps x B slots x S slices
        self.cab_pool_cap = B * nmb * (G * per_mb + peak_mb) + L * (gap + 8) + 64
        self.cab_pool = [torch.empty((self.cab_pool_cap + 64,), dtype=torch.int16, device=dev) for _ in range(2)]
        self.cab_pool_used = torch.zeros((2,), dtype=i64, device=dev)
        # slice RBSP <= header (64 B) + 10 bits per symbol + flush: 1.25 bytes per pool symbol
        comp_cap = (self.cab_pool_cap * 5) // 4 + 80 * L
        self.cab_comp = [torch.empty((comp_cap,), dtype=u8, device=dev) for _ in range(2)]
        self.cab_comp_off = [torch.zeros((L,), dtype=i64, device=dev) for _ in range(2)]
        self.cab_base = [torch.zeros((L,), dtype=i64, device=dev) for _ in range(2)]
        self.cab_total = [torch.zeros((L,), dtype=i32, device=dev) for _ in range(2)]
        self.cab_bytes = [torch.zeros((L,), dtype=i32, device=dev) for _ in range(2)]
        self.h_cab_bytes = [torch.zeros((L,), dtype=i32).pin_memory() for _ in range(2)]
        self.h_pool_used = [torch.zeros((1,), dtype=i64).pin_memory() for _ in range(2)]
        self.cab_hdr_bits = [torch.zeros((L, 16), dtype=i32, device=dev) for _ in range(2)]
        self.cab_hdr_nbits = [torch.zeros((L,), dtype=i32, device=dev) for _ in range(2)]
        self.h_cab_hdr_bits = [torch.zeros((L, 16), dtype=i32).pin_memory() for _ in range(2)]
        self.h_cab_hdr_nbits = [torch.zeros((L,), dtype=i32).pin_memory() for _ in range(2)]
        self.cab_mask = torch.zeros((B, nmb), dtype=i32, device=dev)
        self.cab_nb = torch.zeros((B, nmb, int(self.hip.cabac_nb_bytes())), dtype=u8, device=dev)
        self.cab_cnt = torch.zeros((B, nmb), dtype=i32, device=dev)
        self.cab_off = torch.zeros((B, nmb), dtype=i64, device=dev)
        self.cab_tot = torch.zeros((B * self.S,), dtype=i32, device=dev)
        self.entropy_stream = torch.cuda.Stream(device=dev)
        self.cab_bin_done = [torch.cuda.Event() for _ in range(2)]
        self.cab_done = [torch.cuda.Event() for _ in range(2)]
        # the coder's compaction writes the slice bytes straight into these pinned buffers
        # (one per ring; a group that does not fit falls back to the device buffer + D2H)
        # (capped by the rank's pinned budget: 8 ranks share the host, runtime/device.py)
        from ..runtime.device import pinned_budget
        self.cab_host_cap = min(comp_cap, int(os.environ.get("MIVC_CABAC_HOST_MB", 1024)) << 20, pinned_budget() // 4)
        self.h_cab_out = [torch.empty((self.cab_host_cap,), dtype=u8).pin_memory() for _ in range(2)]
        self.copy_pool = cf.ThreadPoolExecutor(max_workers=1)

    # ------------------------------------------------------------------ helpers
    @staticmethod
    def _ptr(t: torch.Tensor) -> int:
        return t.data_ptr()

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.dev).cuda_stream

    def parameter_sets(self) -> bytes:
        return self.host.parameter_sets(self.cfg)

    # ------------------------------------------------------------------ stages
    def _prep(self, y, u, v, t: int):
        """y/u/v: [B, F, h, w] display-size planes on the device; pads frame t of every slot."""
        B, F, h, w = y.shape
        cs = u.shape[2] * u.shape[3]
        self.hip.prep(y[:, t].data_ptr(), u[:, t].data_ptr(), v[:, t].data_ptr(), w, h, F * h * w, F * cs, B,
                      self._ptr(self.src[0]), self._ptr(self.src[1]), self._ptr(self.src[2]),
                      self.p.width, self.p.height, self.W, self.H, self._stream())

    def _prep_step(self, y, u, v, disp: np.ndarray, disp_d: torch.Tensor):
        """Pad each slot's display picture of this coding step (``disp``: [B] display indices,
        ``disp_d`` the same on the device): one launch, per-slot frame selection."""
        if (disp == disp[0]).all():
            return self._prep(y, u, v, int(disp[0]))
        B, F, h, w = y.shape
        cs = u.shape[2] * u.shape[3]
        self.hip.prep(y.data_ptr(), u.data_ptr(), v.data_ptr(), w, h, F * h * w, F * cs, B,
                      self._ptr(self.src[0]), self._ptr(self.src[1]), self._ptr(self.src[2]),
                      self.p.width, self.p.height, self.W, self.H, self._stream(), disp_d.data_ptr())

    @staticmethod
    def _dist_scale(poc: int, poc0: int, poc1: int) -> tuple[int, int]:
        """(DistScaleFactor, direct_copy) of temporal direct (clause 8.4.1.2.3; C division)."""
        def tdiv(x: int, y: int) -> int:
            q = abs(x) // abs(y)
            return q if (x >= 0) == (y >= 0) else -q
        tb = max(-128, min(127, poc - poc0))
        td = max(-128, min(127, poc1 - poc0))
        if td == 0:
            return 0, 1
        tx = tdiv(16384 + abs(tdiv(td, 2)), td)
        return max(-1024, min(1023, (tb * tx + 32) >> 6)), 0

    def _encode_step(self, st: dict, hdr, coef, cut=None):
        """One coding step of every slot (csrc/kernels/route.h): each slot codes its own
        picture (``st``: the step's routing and host-side tables, built by _step_tables).  P
        and B pictures of different slots share the step: the P kernels skip the B slots and
        the B kernels the P slots (they write disjoint per-slot rows of the shared buffers);
        the intra, deblocking and half-sample kernels then run over all slots at once.
        cut: optional [B] bool device tensor -- slots whose P picture is a scene cut (every MB
        intra, as an I picture would be)."""
        s = self._stream()
        B, wmb, hmb = self.B, self.wmb, self.hmb
        P = self._ptr
        sy, su, sv = (P(x) for x in self.src)
        py, pu, pv = (P(x) for x in self.rec_pool)  # reconstruction pools [B, nbuf, plane]
        hpp = P(self.hp_pool)
        rt, NB = st["route"], self.nbuf
        aq = 0
        mbt = self._mbtree
        stt = self.stage_timer
        if self.p.aq_strength > 0 or mbt is not None:
            aq = P(self.aq)
            extra, stride = 0, 0
            # MB-tree offsets belong to referenced pictures (the routing picks each slot's row)
            if mbt is not None and mbt.shape[2] == self.nmb:
                extra, stride = mbt.data_ptr(), mbt.shape[1] * self.nmb
            with stt("aq"):
                self.hip.aq_offsets(B, wmb, hmb, sy, su, sv, float(self.p.aq_strength), aq, s, extra, stride, rt)
        cqo = self.p.chroma_qp_offset
        inter = st["P"] or st["B"]
        if inter:
            self.intra_count.zero_()
        seed0 = seed1 = 0
        if inter and self._la_mv is not None:
            # the lookahead's lowres vector of each slot's picture (to the previous picture),
            # scaled to the reference distances of its lists
            v = self._la_mv[self._slot_ar, st["disp_d"].long()].reshape(B, self.nmb)
            dxy = torch.stack((((v << 16) >> 16), v >> 16), -1).float()
            self.seed[0].copy_((dxy * st["sscale"][0][:, None, None]).round_().clamp_(-2048, 2047))
            seed0 = P(self.seed[0])
            if st["B"]:
                self.seed[1].copy_((dxy * st["sscale"][1][:, None, None]).round_().clamp_(-2048, 2047))
                seed1 = P(self.seed[1])
        if st["P"]:
            sy_me, wp = sy, 0
            if st["wp"] is not None:
                # weighted RefPicList0[0]: the searches see the inverse-weighted source (identity
                # weights for the other slots)
                wp = st["wp"].data_ptr()
                with stt("weightp"):
                    self.hip.wp_src(sy, P(self.src_me), st["wp_src"].data_ptr(), B, self.H * self.W, s)
                sy_me = P(self.src_me)
            with stt("me_p"):
                self.hip.me(B, wmb, hmb, sy_me, py, P(self.prev_mv), P(self.mv), P(self.me_cost), P(self.pred),
                            P(self.intra_cost), P(self.qp), self.p.me_range, self.p.subpel, s, hpp, aq, 1,
                            self.p.p_early_sad, 0, 0, 0, rt, NB, 0, SK["P"], seed0)
                if getattr(self, "_chg", None) is None:  # p_mv_refine change masks (passes >= 2 skip settled MBs)
                    self._chg = [torch.zeros((B, self.nmb), dtype=torch.uint8, device=self.dev) for _ in range(2)]
                for it in range(int(self.p.skip_refine)):
                    a_, b_ = (self.mv, self.mv_tmp) if it % 2 == 0 else (self.mv_tmp, self.mv)
                    self.hip.p_refine(B, wmb, hmb, sy_me, py, hpp, P(a_), P(b_), P(self.me_cost), P(self.prev_mv),
                                      P(self.pred), P(self.qp), aq, s, rt, NB,
                                      0 if (it == 0 or not self.p.refine_skip) else P(self._chg[(it - 1) % 2]),
                                      P(self._chg[it % 2]) if self.p.refine_skip else 0)
                if int(self.p.skip_refine) % 2:
                    self.mv.copy_(torch.where(st["pmask"][:, None, None], self.mv_tmp, self.mv))
            mv8 = 0
            if self.p.eff_partitions():
                with stt("part"):
                    self.hip.p_part8(B, wmb, hmb, sy_me, py, hpp, P(self.mv), P(self.prev_mv), P(self.me_cost),
                                     P(self.pred), P(self.mv8), P(self.qp), aq, int(self.p.part_overhead),
                                     int(self.p.part_min_satd), s, rt, NB)
                mv8 = P(self.mv8)
            # the next P picture's predictors: the list-0[0] vectors of this one (P slots)
            self.prev_mv.copy_(torch.where(st["pmask"][:, None, None], self.mv, self.prev_mv))
            nr = st["maxn0"]
            if nr > 1:
                # farther list-0 pictures: 16x16 searches seeded by the list-0[0] vectors scaled by
                # the temporal distances (per slot), then the per-MB choice (cost + ref_idx bits)
                with stt("me_ref"):
                    for k in range(1, nr):
                        self.xpm.copy_((self.mv.float() * st["xscale"][k - 1][:, None, None]).round_().clamp_(-2048, 2047))
                        self.hip.me(B, wmb, hmb, sy, py, P(self.xpm), P(self.xmv[k - 1]), P(self.xcost[k - 1]),
                                    P(self.xpred[k - 1]), 0, P(self.qp), int(self.p.ref_range), self.p.subpel, s,
                                    hpp, aq, 1, self.p.p_early_sad, P(self.me_cost), self._ref_gate(),
                                    P(self.prev_mv), rt, NB, k, SK["P"])
                    self.hip.me_ref_select(B, wmb, hmb, nr, P(self.mv), mv8, P(self.me_cost), P(self.pred),
                                           P(self.xmv), P(self.xcost), P(self.xpred), P(self.mref), P(self.qp), aq,
                                           s, rt)
                    self.far_ref_mbs += ((self.mref > 0) & st["pmask"][:, None]).sum()
            else:
                self.mref.zero_()
            if cut is not None:
                self.intra_cost.masked_fill_(cut[:, None], -1)  # intra beats any inter cost
            with stt("inter"):
                self.hip.encode_inter(B, wmb, hmb, sy, su, sv, py, pu, pv, py, pu, pv, P(self.pred), P(self.mv),
                                      P(self.me_cost), P(self.intra_cost), P(self.qp), cqo, P(hdr), P(coef),
                                      P(self.nz), P(self.intra_flag), P(self.intra_count), s, aq,
                                      t8=int(self.p.eff_t8x8()), mv8=mv8, mref=P(self.mref), wp=wp,
                                      trellis=int(self.p.trellis), trellis_lambda=float(self.p.trellis_lambda),
                                      route=rt, nbuf=NB)
        if st["B"]:
            br = self.p.b_me_range
            spatial = self.p.direct == "spatial"
            sfast = spatial and not self.p.spatial_wavefront
            mode = 2 if sfast else int(spatial)
            # wavefront spatial direct cannot be priced before the wavefront: its gate passes
            # static MBs only; the fast path prices its estimate in the pre-pass, which it needs
            bg = int(self.p.b_gate) if (not spatial or sfast or self.p.spatial_gate) else 0
            dbias = int(self.p.tdirect_bias) if not spatial else (int(self.p.direct_bias) if sfast else 0)
            with stt("me_b"):
                self.hip.b_direct(B, wmb, hmb, P(self.col_pool), [0], [1], P(self.dmv), P(self.pm0), P(self.pm1), s,
                                  P(self.dref), rt, NB, P(self.czero))
                if bg != 0 or sfast:  # direct costs first: MBs that direct already predicts well are not searched
                    self.hip.b_decide(B, wmb, hmb, sy, py, py, hpp, hpp, P(self.mv), P(self.mv1), P(self.me_cost),
                                      P(self.me_cost1), P(self.pred), P(self.pred1), P(self.pm0), P(self.pm1),
                                      P(self.dmv), P(self.qp), aq, P(hdr), P(self.pred_b), P(self.cost_b), s, [32],
                                      P(self.dref), [], [], 1, spatial=mode, route=rt, nbuf=NB, czero=P(self.czero))
                gate = P(self.cost_b) if bg != 0 else 0
                self.hip.me(B, wmb, hmb, sy, py, P(self.pm0), P(self.mv), P(self.me_cost), P(self.pred),
                            P(self.intra_cost), P(self.qp), br, self.p.subpel, s, hpp, aq, 1, self.p.b_early_sad,
                            gate, bg, 0, rt, NB, 0, SK["B"], seed0)
                # the L1 search skips the open-loop intra estimate the L0 search just wrote
                self.hip.me(B, wmb, hmb, sy, py, P(self.pm1), P(self.mv1), P(self.me_cost1), P(self.pred1), 0,
                            P(self.qp), br, self.p.subpel, s, hpp, aq, 1, self.p.b_early_sad, gate, bg, 0, rt, NB,
                            4, SK["B"], seed1)
            with stt("b_decide"):
                self.hip.b_decide(B, wmb, hmb, sy, py, py, hpp, hpp, P(self.mv), P(self.mv1), P(self.me_cost),
                                  P(self.me_cost1), P(self.pred), P(self.pred1), P(self.pm0), P(self.pm1),
                                  P(self.dmv), P(self.qp), aq, P(hdr), P(self.pred_b), P(self.cost_b), s, [32],
                                  P(self.dref), [], [], 0, int(self.p.eff_partitions() and self.p.bpartitions),
                                  int(bg != 0 or sfast), mode, dbias, route=rt, nbuf=NB, czero=P(self.czero))
            if sfast:
                with stt("b_spatial"):
                    self.hip.b_spatial_exact(B, wmb, hmb, P(hdr), P(self.intra_cost), P(self.cost_b), P(self.czero),
                                             P(self.sfix), s, rt, self.slice_rows, int(self.p.spatial_fix_tol))
                    self.sfix_mbs += (self.sfix == 1).sum()
                    self.sconv_mbs += (self.sfix == 2).sum()
                    self.hip.b_spatial_fixup(B, wmb, hmb, P(hdr), P(self.sfix), py, hpp, py, hpp, P(self.pred_b), s,
                                             rt, NB)
            elif spatial:
                with stt("b_spatial"):
                    self.hip.b_spatial(B, wmb, hmb, P(hdr), P(self.col_pool), sy, py, hpp, [py], [hpp], [32],
                                       P(self.pred_b), P(self.err), s, P(self.intra_cost), P(self.cost_b), P(self.qp),
                                       aq, int(self.p.direct_bias), rt, NB)
            with stt("inter"):
                self.hip.encode_inter(B, wmb, hmb, sy, su, sv, py, pu, pv, py, pu, pv, P(self.pred_b), P(self.mv),
                                      P(self.cost_b), P(self.intra_cost), P(self.qp), cqo, P(hdr), P(coef),
                                      P(self.nz), P(self.intra_flag), P(self.intra_count), s, aq, pu, pv, 1,
                                      int(self.p.eff_t8x8()), 0, [32], [], [], 0, 0, int(self.p.trellis),
                                      float(self.p.trellis_lambda), rt, NB)
        if inter:
            self.p_intra_mbs += self.intra_count.sum()
            flag_ptr, count_ptr = P(self.intra_flag), P(self.intra_count)
        else:
            self.prev_mv.zero_()
            flag_ptr, count_ptr = 0, 0
        trial = not inter or self.p.i4x4_in_p or cut is not None
        if getattr(self, "_intra_prog", None) is None:
            # cross-workgroup row progress of the multi-workgroup I-picture wavefront (this
            # encoder's own: [slice units][kMaxRows = 272] ints, zeroed by the launcher on `s`)
            per = -(-hmb // self.slice_rows) if self.slice_rows > 0 else 1
            self._intra_prog = torch.zeros(B * per * 272, dtype=torch.int32, device=self.dev)
        with stt("intra"):
            self.hip.encode_intra(B, wmb, hmb, sy, su, sv, py, pu, pv, P(self.qp), cqo, P(hdr), P(coef), P(self.nz),
                                  flag_ptr, count_ptr, P(self.err), int(self.p.i4x4 and trial), s, aq,
                                  int(self.p.i8x8 and self.p.eff_t8x8() and trial), rt, NB, self.slice_rows,
                                  trellis=self.p.eff_intra_trellis(), trellis_lambda=float(self.p.trellis_lambda),
                                  gprog=P(self._intra_prog), gprog_ints=self._intra_prog.numel())
        if aq:
            # MBs without mb_qp_delta take QP_pred (clause 7.4.5): their records must say so
            # before deblocking reads every MB's QP
            self.hip.qp_fixup(B, wmb, hmb, P(hdr), P(coef), P(self.nz), P(self.qp_flags), P(self.qp), s, self.slice_rows)
        # A non-reference B picture's reconstruction feeds nothing but its own intra MBs
        # (which predict from unfiltered samples), so its in-loop filter only matters when
        # someone looks at the picture: metrics (PSNR / SSIM) or keep_recon.  The bitstream
        # is identical either way (cf. x264, which reconstructs non-reference frames fully
        # only with --full-recon): the routing flags SF_DEBLOCK accordingly.
        if self.p.deblock and st["deblock"]:
            with stt("deblock"):
                self.hip.deblock(B, wmb, hmb, py, pu, pv, P(hdr), P(self.nz), cqo, 0, 0, P(self.err), s, rt, NB)
        if st["ref"]:
            # the reference pictures' half-sample planes (shared by every picture predicting from
            # them) and, for B pictures, their records as co-located candidates
            with stt("halfpel"):
                self.hip.me_halfpel(B, self.W, self.H, py, hpp, s, rt, NB)
            if self.nb and st["col_dst"] is not None:
                self.col_pool.view(B * NB, self.nmb, MB_HDR_BYTES).index_copy_(
                    0, st["col_dst"], hdr.index_select(0, st["col_src"]))

    def _plans(self, F: int, cuts_h: np.ndarray, anchors_at) -> list[list[PicPlan]]:
        """Per-slot coding-order plans: B pictures placed by the lookahead (x264 --b-adapt 1,
        rc/badapt.py) when its costs are at hand, else x264's fixed --b-adapt 0 pattern; anchors
        at the forced positions and at each slot's own scene cuts.  ``anchors_at``: display
        indices forced for every slot, or one iterable per slot."""
        per_slot = (isinstance(anchors_at, (list, tuple)) and len(anchors_at) == self.B and len(anchors_at) > 0
                    and all(isinstance(a, (list, tuple, set, frozenset)) for a in anchors_at))
        common = set() if per_slot else {int(d) for d in anchors_at}
        cache: dict[str, list[PicPlan]] = {}
        plans = []
        multi = getattr(self, "_la_multi", None)
        multi_intra = getattr(self, "_la_multi_intra", None) if self.p.badapt_guard else None
        adaptive = multi is not None and multi.shape[:2] == (self.B, F)
        shared = None
        if adaptive:
            from ..rc.badapt import b_adapt_types, with_anchors
            if self.p.badapt_shared:
                mi = None if multi_intra is None else multi_intra.sum(axis=0)
                shared = b_adapt_types(self._la_costs[:, :, 1].sum(axis=0), multi.sum(axis=0), multi[:, :, 0].sum(axis=0),
                                       self.nb, self._la_blocks * self.B, common, int(self.p.b_bias), mi)
        for b in range(self.B):
            forced = {int(d) for d in anchors_at[b]} if per_slot else common
            forced = forced | {d for d in range(1, F) if cuts_h[b, d]}
            if shared is not None:
                ty = with_anchors(shared, forced)
            elif adaptive:
                ty = b_adapt_types(self._la_costs[b, :, 1], multi[b], multi[b, :, 0], self.nb, self._la_blocks, forced,
                                   int(self.p.b_bias), None if multi_intra is None else multi_intra[b])
            else:
                ty = fixed_types(F, self.nb, forced)
            if ty not in cache:
                cache[ty] = h264_plan(ty, self.nref, self.p.eff_pyramid(), self.nref_frames)
            plans.append(cache[ty])
        return plans

    def _step_tables(self, plans: list[list[PicPlan]], F: int) -> list[dict]:
        """Routing of every coding step: the [F, B] SlotRoute table (one upload) and per step the
        picture kinds present, the P-slot mask, far-reference vector scales, explicit weights
        and the record-store indices of its reference pictures."""
        B, NB, dev = self.B, self.nbuf, self.dev
        rt = np.zeros((F, B), dtype=ROUTE_DTYPE)
        rt["l1"] = -1
        rt["l0"] = -1
        rt["disp"] = -1
        rt["w1"] = 32
        rt["dcopy"] = 1
        K = max(1, self.nref - 1)
        xscale = np.zeros((F, K, B), dtype=np.float32)
        # lowres-seed scales (quarter-pel per lowres pixel): list 0 / P and list 1
        sscale = np.zeros((F, 2, B), dtype=np.float32)
        deblock_nonref = bool(self._full_recon)
        col = {}
        colcache: dict[int, tuple] = {}  # one routing column per distinct plan (slots share plans)
        for b in range(B):
            key = id(plans[b])
            if key not in colcache:
                c = np.zeros(F, dtype=ROUTE_DTYPE)
                c["l1"] = -1
                c["l0"] = -1
                c["w1"] = 32
                c["dcopy"] = 1
                xs = np.zeros((F, K), dtype=np.float32)
                ss = np.zeros((F, 2), dtype=np.float32)
                kinds = {pic.d: pic.kind for pic in plans[b]}
                refs_at = []
                for t, pic in enumerate(plans[b]):
                    r = c[t]
                    r["kind"] = SK[pic.kind]
                    r["cur"] = pic.buf
                    r["n0"] = max(1, len(pic.refs0))
                    r["l0"][:len(pic.bufs0)] = pic.bufs0
                    r["flags"] = (SF_REF if pic.ref else 0) | (SF_DEBLOCK if (pic.ref or deblock_nonref) else 0)
                    r["disp"] = pic.d
                    if pic.kind != "I":
                        # lowres vector of picture d points to d - 1: x 2 (full res) x 4 (quarter pel)
                        ss[t, 0] = 8.0 * (pic.d - pic.refs0[0])
                        if pic.kind == "B":
                            ss[t, 1] = -8.0 * (pic.refs1[0] - pic.d)
                    if pic.kind == "P":
                        d0 = max(1, pic.d - pic.refs0[0])
                        for k in range(1, len(pic.refs0)):
                            xs[t, k - 1] = (pic.d - pic.refs0[k]) / d0
                    elif pic.kind == "B":
                        r["l1"] = pic.buf1
                        r["col_l1"] = int(kinds[pic.l1] == "B")
                        for k, rd in enumerate(pic.refs0):
                            dsf, copy = self._dist_scale(pic.poc, 2 * rd, 2 * pic.l1)
                            r["dsf"][k] = dsf
                            r["dcopy"][k] = copy
                            r["w1"][k] = dsf >> 2 if self.p.weightb and not copy and -64 <= (dsf >> 2) <= 128 else 32
                    if pic.ref and pic.kind != "I":
                        refs_at.append((t, pic.buf))
                colcache[key] = (c, xs, refs_at, ss)
            c, xs, refs_at, ss = colcache[key]
            rt[:, b] = c
            xscale[:, :, b] = xs
            sscale[:, :, b] = ss
            for t, buf in refs_at:
                col.setdefault(t, []).append((b, b * NB + buf))
        rt_d = torch.from_numpy(rt.view(np.uint8).reshape(F, B * 32).copy()).to(dev)
        kinds_d = torch.from_numpy(np.ascontiguousarray(rt["kind"])).to(dev)
        xs_d = torch.from_numpy(xscale).to(dev)
        ss_d = torch.from_numpy(sscale).to(dev)
        self._route_dev = rt_d  # keeps the table alive while the launches read it
        pmask_d = kinds_d == 0
        # the co-located motion copies of every reference step: one upload, sliced per step (a
        # pair of small uploads per step cost ~1 ms of host latency each between two batches)
        cts = sorted(col)
        flat = np.array([e for t in cts for e in col[t]], dtype=np.int64).reshape(-1, 2)
        flat_d = torch.from_numpy(np.ascontiguousarray(flat.T)).to(dev) if len(flat) else None
        cofs, o = {}, 0
        for t in cts:
            cofs[t] = (o, o + len(col[t]))
            o += len(col[t])
        steps = []
        for t in range(F):
            k = rt["kind"][t]
            n0p = rt["n0"][t][k == 0]
            st = dict(route=rt_d[t].data_ptr(), P=bool((k == 0).any()), B=bool((k == 1).any()),
                      pmask=pmask_d[t], maxn0=int(n0p.max()) if n0p.size else 1, xscale=xs_d[t],
                      deblock=bool((rt["flags"][t] & SF_DEBLOCK).any()), ref=bool((rt["flags"][t] & SF_REF).any()),
                      wp=None, wp_src=None, col_src=None, col_dst=None, kinds=k, sscale=ss_d[t])
            if t in cofs:
                a0, a1 = cofs[t]
                st["col_src"] = flat_d[0, a0:a1]
                st["col_dst"] = flat_d[1, a0:a1]
            steps.append(st)
        return steps

    # ------------------------------------------------------------------ entropy (GPU CAVLC)
    def _ref_gate(self) -> int:
        return int(self.p.ref_gate)

    def _frame_params(self, b: int, pic: PicPlan, t: int, qp_frame: int, idr_ids: list[int]) -> dict:
        """Slice-header fields of slot b's picture at coding step t."""
        fp = dict(idr=int(pic.kind == "I"), frame_num=pic.frame_num, idr_pic_id=idr_ids[b] & 0xFFFF, qp=qp_frame,
                  slice_type=pic.slice_type, nal_ref_idc=pic.nal_ref_idc, poc=pic.poc,
                  direct_spatial=int(pic.kind == "B" and self.p.direct == "spatial"))
        if pic.kind != "I":
            fp["num_ref_l0"] = max(1, len(pic.refs0))
            fp["num_ref_l1"] = 1
            if pic.mod_l0:
                fp["mod_l0"] = [tuple(m) for m in pic.mod_l0]
        # identity weights (this slot's picture did not qualify, another slot's of the step
        # did) write the same all-default table as a step without weights, so a segment's
        # bytes do not depend on the other segments of its batch
        if pic.kind == "P" and self._wp is not None and any(
                int(x) != (1 << WP_LOG2 if i % 2 == 0 else 0) for i, x in enumerate(self._wp[t, b])):
            fp["wp"] = [WP_LOG2, WP_LOG2] + [int(x) for x in self._wp[t, b]]
        return fp

    def _weights(self, y, u, v, plans: list[list[PicPlan]]) -> None:
        """x264 --weightp: per P picture and slot, the explicit weights of RefPicList0[0] from
        the source statistics (wp_stats: means and variances of the two pictures' planes):
        scale = sqrt(var_cur / var_ref), offset = mean_cur - scale * mean_ref, used when the mean
        moved by wp_min_mean levels or the contrast by wp_min_scale (fades, flashes).  Tables
        are per coding step ([F, B], identity weights elsewhere)."""
        self._wp = None
        self._wp_steps = None
        if not self.p.eff_weightp() or not any(pic.kind == "P" for plan in plans for pic in plan):
            return
        B, F, h, w = y.shape
        st = torch.empty((B, F, 6), dtype=torch.int64, device=self.dev)
        self.hip.wp_stats(y.data_ptr(), u.data_ptr(), v.data_ptr(), w, h, B * F, st.data_ptr(), self._stream())
        sh = st.cpu().numpy().astype(np.float64)
        n = np.array([w * h, w * h / 4, w * h / 4])
        mean = sh[..., 0::2] / n
        var = np.maximum(sh[..., 1::2] / n - mean ** 2, 0.0)
        one = 1 << WP_LOG2
        # every (slot, step) holding a P picture: its display index and its RefPicList0[0]'s
        bs, ts, ds, rs = [], [], [], []
        for b, plan in enumerate(plans):
            for t, pic in enumerate(plan):
                if pic.kind == "P":
                    bs.append(b)
                    ts.append(t)
                    ds.append(pic.d)
                    rs.append(pic.l0)
        bs, ts, ds, rs = (np.array(a, dtype=np.int64) for a in (bs, ts, ds, rs))
        m1, m0 = mean[bs, ds], mean[bs, rs]
        v1, v0 = var[bs, ds], var[bs, rs]
        scale = np.where(v0 > 1e-3, np.sqrt(v1 / np.maximum(v0, 1e-3)), 1.0)
        use = (np.abs(m1[:, 0] - m0[:, 0]) >= self.p.wp_min_mean) | (np.abs(scale[:, 0] - 1) >= self.p.wp_min_scale)
        if not use.any():
            return
        wq = np.clip(np.round(scale * one), 0, 127)
        oq = np.clip(np.round(m1 - wq / one * m0), -128, 127)
        wp = np.zeros((F, B, 6), dtype=np.int32)
        wp[:, :, 0::2] = one
        for c in range(3):
            wp[ts[use], bs[use], 2 * c] = wq[use, c]
            wp[ts[use], bs[use], 2 * c + 1] = oq[use, c]
        on = np.zeros(F, dtype=bool)
        on[ts[use]] = True
        self._wp = wp
        dev8 = np.zeros((F, B, 8), dtype=np.int32)
        dev8[..., 0], dev8[..., 1], dev8[..., 2] = wp[..., 0], wp[..., 1], WP_LOG2
        dev8[..., 3:7], dev8[..., 7] = wp[..., 2:6], WP_LOG2
        wp_dev = torch.from_numpy(dev8).to(self.dev)
        wp_src = torch.from_numpy(np.ascontiguousarray(dev8[..., :3])).to(self.dev)
        self._wp_steps = [(wp_dev[t], wp_src[t]) if on[t] else None for t in range(F)]
        self.stats["weightp_pictures"] = int(use.sum())

    @staticmethod
    def _cabac_groups(F: int, G: int) -> list[tuple[int, int]]:
        """(first step, steps) of the arithmetic-coder groups of an F-step batch: the IDR step
        alone (its slices hold several times the symbols of a P / B slice, so in a group of G
        steps they set the whole launch's length: 205 of 270 ms per batch in round 4's trace),
        then G steps each, the last full-size group split in two so the coder's tail after
        the final encode kernel (nothing left to overlap it with) is half a group."""
        head = [1] if (F > 2 and G > 1) else []
        R = F - len(head)
        sizes = [G] * (R // G) + ([R % G] if R % G else [])
        if sizes and sizes[-1] > max(1, G // 2):
            last = sizes.pop()
            sizes += [(last + 1) // 2, last // 2]
        sizes = head + sizes
        out, t0 = [], 0
        for n in sizes:
            out.append((t0, n))
            t0 += n
        return out

    def _gpu_cabac_bin(self, k: int, g: int, j: int, t: int, pics: list[PicPlan], qps_t, idr_ids: list[int],
                       qp_dev: torch.Tensor, route: int):
        """Binarise coding step t (records hdr[k]/coef[k]) into the symbol pool of its group
        ring, on the *copy* stream (the caller's current stream): the records are free
        again once this is done, whatever the arithmetic coder is doing.  Every slot's slice
        type and list size come from the step's routing.
        qp_dev: [B] int32 slice QPs of this step in a buffer that outlives the launch."""
        B, BS = self.B, self.B * self.S
        r = g & 1
        if j == 0:
            self.cab_pool_used[r].zero_()
        self._header_bits_into(self.h_cab_hdr_bits[r][j * BS:(j + 1) * BS], self.h_cab_hdr_nbits[r][j * BS:(j + 1) * BS],
                               self.cab_hdr_bits[r][j * BS:(j + 1) * BS], self.cab_hdr_nbits[r][j * BS:(j + 1) * BS],
                               pics, t, qps_t, idr_ids)
        P = self._ptr
        self.hip.cabac_bin(B, self.wmb, self.hmb, P(self.hdr[k]), P(self.coef[k]), P(self.cab_mask), P(self.cab_nb),
                           P(self.cab_cnt), P(self.cab_off), P(self.cab_tot), P(self.cab_pool[r]), self.cab_pool_cap,
                           self.cab_pool_used[r].data_ptr(), self.cab_base[r][j * BS:].data_ptr(),
                           self.cab_total[r][j * BS:].data_ptr(), P(qp_dev), pics[0].slice_type, 1, 1,
                           int(self.p.eff_t8x8()), P(self.err), self.copy_stream.cuda_stream, route, self.slice_rows)

    def _gpu_cabac_code(self, g: int, t0: int, n: int, qps_d: torch.Tensor, err_to: torch.Tensor | None = None):
        """Arithmetic-code the n frame steps t0 .. t0 + n - 1 of a group (n * B slices) on
        the entropy stream, after their binarisation; sizes go to pinned host memory (and,
        for a batch's last group, its error flags to ``err_to``)."""
        BS = self.B * self.S
        r = g & 1
        self.cab_bin_done[r].record(self.copy_stream)
        itypes = 1 if t0 == 0 else 0  # frame step 0 is the IDR picture of every slot
        P = self._ptr
        es = self.entropy_stream
        with torch.cuda.stream(es):
            es.wait_event(self.cab_bin_done[r])
            # qps_d: [F, B * S] slice QPs, lane order (step, slot, slice)
            self.hip.cabac_code(n * BS, BS, P(self.cab_pool[r]), P(self.cab_base[r]), P(self.cab_total[r]),
                                P(self.cab_hdr_bits[r]), P(self.cab_hdr_nbits[r]), qps_d[t0].data_ptr(), itypes,
                                P(self.cab_bytes[r]), P(self.cab_comp[r]), P(self.cab_comp_off[r]), P(self.err),
                                es.cuda_stream, P(self.h_cab_out[r]), self.cab_host_cap)
            self.h_cab_bytes[r][: n * BS].copy_(self.cab_bytes[r][: n * BS], non_blocking=True)
            self.h_pool_used[r].copy_(self.cab_pool_used[r:r + 1], non_blocking=True)
            if err_to is not None:
                err_to.copy_(self.err, non_blocking=True)
            self.cab_done[r].record(es)

    def _copy_out_group(self, g: int, t0: int, n: int, copied, wrap_futs, steps_pics: list[list[PicPlan]], groups):
        """Copy thread (groups in order): wait for the coder, then hand each frame step's
        slices (already in pinned host memory, 16-byte aligned) to the NAL-wrapping pool.
        ``copied[g]`` (set once the wraps are submitted) releases ring g % 2 (pool, headers,
        pinned sizes) for group g + 2; the host buffer itself is reused by group g + 2's
        coder only after these wraps finished (the main thread waits for them)."""
        B = self.B * self.S  # lanes (slices) per step
        r = g & 1
        t_0 = time.perf_counter()
        self.cab_done[r].synchronize()
        t_1 = time.perf_counter()
        sizes = self.h_cab_bytes[r][: n * B].numpy().astype(np.int64)
        used = int(self.h_pool_used[r][0])
        self.stats["cabac_pool_peak"] = max(self.stats.get("cabac_pool_peak", 0.0), used / self.cab_pool_cap)
        self.stats["cabac_syms_per_mb_peak"] = max(self.stats.get("cabac_syms_per_mb_peak", 0.0),
                                                   used / (n * B * self.nmb))
        if (sizes < 0).any():
            err = int(self.err.item())
            for f in range(t0, t0 + n):  # nothing of this group will be wrapped
                wrap_futs[f] = self.pool.submit(lambda: [(b"", 0)] * self.B)
            copied[g].set()
            if err & 4:
                raise CabacPoolExhausted("GPU CABAC: symbol pool exhausted (raise MIVC_CABAC_SYMS_PER_MB / "
                                         "MIVC_CABAC_PEAK_SYMS_PER_MB or lower cabac_group)")
            raise RuntimeError("GPU CABAC: arithmetic coder error")
        r16 = (sizes + 15) & ~15
        total = int(r16.sum())
        buf = self.h_cab_out[r]
        if total > self.cab_host_cap:
            # the group did not fit the pinned buffer: the compaction left it on the device
            buf = torch.empty((total,), dtype=torch.uint8).pin_memory()
            with torch.cuda.device(self.dev), torch.cuda.stream(self.entropy_stream):
                buf.copy_(self.cab_comp[r][:total], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.entropy_stream)
            ev.synchronize()
            self.stats["cabac_host_spills"] = self.stats.get("cabac_host_spills", 0) + 1
        t_2 = time.perf_counter()
        self.timings["entropy_wait_gpu_s"] = self.timings.get("entropy_wait_gpu_s", 0.0) + (t_1 - t_0)
        self.timings["d2h_s"] = self.timings.get("d2h_s", 0.0) + (t_2 - t_1)
        off = 0
        for jj in range(n):
            sz = sizes[jj * B:(jj + 1) * B]
            nb = int(r16[jj * B:(jj + 1) * B].sum())
            wrap_futs[t0 + jj] = self.pool.submit(self._wrap, buf[off:off + nb], nb, sz.tolist(), steps_pics[t0 + jj], 16)
            off += nb
        copied[g].set()

    def _header_bits(self, k: int, t: int, pics: list[PicPlan], qps_t, idr_ids: list[int]):
        """Slice headers of this step -> pinned host words -> device (current stream)."""
        self._header_bits_into(self.h_hdr_bits[k], self.h_hdr_nbits[k], self.cav_hdr_bits[k], self.cav_hdr_nbits[k],
                               pics, t, qps_t, idr_ids)

    def _header_bits_into(self, hb, hn, db, dn, pics: list[PicPlan], t: int, qps_t, idr_ids: list[int]):
        """Slice headers of one step, lane order (slot, slice) -- rows of ``hb`` / ``hn``."""
        hbn, hnn = hb.numpy(), hn.numpy()
        cache = {}
        wp = self._wp
        S, first = self.S, self.slice_rows * self.wmb
        for b in range(self.B):
            pic = pics[b]
            for si in range(S):
                # slots sharing a plan share its PicPlan objects: the header differs only by QP,
                # the IDR id, the explicit weights and the slice's first MB
                key = (id(pic), int(qps_t[b]), idr_ids[b] & 0xFFFF if pic.kind == "I" else -1,
                       tuple(wp[t, b]) if (wp is not None and pic.kind == "P") else None, si)
                if key not in cache:
                    fp = self._frame_params(b, pic, t, int(qps_t[b]), idr_ids)
                    if si:
                        fp["first_mb"] = si * first
                    cache[key] = self.host.slice_header_bits(self.cfg, fp)
                words, nbits = cache[key]
                ln = b * S + si
                hbn[ln, :] = 0
                hbn[ln, : len(words)] = np.array(words, dtype=np.uint32).view(np.int32)
                hnn[ln] = nbits
        db.copy_(hb, non_blocking=True)
        dn.copy_(hn, non_blocking=True)

    def _gpu_cavlc(self, k: int, t: int, pics: list[PicPlan], qps_t, idr_ids: list[int]):
        """Launch the CAVLC kernels for the current frame step on the compute stream.
        qps_t: per-slot slice QP of this frame step (sequence of B ints)."""
        if any(pic.kind == "B" for pic in pics):
            raise ValueError("the GPU CAVLC path codes I / P slices only")
        idr = pics[0].kind == "I"
        self._header_bits(k, t, pics, qps_t, idr_ids)
        P = self._ptr
        self.hip.cavlc(self.B, self.wmb, self.hmb, P(self.hdr[k]), P(self.coef[k]), P(self.cav_mbs), P(self.cav_len),
                       P(self.cav_off), P(self.cav_trail), P(self.cav_total), P(self.cav_sizes[k]),
                       P(self.cav_words), self.cap_words, P(self.cav_hdr_bits[k]), P(self.cav_hdr_nbits[k]),
                       0 if idr else 1, int(qps_t[0]), P(self.qp), P(self.cav_out[k]), P(self.cav_out_off),
                       self._stream(), P(self.nz))

    def _copy_out(self, t: int, k: int, pics: list[PicPlan], copied, wrap_futs):
        """Copy thread (frames in order): sizes -> compressed bytes D2H, then hand the NAL
        wrapping to the pool.  ``copied[t]`` releases the device buffers of slot k for frame
        t + 2 as soon as the bytes are on the host; the wrapping is off that critical path."""
        t0 = time.perf_counter()
        self.copy_done[k].synchronize()
        t1 = time.perf_counter()
        sizes = self.h_sizes[k].numpy().astype(np.int64).tolist()
        total = int(sum(sizes))
        h = t % 3
        if t >= 3:
            wrap_futs[t - 3].result()  # host buffer h is free again
        buf = self.h_out[h]
        if buf is None or buf.numel() < total:
            buf = self.h_out[h] = torch.empty((max(total, 1 << 26),), dtype=torch.uint8).pin_memory()
        with torch.cuda.device(self.dev), torch.cuda.stream(self.copy_stream):
            buf[:total].copy_(self.cav_out[k][:total], non_blocking=True)
            self.out_done[k].record(self.copy_stream)
        self.out_done[k].synchronize()
        copied[t].set()
        t2 = time.perf_counter()
        self.timings["entropy_wait_gpu_s"] = self.timings.get("entropy_wait_gpu_s", 0.0) + (t1 - t0)
        self.timings["d2h_s"] = self.timings.get("d2h_s", 0.0) + (t2 - t1)
        wrap_futs[t] = self.pool.submit(self._wrap, buf, total, sizes, pics)

    def _wrap(self, buf, total: int, sizes: list[int], pics: list[PicPlan], align: int = 1) -> list[tuple[bytes, int]]:
        """Slice RBSPs of one step -> one entry per slot: its S slice NAL units back to back."""
        t0 = time.perf_counter()
        S = len(sizes) // len(pics)
        refs = [pic.nal_ref_idc for pic in pics for _ in range(S)]
        types = [5 if pic.kind == "I" else 1 for pic in pics for _ in range(S)]
        nals = self.host.nal_wrap_many(buf[:total].numpy(), sizes, refs[0], types[0], align, refs, types)
        if S > 1:
            nals = [b"".join(nals[b * S:(b + 1) * S]) for b in range(len(pics))]
        self.timings["entropy_s"] = self.timings.get("entropy_s", 0.0) + (time.perf_counter() - t0)
        return [(n, len(n) * 8) for n in nals]

    # ------------------------------------------------------------------ entropy (host)
    def _write_slices(self, k: int, t: int, pics: list[PicPlan], qps_t, idr_ids: list[int]) -> list[tuple[bytes, int]]:
        t0 = time.perf_counter()
        self.copy_done[k].synchronize()
        t1 = time.perf_counter()
        hdr = self.h_hdr[k].numpy()
        coef = self.h_coef[k].numpy()

        S, rows = self.S, self.slice_rows

        def one(b: int):
            fp = self._frame_params(b, pics[b], t, int(qps_t[b]), idr_ids)
            if S == 1:
                nal, st = self.host.write_slice(self.cfg, fp, hdr[b], coef[b])
                return nal, st["bits"]
            nals, bits = [], 0
            for si in range(S):
                r0 = si * rows
                n = min(rows, self.hmb - r0) * self.wmb
                nal, st = self.host.write_slice(self.cfg, dict(fp, first_mb=r0 * self.wmb, num_mbs=n), hdr[b], coef[b])
                nals.append(nal)
                bits += st["bits"]
            return b"".join(nals), bits

        out = list(self.pool.map(one, range(self.B)))
        t2 = time.perf_counter()
        self.timings["entropy_wait_gpu_s"] = self.timings.get("entropy_wait_gpu_s", 0.0) + (t1 - t0)
        self.timings["entropy_s"] = self.timings.get("entropy_s", 0.0) + (t2 - t1)
        return out

    # ------------------------------------------------------------------ rate control
    def _analyse(self, y: torch.Tensor) -> None:
        """GPU lookahead of a batch: frame costs, scene cuts, MB-tree offsets and (b-adapt) the
        multi-distance P / B costs (rc/lookahead.py, csrc/kernels/lookahead.hip)."""
        from ..rc.lookahead import GpuLookahead

        if getattr(self, "_la", None) is None:
            self._la = GpuLookahead(self.dev, self.p.la_range, weighted=self.p.la_weights)
        t0 = time.perf_counter()
        self._apply_analysis(self._analysis(y, self._la))
        self.timings["lookahead_s"] = self.timings.get("lookahead_s", 0.0) + time.perf_counter() - t0

    def _analysis(self, y: torch.Tensor, la) -> dict:
        """The lookahead of one batch on the current stream (host results synchronised, device
        results -- MB-tree offsets, lowres vectors -- left on the device)."""
        from ..rc.lookahead import GpuLookahead
        from ..rc.ratecontrol import MBTREE_STRENGTH, scenecut_flags

        lbw, lbh = GpuLookahead.block_grid(y.shape[3], y.shape[2])
        # MB-tree needs the lookahead's block grid to be the coded MB grid (no -s resize)
        use_mbtree = self.p.mbtree and lbw * lbh == self.nmb
        badapt = bool(self.p.b_adapt) and self.nb > 0 and y.shape[1] >= 3
        multi = multi_intra = mbtree = None
        if use_mbtree:
            costs_d, mbtree = la.mbtree(y, MBTREE_STRENGTH)
            blk, mv = la.last_blk, la.last_mv
        elif badapt:
            costs_d, blk, mv = la.frame_costs(y, block_costs=True, block_mvs=True)
        else:
            costs_d, blk, mv = la.frame_costs(y), None, None
        if badapt:
            multi = la.multi_costs(y, blk, mv, min(7, self.nb + 1), search_range=int(self.p.badapt_range)).cpu().numpy()
            multi_intra = la.last_multi_intra.cpu().numpy()
        costs = costs_d.cpu().numpy()
        return dict(costs=costs, multi=multi, multi_intra=multi_intra, mbtree=mbtree, use_mbtree=use_mbtree, blocks=lbw * lbh,
                    # lowres vectors on the MB grid: the search seeds (lowres_seed)
                    mv=mv if (mv is not None and self.p.lowres_seed and lbw * lbh == self.nmb) else None,
                    scenecuts=scenecut_flags(costs, float(self.p.scenecut)), shape=tuple(y.shape))

    def _apply_analysis(self, a: dict) -> None:
        self._la_costs, self._la_multi, self._mbtree = a["costs"], a["multi"], a["mbtree"]
        self._la_multi_intra = a.get("multi_intra")
        self._la_mv, self._la_blocks, self._use_mbtree = a["mv"], a["blocks"], a["use_mbtree"]
        self._scenecuts = a["scenecuts"]
        self.stats["scenecuts"] = int(self._scenecuts.sum())

    def analyse_async(self, y: torch.Tensor, after: torch.cuda.Event | None = None,
                      stream: torch.cuda.Stream | None = None):
        """Start the lookahead of a *later* batch while the current one encodes: it runs on its
        own stream (after ``after``, e.g. the event that ends the batch's synthesis / decode)
        and host thread, with its own lookahead workspace, and the returned future's state
        goes to :meth:`encode` (``analysis=``).  Its kernels fill the encode's idle gaps
        instead of sitting on the critical path between two batches.  ``stream``: run on the
        caller's stream instead (e.g. the one that produced ``y``: one hardware queue fewer)."""
        from ..rc.lookahead import GpuLookahead
        if getattr(self, "_la_async", None) is None:
            self._la_async = GpuLookahead(self.dev, self.p.la_range, weighted=self.p.la_weights)
            self._la_stream = torch.cuda.Stream(device=self.dev)
            self._la_pool = cf.ThreadPoolExecutor(max_workers=1)

        def job():
            t0 = time.perf_counter()
            st = stream if stream is not None else self._la_stream
            with torch.cuda.device(self.dev), torch.cuda.stream(st):
                if after is not None:
                    st.wait_event(after)
                a = self._analysis(y, self._la_async)
                a["event"] = torch.cuda.Event()
                a["event"].record(st)
            a["seconds"] = time.perf_counter() - t0
            return a
        return self._la_pool.submit(job)

    def _crf_from_plans(self, plans: list[list[PicPlan]]) -> np.ndarray:
        """[B, F] CRF QPs of the anchors (x264's curve over the anchors' complexity at their real
        reference distance, rc/ratecontrol.crf_qps_anchors); B entries are set by the caller."""
        from ..rc.badapt import anchor_complexity
        from ..rc.ratecontrol import crf_qps_anchors
        costs, multi = self._la_costs, self._la_multi
        B, F = costs.shape[0], costs.shape[1]
        cplx = np.empty((B, F))
        for b in range(B):
            types = [""] * F
            for pic in plans[b]:
                types[pic.d] = pic.kind
            cplx[b] = anchor_complexity("".join(types), costs[b], multi[b] if multi is not None else None)
        keys = np.zeros((B, F), dtype=bool)
        keys[:, 0] = True
        keys |= self._scenecuts
        q = crf_qps_anchors(cplx, costs[:, :, 0], float(self.p.crf), self._la_blocks, keys,
                            mbtree=self._use_mbtree, bframes=self.nb)
        self.stats["mean_qp"] = float(q.mean())
        return q

    def crf_qps(self, y: torch.Tensor) -> np.ndarray:
        """[B, F] CRF QPs of a batch (anchors; B pictures at their references' QP + pbratio):
        GPU lookahead frame costs -> per-slot GOP plans -> x264-style CRF curve."""
        from ..rc.ratecontrol import b_qps_from_refs
        self._analyse(y)
        plans = self._plans(y.shape[1], self._scenecuts, ())
        q = self._crf_from_plans(plans)
        return b_qps_from_refs(q, plans, float(self.p.b_qp_offset)) if self.nb else q

    # ------------------------------------------------------------------ public API
    @torch.no_grad()
    def encode(self, y: torch.Tensor, u: torch.Tensor, v: torch.Tensor, idr_base: int = 0,
               keep_recon: bool = False, metrics: bool = True, idr_ids: list[int] | None = None,
               qps=None, anchors_at=(), qp_delta=None, analysis=None) -> list[SegmentResult]:
        """See :meth:`_encode`.  A batch whose CABAC symbols overflow the pool (QPs far below
        the budgeted ones) is encoded again with a pool grown 4x (encoding is a pure
        function of the inputs, so the retry gives the same bytes a big pool would)."""
        if isinstance(analysis, cf.Future):
            analysis = analysis.result()
        self.drain()
        for attempt in range(3):
            try:
                return self._encode(y, u, v, idr_base, keep_recon, metrics, idr_ids, qps, anchors_at, qp_delta,
                                    analysis)
            except CabacPoolExhausted:
                if attempt == 2 or not (self.entropy == "gpu" and self.p.cabac):
                    raise
                torch.cuda.synchronize(self.dev)
                self._alloc_cabac(self.cab_G, grow=self.cab_grow * 4)
                self.stats["cabac_pool_regrow"] = self.stats.get("cabac_pool_regrow", 0) + 1
        raise AssertionError("unreachable")

    def encode_async(self, y: torch.Tensor, u: torch.Tensor, v: torch.Tensor, **kw) -> "PendingEncode":
        """Issue a batch and return before its last arithmetic-coder groups, NAL wrapping and
        result assembly finish (GPU CABAC; other entropy paths complete here).  The batch's
        tail then overlaps the next batch's first steps -- one 256 x 60 1080p batch spends
        ~100 ms in that tail with the compute stream idle.  At most two batches are in
        flight: issuing a third completes the oldest.  ``PendingEncode.result()`` gives what
        :meth:`encode` would have returned (a symbol-pool overflow re-encodes the batch
        synchronously with a grown pool).  ``kw``: :meth:`encode`'s keyword arguments."""
        ana = kw.pop("analysis", None)
        if isinstance(ana, cf.Future):
            ana = ana.result()
        while len(self._inflight) >= 2:
            self._inflight[0].result()
        if not (self.entropy == "gpu" and self.p.cabac):
            return PendingEncode(self, None, (y, u, v), dict(kw, analysis=ana), self.encode(y, u, v, analysis=ana, **kw))
        args = dict(kw)
        fin = self._encode(y, u, v, args.get("idr_base", 0), args.get("keep_recon", False), args.get("metrics", True),
                           args.get("idr_ids"), args.get("qps"), args.get("anchors_at", ()), args.get("qp_delta"),
                           ana, defer=True)
        pend = PendingEncode(self, fin, (y, u, v), dict(kw, analysis=ana))
        self._inflight.append(pend)
        return pend

    def drain(self) -> None:
        """Complete every batch issued by :meth:`encode_async` (their results stay available)."""
        while self._inflight:
            self._inflight[0].result()

    def _encode(self, y: torch.Tensor, u: torch.Tensor, v: torch.Tensor, idr_base: int = 0,
                keep_recon: bool = False, metrics: bool = True, idr_ids: list[int] | None = None,
                qps=None, anchors_at=(), qp_delta=None, analysis=None, defer: bool = False):
        """Encode B segments of F frames each.

        y: [B, F, h, w] uint8 (device), u/v: [B, F, h/2, w/2].  Each slot's output is a
        self-contained Annex-B segment (SPS/PPS + IDR + P/B ...), i.e. one "piece" of the
        reference's split directory, with idr_pic_id = idr_ids[slot] (default idr_base + slot).
        Every slot follows its own GOP plan (its scene cuts become anchors of that slot only).
        When (h, w) differs from the configured size the frames are resampled first (bicubic,
        ``-s WxH``, :mod:`govideocompressor_amd.ops.scale`).
        ``qps``: optional [B, F] per-frame QPs from the rate control (default: the params' CRF/QP,
        I frames 3 lower).  ``qp_delta``: optional [B, F] float offsets (display order) added
        to the final frame QPs -- after the lookahead CRF curve and the B-picture offset --
        with ordered dithering, so fractional offsets move the bitrate smoothly
        (:mod:`govideocompressor_amd.rc.abr`: -b:v, -pass 2, VBV).
        ``analysis``: this batch's lookahead state from :meth:`analyse_async` (computed while
        the previous batch encoded); None = run the lookahead here.
        ``defer`` (GPU CABAC): return a callable that completes the batch (waits for its coder
        and NAL wrapping, checks errors, builds the results) instead of the results, so the
        next batch can be issued while this one's last arithmetic-coder groups still run.
        """
        B, F = y.shape[0], y.shape[1]
        if B != self.B:
            raise ValueError(f"encoder was built for {self.B} slots, got {B}")
        if y.dtype != torch.uint8 or y.device != self.dev or y.dim() != 4:
            raise ValueError("y must be a uint8 [B, F, h, w] tensor on the encoder's device")
        h, w = y.shape[2], y.shape[3]
        if h % 2 or w % 2 or tuple(u.shape) != (B, F, h // 2, w // 2) or tuple(v.shape) != tuple(u.shape):
            raise ValueError("u/v must be [B, F, h/2, w/2] with even h, w")
        if not (y.is_contiguous() and u.is_contiguous() and v.is_contiguous()):
            raise ValueError("planes must be contiguous")
        if F > 0xFFFF:
            raise ValueError("at most 65535 frames per segment (frame_num / POC without wrap)")
        self._full_recon = bool(metrics or keep_recon or self.p.full_recon)
        if (w, h) != (self.p.width, self.p.height):  # -s WxH: bicubic resample (ops/scale.py)
            if getattr(self, "_scaler", None) is None:
                from ..ops.scale import GpuScaler
                self._scaler = GpuScaler(self.dev)
            y, u, v = self._scaler.clip(y, u, v, self.p.width, self.p.height)
        idr_ids = list(idr_ids) if idr_ids is not None else [idr_base + b for b in range(B)]
        if len(idr_ids) != B:
            raise ValueError("idr_ids needs one entry per slot")
        torch.cuda.set_device(self.dev)
        qp_i, qp_p = self.p.frame_qps()
        self._scenecuts = None
        self._mbtree = None
        self._la_multi = self._la_multi_intra = None
        self._la_mv = None
        self._from_la = False
        if qps is None and self.p.crf is not None and self.p.lookahead:
            if analysis is not None and analysis["shape"] == tuple(y.shape):
                torch.cuda.current_stream(self.dev).wait_event(analysis["event"])
                self._apply_analysis(analysis)
                self.timings["lookahead_async_s"] = self.timings.get("lookahead_async_s", 0.0) + analysis["seconds"]
            else:
                self._analyse(y)
            self._from_la = True
        cuts_h = self._scenecuts if self._scenecuts is not None else np.zeros((B, F), dtype=bool)
        # a scene cut becomes an anchor of its slot, so the pictures after it predict from the
        # new scene instead of across the cut (x264 places an I / P picture there); with b-adapt
        # the lookahead's costs place each slot's B pictures
        plans = self._plans(F, cuts_h, anchors_at)
        if self._from_la:
            qps = self._crf_from_plans(plans)
        self.last_plans = plans
        orders = np.array([[pic.d for pic in plans[b]] for b in range(B)], dtype=np.int64)  # [B, F] display per step
        steps_pics = [[plans[b][t] for b in range(B)] for t in range(F)]
        orders_d = torch.from_numpy(np.ascontiguousarray(orders.T.astype(np.int32))).to(self.dev)  # [F, B]
        steps = self._step_tables(plans, F)
        self._weights(y, u, v, plans)
        if qps is None:
            qps_h = np.full((B, F), qp_p, dtype=np.int32)
            qps_h[:, 0] = qp_i
        else:
            qps_h = np.clip(np.asarray(qps, dtype=np.int32).reshape(B, F), 0, 51)
        if self.nb and (qps is None or self._from_la):
            # B pictures: no rate control of their own, the distance-weighted QP of their
            # references + pbratio (x264 / x265 CRF and constant-QP rule)
            from ..rc.ratecontrol import b_qps_from_refs
            qps_h = b_qps_from_refs(qps_h, plans, float(self.p.b_qp_offset))
        if qp_delta is not None:
            from ..rc.abr import apply_delta
            qps_h = apply_delta(qps_h, qp_delta)
        self.last_qps = qps_h.copy()
        # per coding step (rows), [F, B]: the kernels and the entropy stages index coding steps
        qps_c = np.take_along_axis(qps_h, orders, axis=1)
        qps_d = torch.from_numpy(np.ascontiguousarray(qps_c.T)).to(self.dev)
        # the arithmetic coder's per-lane slice QPs (lanes: slot-major slices of each step)
        qps_ls_d = qps_d.repeat_interleave(self.S, dim=1).contiguous() if self.S > 1 else qps_d
        cuts_c = np.take_along_axis(cuts_h, orders, axis=1)
        cuts_d = torch.from_numpy(np.ascontiguousarray(cuts_c.T)).to(self.dev)  # [F, B] coding order
        if self._wp_steps is not None:
            for t, st in enumerate(steps):
                if self._wp_steps[t] is not None:
                    st["wp"], st["wp_src"] = self._wp_steps[t]
        bno = self._batch_no
        self._batch_no += 1
        self.err = self.err_bufs[bno & 1]
        self.err.zero_()
        sse = torch.zeros((F, B, 3), dtype=torch.int64, device=self.dev)   # coding order
        ssim = torch.zeros((F, B), dtype=torch.float32, device=self.dev)
        pending: list[cf.Future] = [None, None]  # type: ignore[list-item]
        outs: list[list[tuple[bytes, int]]] = [None] * F  # type: ignore[list-item]
        import threading
        copied = [threading.Event() for _ in range(F)]
        copy_futs: list = [None] * F
        wrap_futs: list = [None] * F

        def wait_copied(i: int):
            while not copied[i].wait(0.5):
                if copy_futs[i].done() and copy_futs[i].exception() is not None:
                    raise copy_futs[i].exception()
        cabac_gpu = self.entropy == "gpu" and self.p.cabac
        groups = self._cabac_groups(F, self.cab_G) if cabac_gpu else [(t, 1) for t in range(F)]
        step_group = {}
        for gi, (a0, an) in enumerate(groups):
            for jj in range(an):
                step_group[a0 + jj] = (gi, jj)
        ngroups = len(groups)
        group_copied = [threading.Event() for _ in range(ngroups)]
        group_futs: list = [None] * ngroups

        def wait_group(i: int):
            while not group_copied[i].wait(0.5):
                if group_futs[i].done() and group_futs[i].exception() is not None:
                    raise group_futs[i].exception()
        recons = None
        if keep_recon:
            recons = [tuple(torch.empty_like(p[:, 0]) for p in self.rec_pool) for _ in range(F)]
        main = torch.cuda.current_stream(self.dev)
        for t in range(F):  # t: coding step
            k = t & 1
            pics = steps_pics[t]
            st = steps[t]
            qpt = qps_c[:, t]
            # the device/pinned buffers of slot k were last used by step t-2: wait for them
            tw = time.perf_counter()
            if cabac_gpu:
                gi, jj = step_group[t]
                if jj == 0 and gi >= 2:
                    wait_group(gi - 2)  # ring gi % 2 is free again
                elif jj == 0 and self._ring_last[gi & 1] is not None:
                    # the ring's last group of the previous batch (encode_async)
                    ev, fut, _ = self._ring_last[gi & 1]
                    while not ev.wait(0.5):
                        if fut.done() and fut.exception() is not None:
                            break
            elif self.entropy == "gpu" and t >= 2:
                wait_copied(t - 2)
            elif pending[k] is not None:
                outs[t - 2] = pending[k].result()
                pending[k] = None
            self.timings["host_blocked_s"] = self.timings.get("host_blocked_s", 0.0) + time.perf_counter() - tw
            # (steps 0 / 1: the previous batch's last steps, when it is still in flight)
            main.wait_event(self.copy_done[k])
            self._prep_step(y, u, v, orders[:, t], orders_d[t])
            st["disp_d"] = orders_d[t]
            self.qp.copy_(qps_d[t])
            self._encode_step(st, self.hdr[k], self.coef[k], cuts_d[t] if (t > 0 and cuts_c[:, t].any()) else None)
            if metrics:
                P = self._ptr
                self.hip.sse(B, self.W, self.H, self.p.width, self.p.height, P(self.src[0]), P(self.src[1]),
                             P(self.src[2]), P(self.rec_pool[0]), P(self.rec_pool[1]), P(self.rec_pool[2]),
                             sse[t].data_ptr(), ssim[t].data_ptr(), self._stream(), st["route"], self.nbuf)
            if keep_recon:
                bufs = torch.tensor([pic.buf for pic in pics], dtype=torch.long, device=self.dev)
                slots = torch.arange(B, device=self.dev)
                for d in sorted({pic.d for pic in pics}):
                    sel = torch.tensor([b for b in range(B) if pics[b].d == d], dtype=torch.long, device=self.dev)
                    for c in range(3):
                        recons[d][c][sel] = self.rec_pool[c][slots[sel], bufs[sel]]
            if self.entropy == "gpu" and not self.p.cabac:
                self._gpu_cavlc(k, t, pics, qpt, idr_ids)
            self.compute_done[k].record(main)
            with torch.cuda.stream(self.copy_stream):
                self.copy_stream.wait_event(self.compute_done[k])
                if cabac_gpu:
                    self._gpu_cabac_bin(k, gi, jj, t, pics, qpt, idr_ids, qps_d[t], st["route"])
                elif self.entropy == "gpu":
                    self.h_sizes[k].copy_(self.cav_sizes[k], non_blocking=True)
                else:
                    self.h_hdr[k].copy_(self.hdr[k], non_blocking=True)
                    self.h_coef[k].copy_(self.coef[k], non_blocking=True)
                self.copy_done[k].record(self.copy_stream)
            if cabac_gpu:
                if jj == groups[gi][1] - 1:
                    t0 = groups[gi][0]
                    tw = time.perf_counter()
                    if gi >= 2:
                        # this group's compaction overwrites host buffer gi % 2: group gi - 2's
                        # wraps must be done reading it (copied[gi - 2] was waited for above)
                        a0, an = groups[gi - 2]
                        for tt in range(a0, a0 + an):
                            wrap_futs[tt].result()
                    elif self._ring_last[gi & 1] is not None:
                        for f in self._ring_last[gi & 1][2]:
                            try:
                                f.result()
                            except Exception:  # noqa: BLE001  (reported by that batch's finish)
                                pass
                        self._ring_last[gi & 1] = None
                    self.timings["host_blocked_s"] += time.perf_counter() - tw
                    self._gpu_cabac_code(gi, t0, t - t0 + 1, qps_ls_d,
                                         err_to=self.h_err[bno & 1] if gi == ngroups - 1 else None)
                    group_futs[gi] = self.copy_pool.submit(self._copy_out_group, gi, t0, t - t0 + 1, group_copied,
                                                           wrap_futs, steps_pics, groups)
            elif self.entropy == "gpu":
                copy_futs[t] = self.copy_pool.submit(self._copy_out, t, k, pics, copied, wrap_futs)
            else:
                pending[k] = self.pool.submit(self._write_slices, k, t, pics, qpt, idr_ids)
        # ---- end of the batch's issue: snapshot its counters (async) so the next batch can
        # reuse the accumulators, and note which groups last used the two CABAC rings
        B_ = B
        counters = torch.stack([self.p_intra_mbs, self.far_ref_mbs, self.sfix_mbs, self.sconv_mbs]).to(torch.int64)
        self.p_intra_mbs.zero_()
        self.far_ref_mbs.zero_()
        self.sfix_mbs.zero_()
        self.sconv_mbs.zero_()
        h_counters = torch.empty((4,), dtype=torch.int64).pin_memory()
        h_counters.copy_(counters, non_blocking=True)
        h_sse = h_ssim = None
        if metrics:
            h_sse = torch.empty(sse.shape, dtype=sse.dtype).pin_memory()
            h_ssim = torch.empty(ssim.shape, dtype=ssim.dtype).pin_memory()
            h_sse.copy_(sse, non_blocking=True)
            h_ssim.copy_(ssim, non_blocking=True)
        batch_done = torch.cuda.Event()
        batch_done.record(main)
        if cabac_gpu:
            for gi in range(max(0, ngroups - 2), ngroups):
                a0, an = groups[gi]
                self._ring_last[gi & 1] = (group_copied[gi], group_futs[gi], wrap_futs[a0:a0 + an])
        # tensors the in-flight kernels and copy threads still read (freed only after finish)
        keep = (y, u, v, steps, qps_d, qps_ls_d, orders_d, cuts_d, self._route_dev, self._wp_steps, self._la_mv,
                self._mbtree, sse, ssim, counters, analysis)
        err_h = self.h_err[bno & 1]

        def finish() -> list[SegmentResult]:
            if cabac_gpu:
                for f in group_futs:
                    f.result()
                for t in range(F):
                    outs[t] = wrap_futs[t].result()
            elif self.entropy == "gpu":
                for t in range(F):
                    copy_futs[t].result()
                for t in range(F):
                    outs[t] = wrap_futs[t].result()
            for t in range(max(0, F - 2), F):
                k = t & 1
                if pending[k] is not None:
                    outs[t] = pending[k].result()
                    pending[k] = None
            batch_done.synchronize()
            nonlocal keep
            keep = None  # released only now: the batch's kernels have finished
            c = h_counters.numpy()
            if F > 1:
                self.stats["p_intra_ratio"] = float(c[0]) / (B_ * (F - 1) * self.nmb)
                n_p = sum(1 for plan in plans for pic in plan if pic.kind == "P")
                if self.nref > 1 and n_p:
                    # share of P-picture MBs (inter decisions before the intra override) on a farther picture
                    self.stats["p_far_ref_ratio"] = float(c[1]) / (n_p * self.nmb)
                nbp = sum(1 for plan in plans for pic in plan if pic.kind == "B")
                self.stats["b_ratio"] = nbp / float(B_ * F)
                if nbp and self.p.direct == "spatial":
                    # fast spatial direct: share of B-picture MBs whose direct motion the exact
                    # decoding-order pass changed after they were priced on the estimate / made explicit
                    self.stats["spatial_fix_ratio"] = float(c[2]) / (nbp * self.nmb)
                    self.stats["spatial_conv_ratio"] = float(c[3]) / (nbp * self.nmb)
            # the batch's error flags: with the GPU coder from its last group (copied behind the
            # coder on the entropy stream), else from the device after the batch's own work
            err = int(err_h[0]) if cabac_gpu else int(self.err_bufs[bno & 1].cpu()[0])
            if err & 4:
                raise CabacPoolExhausted(f"GPU CABAC: symbol pool exhausted (err={err:#x})")
            if err & 14:
                raise RuntimeError(f"GPU CABAC failed (err={err:#x}: 4 = symbol pool exhausted, 8 = coder error)")
            if err != 0:
                raise RuntimeError("wavefront progress timeout in an encode kernel")
            ps = self.parameter_sets()
            results = []
            npx = self.p.width * self.p.height
            nwin = (self.p.width // 8) * (self.p.height // 8)
            sse_h = h_sse.numpy().astype(np.float64) if metrics else None
            ssim_h = h_ssim.numpy() if metrics else None
            for b in range(B_):
                nals = [outs[t][b][0] for t in range(F)]
                r = SegmentResult(frames=F, nals=nals, bits=[outs[t][b][1] for t in range(F)], header=ps,
                                  order=orders[b].tolist())
                if metrics:
                    def psnr(ssev, n):
                        mse = ssev / n
                        return 100.0 if mse <= 1e-10 else 10.0 * math.log10(255.0 ** 2 / mse)
                    r.psnr_y = float(np.mean([psnr(sse_h[t, b, 0], npx) for t in range(F)]))
                    r.psnr_u = float(np.mean([psnr(sse_h[t, b, 1], npx / 4) for t in range(F)]))
                    r.psnr_v = float(np.mean([psnr(sse_h[t, b, 2], npx / 4) for t in range(F)]))
                    r.ssim_y = float(ssim_h[:, b].sum() / (F * max(1, nwin)))
                results.append(r)
            if keep_recon:
                self.last_recon = recons
            return results

        if defer and cabac_gpu:
            return finish
        return finish()

    def close(self):
        self.pool.shutdown(wait=True)
        if hasattr(self, "copy_pool"):
            self.copy_pool.shutdown(wait=True)


CONTENT_KINDS = ("default", "pan-fast", "static", "fade", "zoom", "cuts", "noise")


def synth_clip(slots: int, frames: int, width: int, height: int, seed: int = 0, frame0: int = 0,
               device: str | torch.device = "cuda", bit_depth: int = 8, slot0: int = 0, kind: int | str = 0):
    """Generate B x F synthetic I420 frames directly in HBM (see csrc/kernels/synth.hip).

    Slot ``b`` shows the content of global slot ``slot0 + b`` (a rank encoding slots
    [r * B, (r + 1) * B) of a global batch renders exactly what one process would).
    ``bit_depth=10`` renders the same content at 10-bit precision into int16 planes
    (values 0..1023: the canvas interpolation, ramp and noise keep their low bits).
    ``kind``: content class (CONTENT_KINDS: the headline content, fast pan, static background
    with small movers, fade, zoom, a cut every 30 frames, heavy noise)."""
    if bit_depth not in (8, 10):
        raise ValueError("synth_clip: bit_depth must be 8 or 10")
    if isinstance(kind, str):
        kind = CONTENT_KINDS.index(kind)
    hip = native.hip()
    dev = _resolve(device)
    dt = torch.uint8 if bit_depth == 8 else torch.int16
    y = torch.empty((slots, frames, height, width), dtype=dt, device=dev)
    u = torch.empty((slots, frames, height // 2, width // 2), dtype=dt, device=dev)
    v = torch.empty_like(u)
    hip.synth(y.data_ptr(), u.data_ptr(), v.data_ptr(), width, height, slots, frames, frame0, seed & 0xFFFFFFFF,
              torch.cuda.current_stream(dev).cuda_stream, bit_depth, slot0, int(kind))
    return y, u, v
