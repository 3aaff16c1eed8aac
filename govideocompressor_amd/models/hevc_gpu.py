"""MI355X HEVC (H.265) encoder: B closed-GOP segments encoded concurrently on one GPU.

Replaces the reference's ``-vcodec libx265 -crf 26`` worker call (server.go:67-68,
client.go:115) with gfx950 kernels, CABAC included:

per frame step t (frame t of every slot):
  prep (u8/u16 -> padded u16 planes)
  -> hevc_aq: per-CTB QP (variance AQ + MB-tree offsets, one quantization group per CTB)
  -> I: hevc_intra_analyze (CTB-parallel open-loop CU/mode decision)
        + hevc_intra_recon (CTB wavefront, closed loop)
     P: lookahead motion search + hevc_inter (CU-parallel) + intra CUs (wavefront)
  -> hevc_qp_fixup (QpY of CTBs / CUs without a coded delta, 8.6.1)
  -> hevc_deblock (vertical, then horizontal edges; picture-parallel)
  -> hevc_sao (per-CTB statistics, decision, apply)
then, on the copy stream while the compute stream runs the next step, hevc_entropy codes
the slice data of the step's pictures on the GPU (one lane per WPP substream, the coder of
csrc/common/hevc_ctu_coder.h) and packs the substreams into pinned host memory, where a
host thread adds slice headers, entry points and emulation prevention
(hevc_assemble_slices).  ``entropy="host"`` instead ships the records and the packed non-zero
level blocks to pinned memory and codes the slices on host threads (csrc/host/hevc_writer.cc,
the same coder: byte-identical output).

Main (8-bit) and Main 10 share one code path: samples are uint16 on the device.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from ..ops import native

CTB = 32


@dataclass
class HevcParams:
    width: int
    height: int
    fps: float = 30.0
    crf: float | None = 26.0
    qp: int = 30                    # used when crf is None
    ip_offset: int = 3
    bit_depth: int = 8
    sao: bool = True
    deblock: bool = True
    intra_only: bool = False
    keyint: int = 0                 # IDR period inside a segment (0: the first picture only)
    max_merge: int = 3              # x265 --max-merge 3 (1080p sweep: 3 / 4 / 5 = 3023 / 3039 / 3042 kb/s)
    me_range: int = 8
    subpel: int = 2
    # CRF per-frame QPs from the GPU lookahead (rc/lookahead.py); False = flat CRF QP
    lookahead: bool = True
    la_range: int = 6
    # lowres weighted prediction in the lookahead (rc/lookahead.py GpuLookahead(weighted=True)):
    # P candidates of fades / flashes priced with the weights the encoder's weightp will use
    la_weights: bool = True
    scenecut: int = 40   # x264/x265 --scenecut: cut frames are coded all-intra at the I QP (0: off)
    # x265 --wpp (its default): one CABAC substream per CTB row; the host codes the rows of
    # one picture on several threads when fewer pictures than entropy threads are in flight
    wpp: bool = True
    # x265 --aq-mode 1 --aq-strength 1.0 --qg-size 32: variance AQ per 16x16 block, averaged
    # into one QP per CTB coded with cu_qp_delta (csrc/kernels/hevc_filters.hip hevc_aq_ctb);
    # 0 disables
    aq_strength: float = 1.0
    # x265 --cutree (default on): lookahead propagation -> per-block QP offsets added before
    # the CTB average (needs the lookahead and its block grid equal to the 16x16 grid)
    cutree: bool = True

    # merge-aware vector choice after the search (Jacobi passes over the spatial merge
    # neighbours' vectors, bframe.hip hevc_merge_refine); 0 disables
    merge_refine: int = 4  # 1080p sweep (tools/hevc_knob_sweep.py): 0 -> 2 -> 4 passes = 3584 -> 3092 -> 3042 kb/s
    # x265 --signhide: the quantiser hides one sign per 4x4 group in the parity of the group's
    # levels (sign_data_hiding_enabled_flag).  Measured on the synthetic 1080p bench content:
    # +0.25 % bits at +0.01 dB (RD-neutral) for -28 % throughput, so off by default and on
    # only at -preset veryslow / placebo
    sdh: bool = False
    # lambda multiples added to the open-loop intra cost of a 16x16 quadrant in P pictures
    # before the inter / intra decision (the closed loop makes intra dearer than its
    # open-loop SATD says)
    intra_bias_p: int = 16  # 1080p sweep 0 / 16 / 32: 2984 / 2956 / 2944 kb/s at 37.132 / 37.118 / 37.111 dB
    # x265 --tu-inter-depth: 1 = inter CUs choose between one TU and four quarter TUs by RD
    # (~0.7 % BD-rate on the synthetic bench content for ~16 % of the 1080p throughput; on from
    # -preset slow)
    tu_inter_depth: int = 0
    # general_level_idc (30 x level, -level); 0 = the lowest level the size / rate fits
    level_idc: int = 0
    # P pictures: run the open-loop intra analysis only on CTBs where intra may still win --
    # some 16x16 block whose motion cost is not below half the motion search's own Intra16x16
    # estimate (a lower bound of the finer intra search) plus the intra bias; elsewhere inter
    # is decisive and the CTB gets no intra candidates
    intra_gate: bool = True
    # x265 --bframes: B pictures between the P anchors (list 0 = the previous reference, list 1 =
    # the next; models/gop.py hevc_gop_plan), coded b_qp_offset above their anchors; 0 = P
    # pictures only.  keyint > 0 and intra_only keep P-only GOPs.  x265 places its 4 B frames
    # adaptively (--b-adapt 2) at --pbratio 1.3 (+2 QP); this encoder's GOP is static (one plan
    # per batch), so its defaults come from the 1080p CRF 22-34 sweep of the benchmark content
    # (profiles/r3_hevc_bframes_rd.md): BD-rate vs P-only -4.4 % for 1 B at +4 QP, while runs of
    # 2-4 B pictures lose there (+2.6 .. +7.9 % at +2 QP: the far anchors cost more than the B
    # pictures save on this content)
    bframes: int = 1
    # content suite (profiles/r4_hevc_bqp_rd.json, BD-rate vs +4): +2 +1.85 %, +3 +0.79 %,
    # +6 -1.36 % -- the B picture between two anchors is worth less than x265's pbratio prices it
    b_qp_offset: int = 6
    # x265 --b-adapt: B runs of up to ``bframes`` pictures placed from the lookahead's lowres
    # costs (rc/badapt.py, x264's fast algorithm on la_multi's P-at-distance and B costs) instead
    # of the fixed pattern; one pattern per batch (the summed costs of every slot, each slot's
    # scene cuts still forced anchors) -- the HEVC kernels code one picture type per step.
    # ``b_bias`` = x264/x265 --b-bias; 0 = the fixed pattern
    b_adapt: int = 0
    b_bias: int = 0
    badapt_range: int = 2
    # x265 --b-pyramid (default on): the middle B of a run of 2+ is a reference picture (at half
    # the B QP offset) and the others predict from their nearest references (models/gop.py)
    pyramid: bool = True
    # x265 --tmvp (default on): temporal merge / AMVP candidates from the collocated anchor
    tmvp: bool = True
    # merge passes offer each 16x16 block the writer's exact merge list for a 16x16 CU
    # (bframe.hip hevc_b_merge; P and B pictures); False: P pictures use the neighbour-vector
    # approximation of round 2 (hevc_merge_refine)
    merge_exact: bool = True
    # merge passes after the first re-evaluate only blocks next to a block the previous pass
    # moved (exact: the others would rebuild the same lists at the same costs); False = every
    # block every pass (A/B switch)
    merge_skip: bool = True
    # x265 --ctu 64 (its default): 64x64 coding tree units over the 32x32 record blocks (the
    # blocks are the CTU's quantization groups and are reconstructed in z-order; one SAO
    # parameter set per CTU; 64x64 skip CUs where four blocks agree) -- False: 32x32 CTBs
    ctu64: bool = True
    # x265 --weightp (its default): explicit weights of a P picture's reference where the
    # source statistics say the brightness or contrast changed (fades, flashes): weight =
    # sqrt(var_cur / var_ref) over 2^6, offset = mean_cur - weight * mean_ref, per component,
    # used when the luma mean moved >= wp_min_mean levels (8-bit scale) or the contrast >=
    # wp_min_scale.  Main 10 too: statistics of the 16-bit planes (weightp.hip wp_stats16),
    # offsets coded in 8-bit units as the standard scales them
    weightp: bool = True
    wp_min_mean: float = 2.0
    wp_min_scale: float = 0.08
    # x265 --ref: active list-0 pictures of a P picture (its nearest earlier reference pictures;
    # models/gop.py hevc_gop_plan).  The farther pictures get 16x16 searches seeded by the
    # distance-scaled list-0[0] vectors (radius ref_range), skipped where the list-0[0] cost is
    # already <= ref_gate; the P init pass picks per block at cost + lambda * ref_idx bins and
    # the merge passes carry each candidate's refIdx.  B pictures keep one picture per list.
    # Content suite (profiles/r6_hevc_refs_rd.md, BD-rate vs refs 1): refs 3 at gate 3000 -0.97 %,
    # gate 6000 -1.05 % (no class worse), ungated +1.15 %; config 4 throughput unchanged
    refs: int = 3
    ref_range: int = 4
    ref_gate: int = 6000
    # 8x8 inter CUs (x265 searches CUs down to its 8x8 minimum): after the merge passes, each
    # 16x16 block of a P picture whose motion is RefPicList0[0] searches one vector per 8x8
    # quadrant (p_part8x8, HEVC form: candidates, half / quarter rings); the four 8x8 CUs win
    # when their SATD + lambda * (mvd bits + inter8_overhead) beats the merge-aware 16x16 cost.
    # Blocks at or below inter8_min_satd are not searched.  B pictures keep 16x16 / 32x32 CUs.
    # Content suite (profiles/r6_hevc_inter8_rd.md, BD-rate vs 16x16 / 32x32 only): overhead 8
    # -0.34 %, 16 -0.28 %, 24 -0.23 %, 16 with a 1000 floor -0.37 % (no class worse); config 4
    # about -0.5 % fps
    inter8: bool = True
    inter8_overhead: int = 16
    inter8_min_satd: int = 1000

    def eff_refs(self) -> int:
        """Active list-0 pictures of P pictures (1 for intra-only and keyint GOPs)."""
        if self.intra_only or self.keyint > 0:
            return 1
        return max(1, min(4, int(self.refs)))

    def eff_weightp(self) -> bool:
        return bool(self.weightp and not self.intra_only)

    def eff_bframes(self) -> int:
        return 0 if (self.intra_only or self.keyint > 0) else max(0, int(self.bframes))

    def adaptive_qp(self) -> bool:
        return self.aq_strength > 0 or (self.cutree and self.lookahead and self.crf is not None)

    def host_cfg(self) -> dict:
        return dict(width=self.width, height=self.height, bit_depth=self.bit_depth, fps=self.fps,
                    sao=int(self.sao), deblock=int(self.deblock), max_merge=self.max_merge, wpp=int(self.wpp),
                    cu_qp_delta=int(self.adaptive_qp()), tu_inter_depth=int(self.tu_inter_depth), sdh=int(self.sdh),
                    level_idc=int(self.level_idc), bframes=self.eff_bframes(), tmvp=int(self.tmvp and not self.intra_only),
                    pyramid=int(self.pyramid), ctu64=int(self.ctu64), weightp=int(self.eff_weightp()),
                    refs=self.eff_refs())

    def frame_qps(self) -> tuple[int, int]:
        qp_p = int(round(self.crf)) if self.crf is not None else int(self.qp)
        qp_p = max(0, min(51, qp_p))
        return max(0, qp_p - self.ip_offset), qp_p


@dataclass
class HevcSegmentResult:
    bitstream: bytes
    frames: int
    nals: list[bytes] = field(default_factory=list)   # coding order
    bits: list[int] = field(default_factory=list)
    psnr_y: float = 0.0
    order: list[int] = field(default_factory=list)    # display index of each NAL

    def display_prefix(self, c: int) -> list[bytes]:
        """Slice NALs of display pictures 0..c-1 (a coding-order prefix when c - 1 is an
        anchor: encode(anchors_at=...))."""
        order = self.order or list(range(len(self.nals)))
        out = [n for n, d in zip(self.nals, order) if d < c]
        if any(d >= c for d in order[:len(out)]):
            raise ValueError(f"pictures 0..{c - 1} are not a coding-order prefix (encode with anchors_at)")
        return out


class PendingHevc:
    """A batch issued by :meth:`GpuHevcEncoder.encode_async`."""

    def __init__(self, enc, finish):
        self._enc, self._finish = enc, finish
        self._res = None
        self._exc: BaseException | None = None

    def done(self) -> bool:
        return self._finish is None

    def result(self) -> list:
        if self._finish is not None:
            try:
                self._res = self._finish()
            except BaseException as e:  # noqa: BLE001
                self._exc = e
            self._finish = None
            if self in self._enc._inflight:
                self._enc._inflight.remove(self)
        if self._exc is not None:
            raise self._exc
        return self._res


class GpuHevcEncoder:
    """Batched gfx950 HEVC encoder (Main / Main 10, CABAC)."""

    def __init__(self, params: HevcParams, slots: int, device="cuda", entropy_threads: int | None = None,
                 entropy: str | None = None):
        if params.width % 2 or params.height % 2:
            raise ValueError("width and height must be even")
        if params.bit_depth not in (8, 10):
            raise ValueError("bit_depth must be 8 or 10")
        self.p = params
        self.B = int(slots)
        d = torch.device(device)
        if d.type == "cuda" and d.index is None:
            d = torch.device("cuda", torch.cuda.current_device())
        self.dev = d
        self.hip = native.hip()
        self.host = native.host()
        self.W = -(-params.width // CTB) * CTB
        self.H = -(-params.height // CTB) * CTB
        self.wctb, self.hctb = self.W // CTB, self.H // CTB
        self.nctb = self.wctb * self.hctb
        B, H, W, dev = self.B, self.H, self.W, self.dev
        u16, i16 = torch.int16, torch.int16  # samples (<= 10 bits) are stored in int16 tensors, read as uint16

        def planes(dt=u16):
            return (torch.zeros((B, H, W), dtype=dt, device=dev), torch.zeros((B, H // 2, W // 2), dtype=dt, device=dev),
                    torch.zeros((B, H // 2, W // 2), dtype=dt, device=dev))

        self.src = planes()
        self.nb = params.eff_bframes()
        self.nrefs = params.eff_refs()
        # reconstruction buffers: one per DPB slot of a reference picture (models/gop.py
        # hevc_ref_slots: 2 for P-only GOPs, 3 with B pictures, more with x265 --ref) + one for
        # non-reference B pictures
        from .gop import hevc_ref_slots
        self.ref_slots = hevc_ref_slots(self.nb, params.pyramid, self.nrefs)
        self.rec = [planes() for _ in range(self.ref_slots)] + ([planes()] if self.nb else [])
        self.dbk = planes()                  # SAO output ping-pong buffer
        self.coefs = [planes(i16), planes(i16)]  # double-buffered: copy-out of t overlaps t + 1
        self.coef = self.coefs[0]
        self.wmb, self.hmb = W // 16, H // 16
        nmb = self.wmb * self.hmb
        self.nmb = nmb
        self.src8 = torch.zeros((B, H, W), dtype=torch.uint8, device=dev)   # motion-search proxies
        self.src8w = torch.zeros_like(self.src8) if params.eff_weightp() else None  # inverse-weighted proxy
        # 8-bit proxies of the reference pictures and their half-sample planes (per DPB slot),
        # built once per reference picture and shared by every picture that references it
        self.ref8s = [torch.zeros((B, H, W), dtype=torch.uint8, device=dev) for _ in range(self.ref_slots)]
        self.me_hps = [torch.empty(B * 3 * (H + 8) * (W + 8) + 64, dtype=torch.uint8, device=dev)
                       for _ in range(self.ref_slots)]
        self.mv = torch.zeros((B, nmb, 2), dtype=torch.int16, device=dev)
        self.prev_mv = torch.zeros((B, nmb, 2), dtype=torch.int16, device=dev)
        self.mv_tmp = torch.zeros((B, nmb, 2), dtype=torch.int16, device=dev)
        self.me_cost = torch.zeros((B, nmb), dtype=torch.int32, device=dev)
        self.me_intra = torch.zeros((B, nmb), dtype=torch.int32, device=dev)
        self.me_pred = torch.zeros((B, nmb, 256), dtype=torch.uint8, device=dev)
        i16_, i32_, u8_ = torch.int16, torch.int32, torch.uint8
        self.tmv = torch.zeros((B, nmb, 4), dtype=i16_, device=dev)
        self.tdir = torch.zeros((B, nmb), dtype=u8_, device=dev)
        self.mvb = [torch.zeros((B, nmb, 4), dtype=i16_, device=dev) for _ in range(2)]
        self.dirb = [torch.zeros((B, nmb), dtype=u8_, device=dev) for _ in range(2)]
        self.bcost = torch.zeros((B, nmb), dtype=i32_, device=dev)
        self.bbits = torch.zeros((B, nmb), dtype=i32_, device=dev)
        self.pm0 = torch.zeros((B, nmb, 2), dtype=i16_, device=dev)
        self.pm1 = torch.zeros((B, nmb, 2), dtype=i16_, device=dev)
        # motion of each reference picture (per DPB slot) per 16x16 block: its records at each
        # block's top-left granule, what TMVP reads after 16x16 motion compression
        R = self.ref_slots
        self.col_dir = torch.zeros((R, B, self.hmb, self.wmb), dtype=u8_, device=dev)
        self.col_mv0 = torch.zeros((R, B, self.hmb, self.wmb, 2), dtype=i32_, device=dev)
        self.col_mv1 = torch.zeros((R, B, self.hmb, self.wmb, 2), dtype=i32_, device=dev)
        # x265 --ref: a collocated P picture whose blocks point at different list-0 pictures keeps
        # each block's list-0 POC distance (None for the slot: every block uses RefPicList0[0])
        self.col_td0 = [None] * R
        if params.inter8 and not params.intra_only:
            self.mv8 = torch.zeros((B, nmb, 4, 2), dtype=i16_, device=dev)
        if self.nrefs > 1:
            nx = self.nrefs - 1
            self.xmv = torch.zeros((nx, B, nmb, 2), dtype=i16_, device=dev)    # farther list-0 searches
            self.xcost = torch.zeros((nx, B, nmb), dtype=i32_, device=dev)
            self.xpm = torch.zeros((nx, B, nmb, 2), dtype=i16_, device=dev)    # their seeds / predictors
            self.xpred = torch.zeros((B, nmb, 256), dtype=u8_, device=dev)     # (prediction scratch)
        if self.nb:
            self.mv1 = torch.zeros((B, nmb, 2), dtype=i16_, device=dev)
            self.me_cost1 = torch.zeros((B, nmb), dtype=i32_, device=dev)
        self.cand = torch.zeros((B, self.nctb, 58), dtype=torch.int32, device=dev)  # kCandStride
        self.ctus = [torch.zeros((B, self.nctb, 32), dtype=torch.uint8, device=dev) for _ in range(2)]
        self.cus = [torch.zeros((B, self.nctb * 16, 16), dtype=torch.uint8, device=dev) for _ in range(2)]
        self.ctu, self.cu = self.ctus[0], self.cus[0]
        # sparse level hand-off (double-buffered like the records: the copy-out of step t
        # overlaps step t + 1)
        self.pack_cap = self.nctb * 96  # 4x4 blocks per slot: every block of every CTB
        self.nzmaps = [torch.zeros((B, self.nctb, 2), dtype=torch.int64, device=dev) for _ in range(2)]
        self.nzoffs = [torch.zeros((B, self.nctb), dtype=torch.int32, device=dev) for _ in range(2)]
        self.nzcnt = torch.zeros((B, self.nctb), dtype=torch.int32, device=dev)
        self.copy_stream = torch.cuda.Stream(device=dev)
        self.copy_done = [torch.cuda.Event() for _ in range(2)]
        self.host_bufs = None  # lazily: 3 sets of pinned host buffers
        self.qp = torch.zeros((B,), dtype=torch.int32, device=dev)
        self.ctb_qp = torch.zeros((B, self.nctb), dtype=torch.int32, device=dev)  # QpY per CTB
        self.mb_aq = torch.zeros((B, nmb), dtype=torch.int8, device=dev)           # ME lambda offsets
        self._cutree = None  # [B, F, nmb] float MB-tree offsets of the batch being encoded
        self.run = torch.zeros((B,), dtype=torch.int8, device=dev)
        self.err = torch.zeros((1,), dtype=torch.int32, device=dev)
        self.params_nal = self.host.hevc_parameter_sets(params.host_cfg())
        # one Python worker hands each step's B pictures to the native batch writer, which
        # codes them on `entropy_threads` C++ threads with the GIL released
        self.entropy_threads = entropy_threads or min(16, os.cpu_count() or 4)
        # entropy "gpu": the slice data is CABAC-coded on the device (kernels/hevc_entropy.hip,
        # the host writer's coder) and only the slice headers, entry points and emulation
        # prevention stay on the host; "host": the native writer codes the records on
        # entropy_threads host threads (csrc/host/hevc_writer.cc)
        # "auto": host threads when this process has cores for them (6+ usable cores and
        # entropy threads: the writer codes a 1080p picture in ~2.5 ms per core, so 6 cores
        # keep up with the GPU's ~2,450 pictures/s), else the GPU.  One rank's share of an
        # 8-GPU node (2 cores): config 4 (256 x 1080p) 731 fps on the host, 2051 on the GPU;
        # config 5 (10 x 8K, a picture's rows spread over 8 workgroups) 27.0 on the host, 36.6
        # on the GPU.  The whole 1-GPU box: config 4 2452 on the host, 2062 on the GPU
        # (profiles/r6_hevc_gpu_entropy.md)
        self.entropy = (entropy or os.environ.get("MIVC_HEVC_ENTROPY", "auto")).lower()
        if self.entropy not in ("gpu", "host", "auto"):
            raise ValueError("entropy must be 'gpu', 'host' or 'auto'")
        if self.entropy == "auto":
            cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
            self.entropy = "gpu" if min(cores, self.entropy_threads) < 6 else "host"
        if self.entropy == "gpu":
            self._alloc_entropy()
        self.pool = cf.ThreadPoolExecutor(max_workers=1)
        self._inflight: list = []               # encode_async batches not yet finished (oldest first)
        self._pending: list[list] = [[], [], []]  # CABAC jobs per pinned host buffer set
        self.timings: dict[str, float] = {}
        self.stats: dict[str, float] = {}
        self.ctb_need = torch.ones((B, self.nctb), dtype=torch.uint8, device=dev)
        self.cu_stats = None  # {} -> the writer's CU counts per picture type are accumulated here
        # per-stage device time (HIP events, resolved once per encode): MIVC_STAGE_TIMING=1
        from ..obs.timers import EventTimer
        self.stage_timer = EventTimer(enabled=os.environ.get("MIVC_STAGE_TIMING", "0") == "1")

    def _chg_args(self, it: int) -> tuple[int, int]:
        """(chg_in, chg_out) of merge pass ``it``: the first pass evaluates every block and
        records which moved; later passes re-evaluate only blocks next to a moved one
        (bframe.hip hevc_b_merge -- the skipped blocks would reach the same decision)."""
        if not self.p.merge_skip:
            return 0, 0
        if getattr(self, "_chg", None) is None:
            self._chg = [torch.zeros((self.B, self.nmb), dtype=torch.uint8, device=self.dev) for _ in range(2)]
        return (0 if it == 0 else self._chg[(it - 1) % 2].data_ptr()), self._chg[it % 2].data_ptr()

    def _intra_gate(self) -> torch.Tensor:
        """[B, nctb] uint8: CTBs of a P picture where intra may beat the motion search (see
        ``HevcParams.intra_gate``); the decision mirrors hevc_p_decide's costs."""
        bd = self.p.bit_depth
        lam = torch.floor(0.755 * torch.exp2((self.qp.float() - 12.0) / 6.0) * float(1 << (bd - 8)) + 0.5)[:, None]
        inter = self.me_cost.float() * float(1 << (bd - 8)) + 3.0 * lam
        intra_lb = self.me_intra.float() * float(1 << (bd - 8)) * 0.5 + float(self.p.intra_bias_p) * lam
        need = (inter >= intra_lb).view(self.B, self.hctb, 2, self.wctb, 2)
        self.ctb_need.copy_(need.any(dim=4).any(dim=2).view(self.B, self.nctb))
        return self.ctb_need

    def _alloc_entropy(self) -> None:
        """Device buffers of the GPU entropy stage: per-picture coder state, one bounded region
        per substream (WPP: one per CTU row) and the collocated pictures' records per DPB slot;
        the packed substreams go to pinned host sets (:meth:`_entropy_host`)."""
        dev, B = self.dev, self.B
        W, H = self.W, self.H
        ctu_log2 = 6 if self.p.ctu64 else 5
        wctu, hctu = -(-W // (1 << ctu_log2)), -(-H // (1 << ctu_log2))
        self.ent_nsub = hctu if self.p.wpp else 1
        if self.ent_nsub > 100:
            raise ValueError("GPU entropy: at most 100 CTU rows (use entropy='host')")
        # bytes per substream: 12 KiB per CTU of a row (about 2 bytes per 4:2:0 sample of a
        # 64x64 CTU), the whole picture without WPP
        per_ctu = 12288 if self.p.ctu64 else 3072
        self.ent_cap = ((per_ctu * wctu * (1 if self.p.wpp else hctu)) + 15) // 16 * 16
        self.ent_state_bytes = int(self.hip.hevc_entropy_state_bytes(W, H))
        self.ent_state = torch.empty((B, self.ent_state_bytes), dtype=torch.uint8, device=dev)
        # one substream area per pinned host set: a step whose slice data outgrows the pinned
        # buffer is read back from its own area, which the next steps do not overwrite
        self.ent_outs = [torch.empty((B * self.ent_nsub * self.ent_cap,), dtype=torch.uint8, device=dev)
                         for _ in range(3)]
        n = B * self.ent_nsub
        self.ent_sizes = torch.zeros((n,), dtype=torch.int32, device=dev)
        self.ent_errs = torch.zeros((n,), dtype=torch.int32, device=dev)
        self.ent_offs = torch.zeros((n + 1,), dtype=torch.int64, device=dev)
        self.ent_over = torch.zeros((1,), dtype=torch.int32, device=dev)
        # narrow batches spread a picture over several workgroups (kernels/hevc_entropy.hip):
        # row progress and the row contexts after CTU 1 then go through device memory
        self.ent_gprog = torch.zeros((n,), dtype=torch.int32, device=dev)
        self.ent_gctx = torch.zeros((n * 151 * 2,), dtype=torch.uint8, device=dev)  # kNumCtx CtxStates per row
        # pinned output per host set: half a byte per luma sample of every picture of a step
        self.ent_dst_cap = max(1 << 22, B * W * H // 2)
        self.ent_host = None
        self.col_cus = None  # per DPB slot: [B, nctb * 16, 16] records of the picture in it (TMVP)

    def _entropy_prof(self, kind: str) -> int:
        """MIVC_HEVC_ENTROPY_PROF=1 (diagnostics): device pointer of a cycle-counter buffer of the
        GPU coder for this step (one per picture type, summed by :meth:`entropy_profile`), else 0."""
        if os.environ.get("MIVC_HEVC_ENTROPY_PROF", "0") != "1":
            return 0
        if getattr(self, "_ent_prof", None) is None:
            self._ent_prof = {}
        buf = torch.zeros((self.B * 16 * 9,), dtype=torch.int64, device=self.dev)
        self._ent_prof.setdefault(kind, []).append(buf)
        return buf.data_ptr()

    def entropy_profile(self) -> dict:
        """Cycles per picture type of the GPU coder's parts (MIVC_HEVC_ENTROPY_PROF=1 runs):
        residual, merge list, AMVP, CU, SAO, whole CTU, nz scan, barrier wait; CTUs coded."""
        names = ("residual", "merge", "amvp", "cu", "sao", "ctu", "scan", "wait", "ctus")
        out = {}
        for kind, bufs in (getattr(self, "_ent_prof", None) or {}).items():
            tot = torch.stack([b.view(-1, 9) for b in bufs]).sum(dim=(0, 1)).cpu().tolist()
            out[kind] = dict(zip(names, tot))
        return out

    def _entropy_host(self):
        if self.ent_host is None:
            n = self.B * self.ent_nsub

            def pinned(shape, dtype):
                return torch.empty(shape, dtype=dtype).pin_memory()
            self.ent_host = [dict(dst=pinned((self.ent_dst_cap,), torch.uint8), offs=pinned((n + 1,), torch.int64),
                                  sizes=pinned((n,), torch.int32), errs=pinned((n,), torch.int32)) for _ in range(3)]
        return self.ent_host

    def _host_buffers(self):
        if self.host_bufs is None:
            def pin(t):
                return torch.empty(t.shape, dtype=t.dtype).pin_memory()
            self.host_bufs = [[pin(self.ctus[0]), pin(self.cus[0]), pin(self.nzmaps[0]), pin(self.nzoffs[0]),
                               torch.empty((self.B, self.pack_cap * 16), dtype=torch.int16).pin_memory()]
                              for _ in range(3)]
        return self.host_bufs

    def parameter_sets(self) -> bytes:
        return self.params_nal

    def close(self):
        self.drain()
        self.pool.shutdown(wait=True)
        if getattr(self, "_la_pool", None) is not None:
            self._la_pool.shutdown(wait=True)

    # ------------------------------------------------------------------ helpers
    @staticmethod
    def _p(t: torch.Tensor) -> int:
        return t.data_ptr()

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.dev).cuda_stream

    def _prep(self, y, u, v, t: int, proxy: bool = False):
        """Frame t of every slot -> padded uint16 planes (+ the 8-bit luma proxy of the
        motion search): one fused launch for the three planes."""
        B, F, h, w = y.shape
        bps = y.element_size()
        in_bd = 8 if bps == 1 else self.p.bit_depth
        shift = self.p.bit_depth - in_bd
        ys, us, vs = y[:, t], u[:, t], v[:, t]
        if ys.stride(2) != 1 or us.stride(2) != 1 or vs.stride(2) != 1 or us.stride(0) != vs.stride(0):
            raise ValueError("input planes need unit sample stride and equal chroma slot strides")
        self.hip.hevc_prep_frame(B, ys.data_ptr(), us.data_ptr(), vs.data_ptr(), ys.stride(0) * bps, us.stride(0) * bps,
                                 ys.stride(1), us.stride(1), bps, w, h, self.src[0].data_ptr(), self.src[1].data_ptr(),
                                 self.src[2].data_ptr(), self.src8.data_ptr() if proxy else 0, self.W, self.H, shift,
                                 self.p.bit_depth, self._stream())

    # ------------------------------------------------------------------ rate control
    def _analysis(self, y: torch.Tensor, la) -> dict:
        """The lookahead of one batch on the current stream: host results (frame costs, scene
        cuts) synchronised, the cutree offsets left on the device."""
        from ..rc.lookahead import GpuLookahead
        from ..rc.ratecontrol import MBTREE_STRENGTH, scenecut_flags

        y8 = y
        if y.dtype != torch.uint8:
            y8 = (y >> (self.p.bit_depth - 8)).clamp_(0, 255).to(torch.uint8)
        lbw, lbh = GpuLookahead.block_grid(y.shape[3], y.shape[2])
        # cutree needs the lookahead's block grid to be the coded 16x16 grid (no -s resize); the
        # 32-aligned coded height may add one 16-row below the lookahead's last row
        # Pieces shorter than 8 pictures give the propagation too little to offset cutree's
        # constant CRF compensation ((1 - qcomp) x 13.5 QP): they keep the plain CRF QPs.
        use_tree = self.p.cutree and lbw == self.wmb and lbh <= self.hmb and y.shape[1] >= 8
        badapt = bool(self.p.b_adapt) and self.nb > 0 and y.shape[1] >= 3
        cutree = multi = None
        if use_tree:
            costs_d, cutree = la.mbtree(y8.contiguous(), MBTREE_STRENGTH)
            blk, mv = la.last_blk, la.last_mv
        elif badapt:
            costs_d, blk, mv = la.frame_costs(y8.contiguous(), block_costs=True, block_mvs=True)
        else:
            costs_d, blk, mv = la.frame_costs(y8.contiguous()), None, None
        if badapt:
            multi = la.multi_costs(y8.contiguous(), blk, mv, min(7, self.nb + 1),
                                   search_range=int(self.p.badapt_range)).cpu().numpy()
        costs = costs_d.cpu().numpy()
        return dict(costs=costs, cutree=cutree, use_tree=use_tree, rows=lbh, blocks=lbw * lbh, multi=multi,
                    scenecuts=scenecut_flags(costs, float(self.p.scenecut), keyint=self.p.keyint or None),
                    shape=tuple(y.shape))

    def crf_qps(self, y: torch.Tensor, analysis: dict | None = None) -> np.ndarray:
        """[B, F] CRF QPs: GPU lookahead on the (8-bit proxy of the) luma -> CRF curve.
        ``analysis``: the batch's lookahead from :meth:`analyse_async` (None: run it here)."""
        from ..rc.lookahead import GpuLookahead
        from ..rc.ratecontrol import crf_qps_batch

        t0 = time.perf_counter()
        if analysis is None or analysis["shape"] != tuple(y.shape):
            if getattr(self, "_la", None) is None:
                self._la = GpuLookahead(self.dev, self.p.la_range, weighted=self.p.la_weights)
            analysis = self._analysis(y, self._la)
        else:
            torch.cuda.current_stream(self.dev).wait_event(analysis["event"])
            self.timings["lookahead_async_s"] = self.timings.get("lookahead_async_s", 0.0) + analysis["seconds"]
        self._cutree, self._cutree_rows = analysis["cutree"], analysis["rows"]
        self._scenecuts = analysis["scenecuts"]
        self._la_costs, self._la_multi, self._la_blocks = analysis["costs"], analysis.get("multi"), analysis["blocks"]
        q = crf_qps_batch(analysis["costs"], float(self.p.crf), analysis["blocks"], keyint=self.p.keyint or None,
                          scenecuts=self._scenecuts, mbtree=analysis["use_tree"], bframes=self.nb)
        self.stats["scenecuts"] = int(self._scenecuts.sum())
        self.timings["lookahead_s"] = self.timings.get("lookahead_s", 0.0) + time.perf_counter() - t0
        return q

    def analyse_async(self, y: torch.Tensor, after: torch.cuda.Event | None = None,
                      stream: torch.cuda.Stream | None = None) -> cf.Future:
        """Start the lookahead of a *later* batch while the current one encodes (as
        GpuH264Encoder.analyse_async): its own stream (after ``after``, e.g. the end of the
        batch's synthesis or decode), host thread and lookahead workspace; the returned future
        goes to :meth:`encode_async` / :meth:`encode` as ``analysis=``."""
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

    # ------------------------------------------------------------------ B-picture helpers
    @staticmethod
    def _dsf(td: int, tb: int) -> int:
        """DistScaleFactor of 8.5.3.2.8 (C division, clipped distances)."""
        td = max(-128, min(127, td))
        tb = max(-128, min(127, tb))
        q = (16384 + (abs(td) >> 1)) // abs(td)
        tx = q if td > 0 else -q
        return max(-4096, min(4095, (tb * tx + 32) >> 6))

    @staticmethod
    def _scale(mv: torch.Tensor, td, tb: int) -> torch.Tensor:
        """8.5.3.2.8 vector scaling by tb / td; ``td``: one distance or a per-block int tensor
        (shaped like mv without its last axis)."""
        if not isinstance(td, torch.Tensor):
            if td == tb or td == 0:
                return mv
            p = mv * GpuHevcEncoder._dsf(td, tb)
            return (torch.sign(p) * ((p.abs() + 127) >> 8)).clamp_(-32768, 32767)
        tdc = td.clamp(-128, 127)
        tbc = max(-128, min(127, tb))
        q = (16384 + (tdc.abs() >> 1)) // tdc.abs().clamp(min=1)
        dsf = ((tbc * torch.where(tdc > 0, q, -q) + 32) >> 6).clamp_(-4096, 4095)
        p = mv * dsf[..., None]
        out = (torch.sign(p) * ((p.abs() + 127) >> 8)).clamp_(-32768, 32767)
        return torch.where(((td == tb) | (td == 0))[..., None], mv, out)

    def _store_col(self, slot: int, pic=None):
        """A reference picture just coded may become the collocated picture of later B
        pictures: its records at each 16x16 block's top-left granule (z-order granules
        0 / 4 / 8 / 12), kept per DPB slot."""
        B, hc, wc = self.B, self.hctb, self.wctb
        rec = self.cu.view(B, hc, wc, 4, 4, 16)[:, :, :, :, 0, :].reshape(B, hc, wc, 2, 2, 16)
        rec = rec.permute(0, 1, 3, 2, 4, 5).reshape(B, self.hmb, self.wmb, 16)
        inter = rec[..., 0] == 1
        d = rec[..., 12]
        self.col_dir[slot].copy_(torch.where(inter, torch.where(d == 0, torch.ones_like(d), d), torch.zeros_like(d)))
        self.col_mv0[slot].copy_(rec[..., 4:8].contiguous().view(torch.int16).to(torch.int32))
        self.col_mv1[slot].copy_(rec[..., 8:12].contiguous().view(torch.int16).to(torch.int32))
        self.col_td0[slot] = None
        if pic is not None and len(pic.refs0) > 1:
            # each block's list-0 POC distance through its refIdx (CuInfo pad[0])
            lut = torch.tensor([pic.d - r for r in pic.refs0] + [pic.d - pic.refs0[0]] * (4 - len(pic.refs0)),
                               dtype=torch.int32, device=self.dev)
            self.col_td0[slot] = lut[rec[..., 13].long().clamp_(0, 3)]

    def _temporal_candidates(self, pic, col_refs: tuple):
        """See _temporal_for; B pictures: the collocated picture is RefPicList1[0]."""
        self._temporal_for(pic, pic.s1, pic.l1, col_refs, (pic.l0, pic.l1))
        self.pm0.copy_(self.tmv[..., 0:2])
        self.pm1.copy_(self.tmv[..., 2:4])

    def _temporal_for(self, pic, cs: int, col: int, col_refs: tuple, targets: tuple):
        """TMVP merge candidate per 16x16 block (the writer's derivation for a 16x16 CU: the
        collocated bottom-right block inside the CTU row, else the centre one; a list-1-only
        collocated block gives its list-1 vector, any other its list-0 vector
        (collocated_from_l0_flag 0)) scaled to both lists, and the two searches' predictors.
        cs / col: DPB slot and display index of the collocated picture, col_refs: its own list-0 /
        list-1 references, targets: the current picture's RefPicList0[0] / RefPicList1[0] (-1: none)."""
        cdir, m0, m1 = self.col_dir[cs], self.col_mv0[cs], self.col_mv1[cs]
        ok = cdir != 0
        use1 = cdir == 2
        mv = torch.where(use1[..., None], m1, m0)
        br_ok = torch.zeros_like(ok)
        br_mv = torch.zeros_like(mv)
        br_1 = torch.zeros_like(use1)
        br_ok[:, :-1, :-1] = ok[:, 1:, 1:]
        br_mv[:, :-1, :-1] = mv[:, 1:, 1:]
        br_1[:, :-1, :-1] = use1[:, 1:, 1:]
        ctd0 = self.col_td0[cs]  # per-block list-0 distances of a multi-reference col picture
        # the bottom-right block must lie in the same CTU row (16x16 rows per CTU: 2 or 4)
        rows = 4 if self.p.ctu64 else 2
        even = (torch.arange(self.hmb, device=self.dev) % rows != rows - 1)[None, :, None]
        use_br = br_ok & even
        sel = torch.where(use_br[..., None], br_mv, mv)
        sel1 = torch.where(use_br, br_1, use1)[..., None]
        avail = (use_br | ok).reshape(self.B, self.nmb)
        td0, td1 = col - col_refs[0], col - col_refs[1]   # the col block's own POC distance per list
        if ctd0 is not None:
            br_td = torch.zeros_like(ctd0)
            br_td[:, :-1, :-1] = ctd0[:, 1:, 1:]
            td0 = torch.where(use_br, br_td, ctd0)
        for x, tgt in enumerate(targets):
            if tgt < 0:
                self.tmv[..., 2 * x:2 * x + 2].zero_()
                continue
            tb = pic.d - tgt
            v = torch.where(sel1, self._scale(sel, td1, tb), self._scale(sel, td0, tb)).reshape(self.B, self.nmb, 2)
            self.tmv[..., 2 * x:2 * x + 2].copy_(v * avail[..., None].to(torch.int32))
        self.tdir.copy_(avail.to(torch.uint8) * (3 if targets[1] >= 0 else 1))

    def _weights(self, y, u, v, plan) -> dict:
        """x265 --weightp: per P picture (coding step) and slot, the explicit weights of its
        reference from the source statistics (kernels/weightp.hip wp_stats: means and variances
        of the two source pictures' planes).  Returns {step: (host rows [B] of [w, o] x 3 or
        None, device int16 [B, 6] with weight 0 = not weighted, device int32 [B, 3] luma
        (w, o, log2) for the search's inverse-weighted source)}."""
        if not self.p.eff_weightp():
            return {}
        steps = [(t, pic) for t, pic in enumerate(plan) if pic.kind == "P"]
        if not steps:
            return {}
        B, F, h, w = y.shape
        st = torch.empty((B, F, 6), dtype=torch.int64, device=self.dev)
        stats = self.hip.wp_stats if y.dtype == torch.uint8 else self.hip.wp_stats16
        stats(y.data_ptr(), u.data_ptr(), v.data_ptr(), w, h, B * F, st.data_ptr(), self._stream())
        sh = st.cpu().numpy().astype(np.float64)
        n = np.array([w * h, w * h / 4, w * h / 4])
        # weights are unit-free; offsets are coded in 8-bit units (7.4.7.3, no high-precision
        # offsets: the decoder scales them by 2^(BitDepth - 8)), so 10-bit input is measured
        # at 8-bit scale
        unit = 1.0 if y.dtype == torch.uint8 else float(1 << (self.p.bit_depth - 8))
        mean = sh[..., 0::2] / n / unit
        var = np.maximum(sh[..., 1::2] / n / unit ** 2 - mean ** 2, 0.0)
        out = {}
        for t, pic in steps:
            m1, m0 = mean[:, pic.d], mean[:, pic.l0]
            v1, v0 = var[:, pic.d], var[:, pic.l0]
            scale = np.where(v0 > 1e-3, np.sqrt(v1 / np.maximum(v0, 1e-3)), 1.0)
            use = (np.abs(m1[:, 0] - m0[:, 0]) >= self.p.wp_min_mean) | (np.abs(scale[:, 0] - 1) >= self.p.wp_min_scale)
            if not use.any():
                continue
            # weight >= 1: the kernels read weight 0 as "this slot is not weighted" (hevc_inter.hip),
            # so a fade to a flat plane (variance -> 0) must not quantise to 0 while the writer
            # still codes the flag -- the decoder would predict offset-only samples
            wq = np.clip(np.round(scale * 64), 1, 127).astype(np.int64)
            oq = np.clip(np.round(m1 - wq / 64.0 * m0), -128, 127).astype(np.int64)
            rows = [[int(x) for c in range(3) for x in (wq[b, c], oq[b, c])] if use[b] else None for b in range(B)]
            dev = np.zeros((B, 6), np.int16)
            wsrc = np.zeros((B, 3), np.int32)
            wsrc[:, 0], wsrc[:, 2] = 64, 6
            for b in range(B):
                if use[b]:
                    dev[b] = rows[b]
                    wsrc[b, 0], wsrc[b, 1] = rows[b][0], rows[b][1]
            out[t] = (rows, torch.from_numpy(dev).to(self.dev), torch.from_numpy(wsrc).to(self.dev))
        self.stats["weightp_pictures"] = int(sum(sum(r is not None for r in v[0]) for v in out.values()))
        return out

    def _plan(self, F: int, cuts_h: np.ndarray, anchors_at) -> list:
        from .gop import GopPic, hevc_gop_plan
        forced = set(anchors_at) | {d for d in range(1, F) if cuts_h[:, d].any()}
        types = None
        multi = getattr(self, "_la_multi", None)
        if self.p.b_adapt and self.nb and multi is not None and multi.shape[:2] == (self.B, F):
            # x265 --b-adapt, one pattern for the batch: the slots' summed lowres costs
            from ..rc.badapt import b_adapt_types
            costs = self._la_costs
            types = b_adapt_types(costs[:, :, 1].sum(axis=0), multi.sum(axis=0), multi[:, :, 0].sum(axis=0), self.nb,
                                  self._la_blocks * self.B, forced, int(self.p.b_bias))
            self.stats["b_ratio"] = types.count("B") / max(1, F)
        if self.nb or self.nrefs > 1:
            return hevc_gop_plan(F, self.nb, self.p.pyramid, forced, ref_slots=self.ref_slots, refs=self.nrefs,
                                 types=types)
        out = []
        for t in range(F):
            idr = t == 0 or self.p.intra_only or (self.p.keyint > 0 and t % self.p.keyint == 0)
            if idr:
                out.append(GopPic(t, "I", True, t & 1))
            else:
                out.append(GopPic(t, "P", True, t & 1, ((t - 1, True),), t - 1, -1, (t - 1) & 1))
        return out

    # ------------------------------------------------------------------ encode
    def encode(self, y: torch.Tensor, u: torch.Tensor, v: torch.Tensor, qps: np.ndarray | None = None,
               keep_recon: bool = False, metrics: bool = True, qp_delta=None, rate_fb=None,
               anchors_at=(), analysis=None) -> list[HevcSegmentResult]:
        """See :meth:`_encode`; completes the batch (and any batch still in flight first)."""
        self.drain()
        if isinstance(analysis, cf.Future):
            analysis = analysis.result()
        return self._encode(y, u, v, qps, keep_recon, metrics, qp_delta, rate_fb, anchors_at, analysis)()

    def encode_async(self, y: torch.Tensor, u: torch.Tensor, v: torch.Tensor, **kw) -> "PendingHevc":
        """Issue a batch and return before its CABAC tail finishes: the last steps' entropy jobs
        (host threads) and the result assembly overlap the next batch's GPU work.  At most two
        batches are in flight (issuing a third completes the oldest).  ``.result()`` gives what
        :meth:`encode` returns.  ``kw``: :meth:`encode`'s keyword arguments; ``analysis`` may be
        the future from :meth:`analyse_async`."""
        ana = kw.pop("analysis", None)
        if isinstance(ana, cf.Future):
            ana = ana.result()
        while len(self._inflight) >= 2:
            self._inflight[0].result()
        fin = self._encode(y, u, v, kw.get("qps"), kw.get("keep_recon", False), kw.get("metrics", True),
                           kw.get("qp_delta"), kw.get("rate_fb"), kw.get("anchors_at", ()), ana)
        pend = PendingHevc(self, fin)
        self._inflight.append(pend)
        return pend

    def drain(self) -> None:
        """Complete every batch issued by :meth:`encode_async`."""
        while self._inflight:
            self._inflight[0].result()

    def _encode(self, y: torch.Tensor, u: torch.Tensor, v: torch.Tensor, qps: np.ndarray | None = None,
                keep_recon: bool = False, metrics: bool = True, qp_delta=None, rate_fb=None,
                anchors_at=(), analysis=None):
        """y: [B, F, h, w] (uint8, or uint16 holding bit_depth-bit samples), u/v half size.
        Every segment starts with an IDR picture; then P anchors and (bframes) the B pictures
        between them, in coding order (models/gop.py; a scene cut becomes an anchor coded all
        intra).  ``qps``: [B, F] display order.  ``anchors_at``: display indices that must be
        anchors, so a segment shorter than F ends on a coding-order prefix (display_prefix).

        ``rate_fb`` (:class:`~govideocompressor_amd.rc.ratecontrol.TwoPassFeedback`): pass-2
        rate feedback -- before every frame step the controller sees the bits of the pictures
        whose CABAC has finished and may re-solve the QPs of the frames not yet started (its
        arrays are in coding order, ``self.last_order``)."""
        B, F, h, w = y.shape
        if B != self.B or (w, h) != (self.p.width, self.p.height):
            raise ValueError(f"expected [{self.B}, F, {self.p.height}, {self.p.width}], got {list(y.shape)}")
        # Returns the batch's finisher: waits for its CABAC jobs, checks the device error flag
        # and builds the results (encode calls it at once, encode_async later).
        if y.device != self.dev:
            raise ValueError("inputs must live on the encoder's device")
        qi, qpp = self.p.frame_qps()
        self._scenecuts = None
        self._cutree = None
        self._la_multi = None
        from_la = False
        if qps is None and self.p.crf is not None and self.p.lookahead and not self.p.intra_only:
            qps = self.crf_qps(y, analysis)
            from_la = True
        cuts_h = self._scenecuts if self._scenecuts is not None else np.zeros((B, F), dtype=bool)
        plan = self._plan(F, cuts_h, anchors_at)
        order = [pic.d for pic in plan]
        self.last_order = order
        wps = self._weights(y, u, v, plan)  # coding step -> (host [B, 6] or None rows, device tables)
        if qps is None:
            qps = np.array([[qi if pic.kind == "I" else qpp for pic in sorted(plan, key=lambda q: q.d)]
                            for _ in range(B)], dtype=np.int32)
            from_la = True
        cfg = self.p.host_cfg()
        if self.p.wpp:  # spread the native threads over the B pictures of a step
            cfg["threads"] = max(1, min(32, self.entropy_threads // max(1, B)))
        qps = np.clip(np.asarray(qps, dtype=np.int32).reshape(B, F), 0, 51)
        if self.nb and from_la:
            # x265 --pbratio: a B picture takes the distance-weighted QP of its references plus
            # the offset (half of it for a pyramid's reference B)
            from ..rc.ratecontrol import b_qps_from_refs
            qps = b_qps_from_refs(qps, plan, float(self.p.b_qp_offset))
        if qp_delta is not None:
            from ..rc.abr import apply_delta
            qps = apply_delta(qps, qp_delta)
        qps_c = np.ascontiguousarray(qps[:, order])  # coding order
        if rate_fb is not None:
            qps_c = np.array(rate_fb.qps, dtype=np.int32).reshape(B, F)
        qps_d = torch.from_numpy(np.ascontiguousarray(qps_c.T)).to(self.dev)  # [F, B] coding order, one upload
        cuts_c = cuts_h[:, order]
        cuts_d = torch.from_numpy(np.ascontiguousarray(cuts_c.T)).to(self.dev)  # [F, B]
        fb_known, fb_spent, fb_stage = 0, np.zeros((B, F)), []
        nals: list[list] = [[None] * F for _ in range(B)]
        futs = []
        pending = self._pending  # per pinned host buffer set: CABAC jobs still reading it (across batches)
        sse = []
        recon = [None] * F if keep_recon else None
        t_gpu = t_host = t_blocked = 0.0
        cabac_s = [0.0]
        p = self._p
        s = self._stream()
        bd = self.p.bit_depth
        st = self.stage_timer
        gate_sum: list[torch.Tensor] = []
        tmvp = bool(cfg.get("tmvp", 0))
        anchor_cu: dict = {}   # display index of a reference picture -> (host copy of its CU records or None, l0, l1)
        ref_lists: dict = {}   # display index of a reference picture -> its (l0, l1) display indices
        anchor_meta: dict = {}  # (GPU entropy) display index of a reference picture -> (DPB slot, l0, l1, refs0)
        # the writer's CU statistics (cu_stats diagnostics) come from the host writer
        gpu_entropy = self.entropy == "gpu" and self.cu_stats is None
        plan_refs = {pic.d: pic.kind for pic in plan if pic.ref}
        idr_d = 0              # display index of the latest IDR picture (POC 0)
        for t in range(F):
            pic = plan[t]
            d = pic.d
            if pic.kind == "I":
                idr_d = d
            t0 = time.perf_counter()
            if rate_fb is not None and t > 0:
                # bits of the pictures whose CABAC jobs have finished (coding order prefix)
                while fb_known < len(futs) and futs[fb_known][1].done():
                    for b, nal in enumerate(futs[fb_known][1].result()):
                        fb_spent[b, fb_known] = 8 * len(nal)
                    fb_known += 1
                newq = np.asarray(rate_fb.update(fb_known, fb_spent, t), dtype=np.int32)
                if not np.array_equal(newq[:, t:], qps_c[:, t:]):
                    qps_c[:, t:] = newq[:, t:]
                    staged = torch.from_numpy(np.ascontiguousarray(qps_c[:, t:].T)).pin_memory()
                    qps_d[t:].copy_(staged, non_blocking=True)  # stream-ordered before frame t's read
                    fb_stage.append(staged)  # keep the pinned source alive until the encode ends
            idr = pic.kind == "I"
            self._prep(y, u, v, d, proxy=not idr)
            self.qp.copy_(qps_d[t])  # device-to-device: no host sync inside the frame loop
            # per-CTB QPs (AQ + cutree offsets of frame d); without them every CTB at the frame QP.
            # cutree offsets belong to referenced pictures: B pictures get variance AQ only
            extra, estride, erows = 0, 0, 0
            if self._cutree is not None and self.p.adaptive_qp() and pic.ref:
                ct = self._cutree
                extra, estride, erows = ct.data_ptr() + d * ct.shape[2] * 4, ct.shape[1] * ct.shape[2], self._cutree_rows
            with st("aq"):
                self.hip.hevc_aq(B, self.W, self.H, bd, p(self.src[0]), p(self.src[1]), p(self.src[2]), p(self.qp),
                                 float(self.p.aq_strength) if self.p.adaptive_qp() else 0.0, extra, estride, erows,
                                 p(self.ctb_qp), p(self.mb_aq), s)
            ci, r0, r1 = pic.slot, pic.s0, pic.s1
            cur, ref = self.rec[ci], self.rec[r0]
            kb = t % 2
            # the copy-out of step t - 2 must have read these buffers before they are rewritten
            torch.cuda.current_stream(self.dev).wait_event(self.copy_done[kb])
            self.coef, self.ctu, self.cu = self.coefs[kb], self.ctus[kb], self.cus[kb]
            intra_args = (B, self.W, self.H, p(self.src[0]), p(self.src[1]), p(self.src[2]), p(cur[0]), p(cur[1]),
                          p(cur[2]), p(self.ctu), p(self.cu), p(self.coef[0]), p(self.coef[1]), p(self.coef[2]),
                          p(self.ctb_qp), p(self.run), p(self.cand), bd)
            if idr:
                self.run.fill_(1)
                self.prev_mv.zero_()  # no motion predictors across a closed GOP (or from an earlier call)
                with st("intra_i"):
                    self.hip.hevc_intra(*intra_args, 1, 1, p(self.err), s, int(self.p.sdh), 0, int(self.p.ctu64))
            else:
                self.run.fill_(2)
                ref8, hp = self.ref8s[r0], self.me_hps[r0]
                inter_kw = {}
                s8 = p(self.src8)
                if t in wps:
                    # weighted P picture: the searches see the inverse-weighted source proxy
                    # against the unweighted reference (kernels/weightp.hip wp_src)
                    self.hip.wp_src(p(self.src8), p(self.src8w), p(wps[t][2]), B, self.H * self.W, s)
                    s8 = p(self.src8w)
                    inter_kw["wp"] = p(wps[t][1])
                if pic.kind == "P":
                    with st("me"):
                        self.hip.me(B, self.wmb, self.hmb, s8, p(ref8), p(self.prev_mv), p(self.mv),
                                    p(self.me_cost), p(self.me_pred), p(self.me_intra), p(self.qp), self.p.me_range,
                                    self.p.subpel, s, p(hp), p(self.mb_aq), 1)
                    nr = len(pic.refs0) if self.nrefs > 1 else 1
                    far = {}
                    if nr > 1:
                        # x265 --ref: the farther list-0 pictures, 16x16 searches seeded by the list-0[0]
                        # vectors scaled by the temporal distances (unweighted source: explicit
                        # weights belong to RefPicList0[0]), skipped where list-0[0] is good enough
                        sk = pic.srefs0[1:]
                        with st("me_ref"):
                            for k in range(1, nr):
                                scale = (pic.d - pic.refs0[k]) / float(pic.d - pic.refs0[0])
                                self.xpm[k - 1].copy_((self.mv.float() * scale).round_().clamp_(-2048, 2047))
                                self.hip.me(B, self.wmb, self.hmb, p(self.src8), p(self.ref8s[sk[k - 1]]),
                                            p(self.xpm[k - 1]), p(self.xmv[k - 1]), p(self.xcost[k - 1]), p(self.xpred),
                                            0, p(self.qp), int(self.p.ref_range), self.p.subpel, s,
                                            p(self.me_hps[sk[k - 1]]), p(self.mb_aq), 1, gate_cost=p(self.me_cost),
                                            gate_thresh=int(self.p.ref_gate))
                        far = dict(nref0=nr, xref=[p(self.ref8s[k]) for k in sk], xhp=[p(self.me_hps[k]) for k in sk])
                        inter_kw["xref"] = [p(c) for k in sk for c in self.rec[k]]
                    with st("merge_refine"):
                        if self.p.merge_exact:
                            # the search as list-0 motion, then the writer-exact merge passes
                            # (temporal candidates from RefPicList0[0]'s motion)
                            tm_, td_ = 0, 0
                            if tmvp and plan_refs.get(pic.l0, "I") != "I":
                                self._temporal_for(pic, r0, pic.l0, ref_lists[pic.l0], (pic.l0, -1))
                                tm_, td_ = p(self.tmv), p(self.tdir)
                            pargs = (B, self.wmb, self.hmb, s8, p(ref8), p(ref8), p(hp), p(hp))
                            xs = dict(xmv=p(self.xmv), xcost=p(self.xcost), xpm=p(self.xpm)) if far else {}
                            self.hip.hevc_b(2, *pargs, p(self.mv), 0, p(self.me_cost), 0, p(self.prev_mv), 0, 0, 0, 0, 0,
                                            p(self.mvb[0]), p(self.dirb[0]), p(self.bcost), p(self.bbits), p(self.qp),
                                            p(self.mb_aq), s, 0, int(self.p.max_merge), int(self.p.ctu64), **far, **xs)
                            for it in range(int(self.p.merge_refine)):
                                i_, o_ = it % 2, (it + 1) % 2
                                self.hip.hevc_b(1, *pargs, 0, 0, 0, 0, 0, 0, tm_, td_, p(self.mvb[i_]), p(self.dirb[i_]),
                                                p(self.mvb[o_]), p(self.dirb[o_]), p(self.bcost), p(self.bbits),
                                                p(self.qp), p(self.mb_aq), s, 0, int(self.p.max_merge), int(self.p.ctu64),
                                                *self._chg_args(it), **far)
                            fin = int(self.p.merge_refine) % 2
                            self.me_cost.copy_(self.bcost)
                            self.mv.copy_(self.mvb[fin][..., 0:2])
                            inter_kw.update(mvb=p(self.mvb[fin]), dirb=p(self.dirb[fin]), f1y=p(ref[0]), f1u=p(ref[1]),
                                            f1v=p(ref[2]))
                            if self.p.inter8:
                                # 8x8 inter CUs: per-quadrant vectors of RefPicList0[0] blocks, priced
                                # against the merge-aware 16x16 cost (me_cost updated where they win)
                                with st("inter8"):
                                    self.hip.p_part8(B, self.wmb, self.hmb, s8, p(ref8), p(hp), p(self.mv),
                                                     p(self.prev_mv), p(self.me_cost), 0, p(self.mv8), p(self.qp),
                                                     p(self.mb_aq), int(self.p.inter8_overhead),
                                                     int(self.p.inter8_min_satd), s, bits16=p(self.bbits),
                                                     dir16=p(self.dirb[fin]))
                                inter_kw["mv8"] = p(self.mv8)
                        else:
                            if far:
                                raise ValueError("HevcParams.refs > 1 needs merge_exact")
                            for it in range(int(self.p.merge_refine)):
                                a_, b_ = (self.mv, self.mv_tmp) if it % 2 == 0 else (self.mv_tmp, self.mv)
                                self.hip.hevc_merge_refine(B, self.wmb, self.hmb, s8, p(ref8), p(hp), p(a_),
                                                           p(b_), p(self.me_cost), p(self.prev_mv), p(self.qp),
                                                           p(self.mb_aq), s)
                            if int(self.p.merge_refine) % 2:
                                self.mv.copy_(self.mv_tmp)
                else:
                    ref8b, hpb = self.ref8s[r1], self.me_hps[r1]
                    with st("me_b"):
                        self._temporal_candidates(pic, ref_lists[pic.l1])
                        self.hip.me(B, self.wmb, self.hmb, p(self.src8), p(ref8), p(self.pm0), p(self.mv),
                                    p(self.me_cost), p(self.me_pred), p(self.me_intra), p(self.qp), self.p.me_range,
                                    self.p.subpel, s, p(hp), p(self.mb_aq), 1)
                        # the list-1 search skips the open-loop intra estimate the list-0 search wrote
                        self.hip.me(B, self.wmb, self.hmb, p(self.src8), p(ref8b), p(self.pm1), p(self.mv1),
                                    p(self.me_cost1), p(self.me_pred), 0, p(self.qp), self.p.me_range, self.p.subpel,
                                    s, p(hpb), p(self.mb_aq), 1)
                    with st("b_decide"):
                        bargs = (B, self.wmb, self.hmb, p(self.src8), p(ref8), p(ref8b), p(hp), p(hpb))
                        self.hip.hevc_b(0, *bargs, p(self.mv), p(self.mv1), p(self.me_cost), p(self.me_cost1),
                                        p(self.pm0), p(self.pm1), 0, 0, 0, 0, p(self.mvb[0]), p(self.dirb[0]),
                                        p(self.bcost), p(self.bbits), p(self.qp), p(self.mb_aq), s, 1, int(self.p.max_merge), int(self.p.ctu64))
                        tm_, td_ = (p(self.tmv), p(self.tdir)) if tmvp else (0, 0)
                        for it in range(int(self.p.merge_refine)):
                            i_, o_ = it % 2, (it + 1) % 2
                            self.hip.hevc_b(1, *bargs, 0, 0, 0, 0, 0, 0, tm_, td_, p(self.mvb[i_]), p(self.dirb[i_]),
                                            p(self.mvb[o_]), p(self.dirb[o_]), p(self.bcost), p(self.bbits), p(self.qp),
                                            p(self.mb_aq), s, 1, int(self.p.max_merge), int(self.p.ctu64),
                                            *self._chg_args(it))
                        fin = int(self.p.merge_refine) % 2
                        self.me_cost.copy_(self.bcost)
                    r1p = self.rec[r1]
                    inter_kw = dict(mvb=p(self.mvb[fin]), dirb=p(self.dirb[fin]), f1y=p(r1p[0]), f1u=p(r1p[1]),
                                    f1v=p(r1p[2]))
                if cuts_c[:, t].any():  # scene cut: every CU of these slots goes intra
                    self.me_cost.masked_fill_(cuts_d[t][:, None], 1 << 26)
                with st("intra_analyze"):  # open-loop intra candidates where intra may still win
                    mask = p(self._intra_gate()) if self.p.intra_gate else 0
                    if mask:
                        gate_sum.append(self.ctb_need.sum(dtype=torch.int64))
                    self.hip.hevc_intra(*intra_args, 1, 0, p(self.err), s, int(self.p.sdh), mask, int(self.p.ctu64))
                with st("inter"):
                    self.hip.hevc_inter(B, self.W, self.H, p(self.src[0]), p(self.src[1]), p(self.src[2]), p(ref[0]),
                                        p(ref[1]), p(ref[2]), p(cur[0]), p(cur[1]), p(cur[2]), p(self.ctu), p(self.cu),
                                        p(self.coef[0]), p(self.coef[1]), p(self.coef[2]), p(self.ctb_qp), p(self.run),
                                        p(self.cand), p(self.mv), p(self.me_cost), bd, s, int(self.p.tu_inter_depth),
                                        int(self.p.sdh), int(self.p.intra_bias_p), **inter_kw)
                with st("intra_recon"):
                    self.hip.hevc_intra(*intra_args, 0, 1, p(self.err), s, int(self.p.sdh), 0,
                                        int(self.p.ctu64))   # intra CUs, wavefront
                if pic.kind == "P":
                    self.prev_mv.copy_(self.mv)
            self.hip.hevc_qp_fixup(B, self.W, self.H, p(self.ctu), p(self.cu), p(self.qp), p(self.run), int(self.p.wpp), s,
                                   int(self.p.ctu64))
            if self.p.deblock:
                with st("deblock"):
                    self.hip.hevc_deblock(B, self.W, self.H, bd, p(cur[0]), p(cur[1]), p(cur[2]), p(self.cu),
                                          p(self.ctu), p(self.run), s)
            if self.p.sao:
                # SAO reads the deblocked picture and writes every sample of the output:
                # ping-pong with the spare buffer instead of copying the input
                out_pl = self.dbk
                with st("sao"):
                    self.hip.hevc_sao(B, self.W, self.H, bd, p(cur[0]), p(cur[1]), p(cur[2]), p(out_pl[0]),
                                      p(out_pl[1]), p(out_pl[2]), p(self.src[0]), p(self.src[1]), p(self.src[2]),
                                      p(self.ctu), p(self.ctb_qp), p(self.run), 1, s, int(self.p.ctu64))
                self.dbk = cur
                self.rec[ci] = cur = out_pl
            if pic.ref:
                # a reference picture's 8-bit proxy and half-sample planes (shared by every
                # picture that references it) and its motion as a collocated field
                with st("halfpel"):
                    self.hip.hevc_proxy8(p(cur[0]), p(self.ref8s[ci]), cur[0].numel(), bd - 8, s)
                    self.hip.me_halfpel(B, self.W, self.H, p(self.ref8s[ci]), p(self.me_hps[ci]), s)
                ref_lists[d] = (pic.l0, pic.l1)
                if tmvp:
                    if idr:
                        self.col_dir[ci].zero_()
                        self.col_td0[ci] = None
                    else:
                        self._store_col(ci, pic)
            if metrics:
                dd = (cur[0][:, :h, :w].to(torch.int32) - self.src[0][:, :h, :w].to(torch.int32))
                sse.append((dd * dd).sum(dim=(1, 2)).to(torch.float64))
            if keep_recon:
                recon[d] = tuple(c.clone() for c in cur)
            # records to pinned host memory on the copy stream; CABAC on the thread pool
            hb = t % 3
            if pending[hb]:  # the CABAC jobs of step t - 3 still read this host buffer set
                # (a CABAC job first waits for its records' copy, i.e. for step t - 3's GPU work:
                # this wait is GPU time as much as entropy time)
                tb = time.perf_counter()
                for f in pending[hb]:
                    f.result()
                pending[hb] = []
                t_blocked += time.perf_counter() - tb
            nzmap, nzoff = self.nzmaps[kb], self.nzoffs[kb]
            qcol = qps_c[:, t].copy()
            wrow = wps[t][0] if t in wps else None
            if gpu_entropy:
                job = self._gpu_entropy_step(t, pic, idr_d, kb, hb, cfg, qps_d[t], qcol, wrow, tmvp, anchor_meta,
                                             ref_lists, cabac_s)
                t1 = time.perf_counter()
                t_gpu += t1 - t0
            else:
                host = self._host_buffers()[hb]
                # non-zero level blocks straight into this step's pinned host buffer
                self.hip.hevc_pack_levels(B, self.W, self.H, p(self.coef[0]), p(self.coef[1]), p(self.coef[2]), p(nzmap),
                                          p(self.nzcnt), p(nzoff), self.pack_cap, host[4].data_ptr(), p(self.err), s)
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.dev))
                with torch.cuda.stream(self.copy_stream):
                    self.copy_stream.wait_event(ev)
                    for dst, src_t in zip(host[:4], (self.ctu, self.cu, nzmap, nzoff)):
                        dst.copy_(src_t, non_blocking=True)
                    done = torch.cuda.Event()
                    done.record(self.copy_stream)
                    self.copy_done[kb].record(self.copy_stream)
                ctu, cu = host[0].numpy(), host[1].numpy()
                nz, off, lv = host[2].numpy().view(np.uint64), host[3].numpy().view(np.uint32), host[4].numpy()
                t1 = time.perf_counter()
                t_gpu += t1 - t0

                def job(done=done, pic=pic, qcol=qcol, ctu=ctu, cu=cu, nz=nz, off=off, lv=lv, i0=idr_d, wrow=wrow):
                    done.synchronize()
                    tj = time.perf_counter()
                    # POC counts display pictures from the latest IDR
                    base = dict(idr=int(pic.kind == "I"), poc=pic.d - i0, slice_type={"I": 2, "P": 1, "B": 0}[pic.kind],
                                nal_ref=int(pic.ref), rps=[(rd - i0, int(u)) for rd, u in pic.rps])
                    if pic.kind != "I":
                        base["ref_poc0"] = pic.l0 - i0
                        if len(pic.refs0) > 1:
                            base["refs0"] = [r - i0 for r in pic.refs0]
                    if pic.kind == "B":
                        base["ref_poc1"] = pic.l1 - i0
                    col = None
                    if tmvp and pic.kind != "I":
                        cd = pic.l1 if pic.kind == "B" else pic.l0
                        col = anchor_cu[cd]
                        base.update(col_poc=cd - i0, col_ref_poc0=col[1] - i0, col_ref_poc1=col[2] - i0)
                        if len(col[3]) > 1:
                            base["col_refs0"] = [r - i0 for r in col[3]]
                    fps = []
                    for b in range(B):
                        fp = dict(base, qp=int(qcol[b]))
                        if wrow is not None and wrow[b] is not None:
                            fp["wp"] = wrow[b]
                        if col is not None:
                            fp["col_cu"] = None if col[0] is None else col[0][b]
                        fps.append(fp)
                    if self.cu_stats is None:
                        r = self.host.hevc_write_slices_packed(cfg, fps, ctu, cu, nz, off, lv, self.entropy_threads)
                    else:  # diagnostics: CU mix per picture type (tools/diag/hevc_bframe_stats.py)
                        rs = self.host.hevc_write_slices_packed(cfg, fps, ctu, cu, nz, off, lv, self.entropy_threads, True)
                        r = [n for n, _ in rs]
                        agg = self.cu_stats.setdefault(pic.kind + ("ref" if pic.kind == "B" and pic.ref else ""), {})
                        for _, stt in rs:
                            for k_, v_ in stt.items():
                                agg[k_] = agg.get(k_, 0) + v_
                    if tmvp and pic.ref:
                        # later pictures' collocated records (the host buffer set is reused at t + 3);
                        # only pictures still in the DPB can be collocated pictures
                        anchor_cu[pic.d] = (None if pic.kind == "I" else cu[:B].copy(), pic.l0, pic.l1, pic.refs0)
                        live = {rd for rd, _ in pic.rps} | {pic.d}
                        for k in [k for k in anchor_cu if k not in live]:
                            del anchor_cu[k]
                    cabac_s[0] += time.perf_counter() - tj
                    return r

            f = self.pool.submit(job)
            futs.append((t, f))
            pending[hb].append(f)
        qps = np.empty_like(qps_c)
        qps[:, order] = qps_c
        self.last_qps = qps.copy()
        return lambda: self._finish(futs, nals, B, F, h, w, bd, sse, metrics, keep_recon, recon, order, gate_sum,
                                    st, t_gpu, t_blocked, cabac_s)

    @staticmethod
    def _slice_base(pic, i0: int, col_meta) -> dict:
        """Frame parameters shared by the B pictures of a coding step (POCs count display
        pictures from the latest IDR ``i0``); ``col_meta``: (l0, l1, refs0) of the collocated
        picture, or None."""
        base = dict(idr=int(pic.kind == "I"), poc=pic.d - i0, slice_type={"I": 2, "P": 1, "B": 0}[pic.kind],
                    nal_ref=int(pic.ref), rps=[(rd - i0, int(u)) for rd, u in pic.rps])
        if pic.kind != "I":
            base["ref_poc0"] = pic.l0 - i0
            if len(pic.refs0) > 1:
                base["refs0"] = [r - i0 for r in pic.refs0]
        if pic.kind == "B":
            base["ref_poc1"] = pic.l1 - i0
        if col_meta is not None:
            cd = pic.l1 if pic.kind == "B" else pic.l0
            base.update(col_poc=cd - i0, col_ref_poc0=col_meta[0] - i0, col_ref_poc1=col_meta[1] - i0)
            if len(col_meta[2]) > 1:
                base["col_refs0"] = [r - i0 for r in col_meta[2]]
        return base

    def _gpu_entropy_step(self, t, pic, i0, kb, hb, cfg, qp_row, qcol, wrow, tmvp, anchor_meta, ref_lists, cabac_s):
        """Issue coding step t's GPU entropy on the copy stream (after the step's records are
        final): the nz maps, the CABAC substreams of the B pictures (kernels/hevc_entropy.hip)
        packed into pinned host set ``hb``, and -- for a reference picture with TMVP -- a device
        copy of its records for the pictures that will use it as collocated picture.  The
        compute stream moves on to step t + 1 at once; buffers of step t are released through
        ``copy_done[kb]``.  Returns the host job: the slice headers, entry points and emulation
        prevention of the step's pictures (hevc_assemble_slices)."""
        B, p = self.B, self._p
        nzmap, nzoff = self.nzmaps[kb], self.nzoffs[kb]
        eh = self._entropy_host()[hb]
        col_meta, col_ptr = None, 0
        if tmvp and pic.kind != "I":
            cd = pic.l1 if pic.kind == "B" else pic.l0
            slot, l0, l1, refs0 = anchor_meta[cd]
            col_meta = (l0, l1, refs0)
            col_ptr = p(self.col_cus[slot])
        base = self._slice_base(pic, i0, col_meta)
        pic_bytes = self.host.hevc_coder_pic(cfg, dict(base, qp=0))
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        cs = self.copy_stream
        with torch.cuda.stream(cs):
            cs.wait_event(ev)
            sc = cs.cuda_stream
            self.hip.hevc_pack_levels(B, self.W, self.H, p(self.coef[0]), p(self.coef[1]), p(self.coef[2]), p(nzmap),
                                      p(self.nzcnt), p(nzoff), self.pack_cap, 0, p(self.err), sc)
            self.hip.hevc_entropy(pic_bytes, B, p(qp_row), p(self.ctu), p(self.cu), col_ptr, p(nzmap), p(self.coef[0]),
                                  p(self.coef[1]), p(self.coef[2]), p(self.ent_state), self.ent_state_bytes,
                                  p(self.ent_outs[hb]), self.ent_cap, p(self.ent_sizes), p(self.ent_errs), p(self.ent_offs),
                                  eh["offs"].data_ptr(), eh["dst"].data_ptr(), self.ent_dst_cap, p(self.ent_over), sc,
                                  self._entropy_prof(pic.kind), p(self.ent_gprog), p(self.ent_gctx))
            # the batch's QP table is freed when the encode returns: keep its block from being
            # reused (by the compute stream's next batch) before this stream has read it
            qp_row.record_stream(cs)
            eh["sizes"].copy_(self.ent_sizes, non_blocking=True)
            eh["errs"].copy_(self.ent_errs, non_blocking=True)
            if tmvp and pic.ref:
                if self.col_cus is None:
                    self.col_cus = [torch.empty_like(self.cus[0]) for _ in range(self.ref_slots)]
                self.col_cus[pic.slot].copy_(self.cu, non_blocking=True)
            done = torch.cuda.Event()
            done.record(cs)
            self.copy_done[kb].record(cs)
        if tmvp and pic.ref:
            anchor_meta[pic.d] = (pic.slot, pic.l0, pic.l1, pic.refs0)
        n = B * self.ent_nsub

        def job(done=done, base=base, qcol=qcol, wrow=wrow, eh=eh, hb=hb):
            done.synchronize()
            tj = time.perf_counter()
            offs = eh["offs"].numpy().view(np.uint64)
            sizes = eh["sizes"].numpy().view(np.uint32)
            data = eh["dst"].numpy()
            if int(offs[n]) > self.ent_dst_cap:
                # the step's slice data outgrew the pinned buffer (the gather skipped it): read the
                # substreams back from this host set's device area (dense content, low QPs)
                cap = self.ent_cap
                dev = self.ent_outs[hb].view(n, cap)
                data = np.concatenate([dev[i, :int(sizes[i])].cpu().numpy() for i in range(n)]) if n else data
                offs = np.zeros(n + 1, dtype=np.uint64)
                offs[1:] = np.cumsum(sizes.astype(np.uint64))
                self.stats["entropy_readback_steps"] = self.stats.get("entropy_readback_steps", 0) + 1
            fps = []
            for b in range(B):
                fp = dict(base, qp=int(qcol[b]))
                if wrow is not None and wrow[b] is not None:
                    fp["wp"] = wrow[b]
                fps.append(fp)
            r = self.host.hevc_assemble_slices(cfg, fps, data, offs, sizes, eh["errs"].numpy(), self.entropy_threads)
            cabac_s[0] += time.perf_counter() - tj
            return r
        return job

    def _finish(self, futs, nals, B, F, h, w, bd, sse, metrics, keep_recon, recon, order, gate_sum, st, t_gpu,
                t_blocked, cabac_s) -> list[HevcSegmentResult]:
        if int(self.err.item()) != 0:
            raise RuntimeError("HEVC encoder: wavefront progress timeout")
        t2 = time.perf_counter()
        bits = [[0] * F for _ in range(B)]
        for t, f in futs:
            for b, nal in enumerate(f.result()):
                nals[b][t] = nal
                bits[b][t] = 8 * len(nal)
        t_host = time.perf_counter() - t2
        # cabac_batch_s: wall time of the native batch writer (entropy_threads threads)
        if gate_sum:
            n_p = len(gate_sum)
            self.stats["intra_analyzed_ctb_ratio"] = float(torch.stack(gate_sum).sum().item()) / (n_p * B * self.nctb)
        if st.enabled:
            self.stage_ms = {k: round(v["s"] * 1000.0, 2) for k, v in st.summary().items()}
        # loop_waits_on_step_t_minus_3_s: the frame loop waiting for the CABAC jobs of step
        # t - 3 to release their pinned host buffers -- those jobs first wait for their
        # records' device-to-host copy, so this includes GPU completion, not only entropy coding
        self.timings.update(loop_s=t_gpu, loop_waits_on_step_t_minus_3_s=t_blocked, host_wait_s=t_host,
                            cabac_batch_s=cabac_s[0], cabac_ms_per_picture_wall=1000.0 * cabac_s[0] / max(1, B * F),
                            entropy_threads=self.entropy_threads)
        out = []
        maxv = float((1 << bd) - 1)
        for b in range(B):
            ps = 0.0
            if metrics:
                mse = float(sum(x[b].item() for x in sse)) / (F * w * h)
                ps = 99.0 if mse == 0 else 10.0 * np.log10(maxv * maxv / mse)
            out.append(HevcSegmentResult(bitstream=self.params_nal + b"".join(nals[b]), frames=F, nals=nals[b],
                                         bits=bits[b], psnr_y=ps, order=list(order)))
        if keep_recon:
            self.last_recon = recon
        return out
