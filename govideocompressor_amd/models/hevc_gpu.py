"""MI355X HEVC (H.265) encoder: B closed-GOP segments encoded concurrently on one GPU.

Replaces the reference's ``-vcodec libx265 -crf 26`` worker call (server.go:67-68,
client.go:115) with gfx950 kernels + a host CABAC writer:

per frame step t (frame t of every slot):
  prep (u8/u16 -> padded u16 planes)
  -> hevc_aq: per-CTB QP (variance AQ + MB-tree offsets, one quantization group per CTB)
  -> I: hevc_intra_analyze (CTB-parallel open-loop CU/mode decision)
        + hevc_intra_recon (CTB wavefront, closed loop)
     P: lookahead motion search + hevc_inter (CU-parallel) + intra CUs (wavefront)
  -> hevc_qp_fixup (QpY of CTBs / CUs without a coded delta, 8.6.1)
  -> hevc_deblock (vertical, then horizontal edges; picture-parallel)
  -> hevc_sao (per-CTB statistics, decision, apply)
then the decision records go to pinned host memory, the non-zero 4x4 level blocks are
packed straight into pinned host memory (hevc_pack_levels: only coded levels cross
PCIe), and a host thread pool writes one CABAC slice per picture
(csrc/host/hevc_writer.cc) while the GPU works on the next step.

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

    def adaptive_qp(self) -> bool:
        return self.aq_strength > 0 or (self.cutree and self.lookahead and self.crf is not None)

    def host_cfg(self) -> dict:
        return dict(width=self.width, height=self.height, bit_depth=self.bit_depth, fps=self.fps,
                    sao=int(self.sao), deblock=int(self.deblock), max_merge=self.max_merge, wpp=int(self.wpp),
                    cu_qp_delta=int(self.adaptive_qp()), tu_inter_depth=int(self.tu_inter_depth), sdh=int(self.sdh),
                    level_idc=int(self.level_idc))

    def frame_qps(self) -> tuple[int, int]:
        qp_p = int(round(self.crf)) if self.crf is not None else int(self.qp)
        qp_p = max(0, min(51, qp_p))
        return max(0, qp_p - self.ip_offset), qp_p


@dataclass
class HevcSegmentResult:
    bitstream: bytes
    frames: int
    nals: list[bytes] = field(default_factory=list)
    bits: list[int] = field(default_factory=list)
    psnr_y: float = 0.0

    def display_prefix(self, c: int) -> list[bytes]:
        """Slice NALs of pictures 0..c-1 (P-only GOPs: coding order == display order)."""
        return self.nals[:c]


class GpuHevcEncoder:
    """Batched gfx950 HEVC encoder (Main / Main 10, CABAC)."""

    def __init__(self, params: HevcParams, slots: int, device="cuda", entropy_threads: int | None = None):
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
        self.rec = [planes(), planes()]      # current / reference
        self.dbk = planes()                  # SAO output ping-pong buffer
        self.coefs = [planes(i16), planes(i16)]  # double-buffered: copy-out of t overlaps t + 1
        self.coef = self.coefs[0]
        self.wmb, self.hmb = W // 16, H // 16
        nmb = self.wmb * self.hmb
        self.src8 = torch.zeros((B, H, W), dtype=torch.uint8, device=dev)   # motion-search proxies
        self.ref8 = torch.zeros((B, H, W), dtype=torch.uint8, device=dev)
        self.mv = torch.zeros((B, nmb, 2), dtype=torch.int16, device=dev)
        self.prev_mv = torch.zeros((B, nmb, 2), dtype=torch.int16, device=dev)
        self.mv_tmp = torch.zeros((B, nmb, 2), dtype=torch.int16, device=dev)
        self.me_cost = torch.zeros((B, nmb), dtype=torch.int32, device=dev)
        self.me_intra = torch.zeros((B, nmb), dtype=torch.int32, device=dev)
        self.me_pred = torch.zeros((B, nmb, 256), dtype=torch.uint8, device=dev)
        self.me_hp = torch.empty(B * 3 * (H + 8) * (W + 8) + 64, dtype=torch.uint8, device=dev)
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
        self.pool = cf.ThreadPoolExecutor(max_workers=1)
        self.timings: dict[str, float] = {}
        self.stats: dict[str, float] = {}
        self.ctb_need = torch.ones((B, self.nctb), dtype=torch.uint8, device=dev)
        # per-stage device time (HIP events, resolved once per encode): MIVC_STAGE_TIMING=1
        from ..obs.timers import EventTimer
        self.stage_timer = EventTimer(enabled=os.environ.get("MIVC_STAGE_TIMING", "0") == "1")

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
        self.pool.shutdown(wait=True)

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
    def crf_qps(self, y: torch.Tensor) -> np.ndarray:
        """[B, F] CRF QPs: GPU lookahead on the (8-bit proxy of the) luma -> CRF curve."""
        from ..rc.lookahead import GpuLookahead
        from ..rc.ratecontrol import crf_qps_batch

        if getattr(self, "_la", None) is None:
            self._la = GpuLookahead(self.dev, self.p.la_range)
        t0 = time.perf_counter()
        y8 = y
        if y.dtype != torch.uint8:
            y8 = (y >> (self.p.bit_depth - 8)).clamp_(0, 255).to(torch.uint8)
        lbw, lbh = GpuLookahead.block_grid(y.shape[3], y.shape[2])
        from ..rc.ratecontrol import MBTREE_STRENGTH, scenecut_flags
        # cutree needs the lookahead's block grid to be the coded 16x16 grid (no -s resize); the
        # 32-aligned coded height may add one 16-row below the lookahead's last row
        # Pieces shorter than 8 pictures give the propagation too little to offset cutree's
        # constant CRF compensation ((1 - qcomp) x 13.5 QP): they keep the plain CRF QPs.
        use_tree = self.p.cutree and lbw == self.wmb and lbh <= self.hmb and y.shape[1] >= 8
        self._cutree_rows = lbh
        if use_tree:
            costs_d, self._cutree = self._la.mbtree(y8.contiguous(), MBTREE_STRENGTH)
            costs = costs_d.cpu().numpy()
        else:
            costs = self._la.frame_costs(y8.contiguous()).cpu().numpy()
        self._scenecuts = scenecut_flags(costs, float(self.p.scenecut), keyint=self.p.keyint or None)
        q = crf_qps_batch(costs, float(self.p.crf), lbw * lbh, keyint=self.p.keyint or None,
                          scenecuts=self._scenecuts, mbtree=use_tree)
        self.stats["scenecuts"] = int(self._scenecuts.sum())
        self.timings["lookahead_s"] = self.timings.get("lookahead_s", 0.0) + time.perf_counter() - t0
        return q

    # ------------------------------------------------------------------ encode
    def encode(self, y: torch.Tensor, u: torch.Tensor, v: torch.Tensor, qps: np.ndarray | None = None,
               keep_recon: bool = False, metrics: bool = True, qp_delta=None, rate_fb=None) -> list[HevcSegmentResult]:
        """y: [B, F, h, w] (uint8, or uint16 holding bit_depth-bit samples), u/v half size.
        Every segment starts with an IDR picture; the others are P pictures
        (intra_only: IDR pictures only).

        ``rate_fb`` (:class:`~govideocompressor_amd.rc.ratecontrol.TwoPassFeedback`): pass-2
        rate feedback -- before every frame step the controller sees the bits of the pictures
        whose CABAC has finished and may re-solve the QPs of the frames not yet started."""
        B, F, h, w = y.shape
        if B != self.B or (w, h) != (self.p.width, self.p.height):
            raise ValueError(f"expected [{self.B}, F, {self.p.height}, {self.p.width}], got {list(y.shape)}")
        if y.device != self.dev:
            raise ValueError("inputs must live on the encoder's device")
        qi, qpp = self.p.frame_qps()
        self._scenecuts = None
        self._cutree = None
        if qps is None and self.p.crf is not None and self.p.lookahead and not self.p.intra_only:
            qps = self.crf_qps(y)
        cuts_h = self._scenecuts if self._scenecuts is not None else np.zeros((B, F), dtype=bool)
        cuts_d = torch.from_numpy(np.ascontiguousarray(cuts_h.T)).to(self.dev)  # [F, B]
        if qps is None:
            qps = np.array([[qi if t == 0 else qpp for t in range(F)] for _ in range(B)], dtype=np.int32)
        cfg = self.p.host_cfg()
        if self.p.wpp:  # spread the native threads over the B pictures of a step
            cfg["threads"] = max(1, min(32, self.entropy_threads // max(1, B)))
        qps = np.clip(np.asarray(qps, dtype=np.int32).reshape(B, F), 0, 51)
        if qp_delta is not None:
            from ..rc.abr import apply_delta
            qps = apply_delta(qps, qp_delta)
        if rate_fb is not None:
            qps = np.array(rate_fb.qps, dtype=np.int32).reshape(B, F)
        qps_d = torch.from_numpy(np.ascontiguousarray(qps.T)).to(self.dev)  # [F, B], one upload
        fb_known, fb_spent, fb_stage = 0, np.zeros((B, F)), []
        nals: list[list] = [[None] * F for _ in range(B)]
        futs = []
        pending: list[list] = [[], [], []]
        sse = []
        recon = [] if keep_recon else None
        t_gpu = t_host = t_blocked = 0.0
        cabac_s = [0.0]
        p = self._p
        s = self._stream()
        bd = self.p.bit_depth
        st = self.stage_timer
        gate_sum: list[torch.Tensor] = []
        for t in range(F):
            t0 = time.perf_counter()
            if rate_fb is not None and t > 0:
                # bits of the pictures whose CABAC jobs have finished (coding order prefix)
                while fb_known < len(futs) and futs[fb_known][1].done():
                    for b, nal in enumerate(futs[fb_known][1].result()):
                        fb_spent[b, fb_known] = 8 * len(nal)
                    fb_known += 1
                newq = np.asarray(rate_fb.update(fb_known, fb_spent, t), dtype=np.int32)
                if not np.array_equal(newq[:, t:], qps[:, t:]):
                    qps[:, t:] = newq[:, t:]
                    staged = torch.from_numpy(np.ascontiguousarray(qps[:, t:].T)).pin_memory()
                    qps_d[t:].copy_(staged, non_blocking=True)  # stream-ordered before frame t's read
                    fb_stage.append(staged)  # keep the pinned source alive until the encode ends
            idr = t == 0 or self.p.intra_only or (self.p.keyint > 0 and t % self.p.keyint == 0)
            self._prep(y, u, v, t, proxy=not idr)
            self.qp.copy_(qps_d[t])  # device-to-device: no host sync inside the frame loop
            # per-CTB QPs (AQ + cutree offsets of frame t); without them every CTB at the frame QP
            extra, estride, erows = 0, 0, 0
            if self._cutree is not None and self.p.adaptive_qp():
                ct = self._cutree
                extra, estride, erows = ct.data_ptr() + t * ct.shape[2] * 4, ct.shape[1] * ct.shape[2], self._cutree_rows
            with st("aq"):
                self.hip.hevc_aq(B, self.W, self.H, bd, p(self.src[0]), p(self.src[1]), p(self.src[2]), p(self.qp),
                                 float(self.p.aq_strength) if self.p.adaptive_qp() else 0.0, extra, estride, erows,
                                 p(self.ctb_qp), p(self.mb_aq), s)
            cur, ref = self.rec[t % 2], self.rec[(t + 1) % 2]
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
                    self.hip.hevc_intra(*intra_args, 1, 1, p(self.err), s, int(self.p.sdh))
            else:
                self.run.fill_(2)
                with st("me"):
                    self.hip.hevc_proxy8(p(ref[0]), p(self.ref8), ref[0].numel(), bd - 8, s)
                    self.hip.me(B, self.wmb, self.hmb, p(self.src8), p(self.ref8), p(self.prev_mv), p(self.mv),
                                p(self.me_cost), p(self.me_pred), p(self.me_intra), p(self.qp), self.p.me_range,
                                self.p.subpel, s, p(self.me_hp), p(self.mb_aq))
                with st("merge_refine"):
                    for it in range(int(self.p.merge_refine)):
                        a_, b_ = (self.mv, self.mv_tmp) if it % 2 == 0 else (self.mv_tmp, self.mv)
                        self.hip.hevc_merge_refine(B, self.wmb, self.hmb, p(self.src8), p(self.ref8), p(self.me_hp),
                                                   p(a_), p(b_), p(self.me_cost), p(self.prev_mv), p(self.qp),
                                                   p(self.mb_aq), s)
                    if int(self.p.merge_refine) % 2:
                        self.mv.copy_(self.mv_tmp)
                if cuts_h[:, t].any():  # scene cut: every CU of these slots goes intra
                    self.me_cost.masked_fill_(cuts_d[t][:, None], 1 << 26)
                with st("intra_analyze"):  # open-loop intra candidates where intra may still win
                    mask = p(self._intra_gate()) if self.p.intra_gate else 0
                    if mask:
                        gate_sum.append(self.ctb_need.sum(dtype=torch.int64))
                    self.hip.hevc_intra(*intra_args, 1, 0, p(self.err), s, int(self.p.sdh), mask)
                with st("inter"):
                    self.hip.hevc_inter(B, self.W, self.H, p(self.src[0]), p(self.src[1]), p(self.src[2]), p(ref[0]),
                                        p(ref[1]), p(ref[2]), p(cur[0]), p(cur[1]), p(cur[2]), p(self.ctu), p(self.cu),
                                        p(self.coef[0]), p(self.coef[1]), p(self.coef[2]), p(self.ctb_qp), p(self.run),
                                        p(self.cand), p(self.mv), p(self.me_cost), bd, s, int(self.p.tu_inter_depth),
                                        int(self.p.sdh), int(self.p.intra_bias_p))
                with st("intra_recon"):
                    self.hip.hevc_intra(*intra_args, 0, 1, p(self.err), s, int(self.p.sdh))   # intra CUs, wavefront
                self.prev_mv.copy_(self.mv)
            self.hip.hevc_qp_fixup(B, self.W, self.H, p(self.ctu), p(self.cu), p(self.qp), p(self.run), int(self.p.wpp), s)
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
                                      p(self.ctu), p(self.ctb_qp), p(self.run), 1, s)
                self.dbk = cur
                self.rec[t % 2] = cur = out_pl
            if metrics:
                d = (cur[0][:, :h, :w].to(torch.int32) - self.src[0][:, :h, :w].to(torch.int32))
                sse.append((d * d).sum(dim=(1, 2)).to(torch.float64))
            if keep_recon:
                recon.append(tuple(c.clone() for c in cur))
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
            host = self._host_buffers()[hb]
            nzmap, nzoff = self.nzmaps[kb], self.nzoffs[kb]
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

            fps = [dict(idr=int(idr), poc=t, qp=int(qps[b, t]), slice_type=2 if idr else 1) for b in range(B)]

            def job(done=done, fps=fps, ctu=ctu, cu=cu, nz=nz, off=off, lv=lv):
                done.synchronize()
                tj = time.perf_counter()
                r = self.host.hevc_write_slices_packed(cfg, fps, ctu, cu, nz, off, lv, self.entropy_threads)
                cabac_s[0] += time.perf_counter() - tj
                return r

            f = self.pool.submit(job)
            futs.append((t, f))
            pending[hb].append(f)
        self.last_qps = qps.copy()
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
        self.timings = dict(loop_s=t_gpu, loop_waits_on_step_t_minus_3_s=t_blocked, host_wait_s=t_host,
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
                                         bits=bits[b], psnr_y=ps))
        if keep_recon:
            self.last_recon = recon
        return out
