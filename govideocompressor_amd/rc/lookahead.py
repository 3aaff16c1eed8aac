"""GPU lookahead: lowres frame costs of B segments x F frames in one pass.

Reference behaviour replaced: the per-frame quantiser of libx264's CRF mode
(``-vcodec libx264`` -> CRF 23 default, server.go:67-71, run by the worker at
client.go:115) comes from x264's half-resolution lookahead.  Here the lookahead
is ``csrc/kernels/lookahead.hip``: a 2x2 downscale, an integer full search per
8x8 lowres block, DC/H/V intra candidates and the 8x8 Hadamard SATD of every
candidate as an int8 GEMM on the MFMA units.  Every frame of every slot is
independent work, so one launch covers the whole batch; the [B, F, 2] frame
costs feed :func:`~govideocompressor_amd.rc.ratecontrol.crf_qps_batch`.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import native

RANGES = (4, 6, 8)
INTRA_SHIFT = 40  # la_multi packs its intra block counts above the cost sums (lookahead.hip kLaIntraShift)


class GpuLookahead:
    """Lowres cost analysis on gfx950 (workspace cached across calls)."""

    def __init__(self, device: str | torch.device = "cuda", search_range: int = 6, hierarchical: bool = True,
                 weighted: bool = False, wt_min_mean: float = 2.0, wt_min_scale: float = 0.08):
        """``hierarchical``: search every lowres block around twice its quarter-resolution
        block's vector (a +-8 full search at quarter resolution, +-32 full-resolution pixels)
        instead of around zero -- fast pans, which the lowres window alone (+-2 * range
        pixels) cannot follow, would otherwise look like scene cuts.

        ``weighted``: lowres weighted prediction (x264 analyses weights in its lookahead):
        per (picture, reference distance) weights from the lowres planes' means and variances
        (w = sqrt(var_cur / var_ref), o = mean_cur - w * mean_ref, used when the mean moves by
        >= ``wt_min_mean`` levels or the contrast by >= ``wt_min_scale``); weighted P
        candidates are priced as the encoder's weighted prediction will code them, so fades
        stop looking like new content to the P / B placement, the CRF curve and MB-tree."""
        if search_range not in RANGES:
            raise ValueError(f"search_range must be one of {RANGES}")
        self.hierarchical = bool(hierarchical)
        self.dev = torch.device(device)
        if self.dev.type == "cuda" and self.dev.index is None:
            self.dev = torch.device("cuda", torch.cuda.current_device())
        self.range = int(search_range)
        self.weighted = bool(weighted)
        self.wt_min_mean, self.wt_min_scale = float(wt_min_mean), float(wt_min_scale)
        self.last_weights: torch.Tensor | None = None  # [B, F, 8, 2] (w, o) per distance, w = 0: none
        self.hip = native.hip()
        self._low: torch.Tensor | None = None
        self._cost: torch.Tensor | None = None

    @staticmethod
    def block_grid(width: int, height: int) -> tuple[int, int]:
        """(lowres 8x8 blocks per row, per column) = one per 16x16 macroblock."""
        return ((width // 2) + 7) // 8, ((height // 2) + 7) // 8

    def _workspace(self, w: int, h: int, n: int) -> tuple[torch.Tensor, torch.Tensor]:
        need = int(self.hip.lookahead_low_bytes(w, h, n))
        if self._low is None or self._low.numel() < need:
            self._low = torch.empty((need,), dtype=torch.uint8, device=self.dev)
        if self._cost is None or self._cost.shape[0] < n:
            self._cost = torch.empty((n, 2), dtype=torch.int64, device=self.dev)
        return self._low, self._cost[:n]

    @torch.no_grad()
    def mbtree(self, y: torch.Tensor, strength: float = 2.0):
        """Frame costs plus MB-tree QP offsets (csrc/kernels/mbtree.hip).

        Returns ([B, F, 2] int64 frame costs, [B, F, lbh * lbw] float32 per-MB QP offsets,
        one lowres 8x8 block per 16x16 MB), both on the device."""
        B, F, h, w = y.shape
        lbw, lbh = self.block_grid(w, h)
        costs, blk, mv = self.frame_costs(y, block_costs=True, block_mvs=True)
        self.last_blk, self.last_mv = blk, mv  # for multi_costs (b-adapt)
        n = B * F * lbw * lbh
        if getattr(self, "_prop", None) is None or self._prop.numel() < n:
            self._prop = torch.empty((n,), dtype=torch.int64, device=self.dev)  # fixed-point accumulators
        out = torch.empty((B, F, lbh * lbw), dtype=torch.float32, device=self.dev)
        self.hip.mbtree(B, F, lbw, lbh, blk.data_ptr(), mv.data_ptr(), self._prop.data_ptr(), float(strength),
                        out.data_ptr(), torch.cuda.current_stream(self.dev).cuda_stream)
        return costs, out

    @torch.no_grad()
    def frame_costs(self, y: torch.Tensor, block_costs: bool = False, block_mvs: bool = False):
        """y: [B, F, h, w] uint8 luma on the device (the encoder's input layout).

        Returns a device tensor [B, F, 2] int64 = (sum of intra costs, sum of
        min(intra, inter) costs) per frame (the first frame of a segment is intra
        only), and with ``block_costs`` also [B, F, 2, lbh, lbw] int32 per-block costs
        (and with ``block_mvs`` [B, F, lbh, lbw] int32 packed lowres vectors, dx | dy << 16).
        """
        if y.dtype != torch.uint8 or y.dim() != 4 or y.device != self.dev:
            raise ValueError("y must be a uint8 [B, F, h, w] tensor on the lookahead's device")
        if y.stride(3) != 1 or y.stride(2) != y.shape[3] or y.stride(0) != y.shape[1] * y.stride(1):
            raise ValueError("y frames must be dense rows with slot-major frame order")
        B, F, h, w = y.shape
        if h % 2 or w % 2 or h < 16 or w < 16:
            raise ValueError("frame size must be even and at least 16x16")
        n = B * F
        low, cost = self._workspace(w, h, n)
        blk = mv = None
        lbw, lbh = self.block_grid(w, h)
        if block_costs:
            blk = torch.zeros((B, F, 2, lbh, lbw), dtype=torch.int32, device=self.dev)
        if block_mvs:
            mv = torch.zeros((B, F, lbh, lbw), dtype=torch.int32, device=self.dev)
        low4 = mv4 = cost4 = 0
        if self.hierarchical and w >= 64 and h >= 64:
            qbytes = int(self.hip.lookahead_quarter_bytes(w, h, n))
            qbw, qbh = ((((w >> 1) & ~1) >> 1) + 7) // 8, ((((h >> 1) & ~1) >> 1) + 7) // 8
            if getattr(self, "_low4", None) is None or self._low4.numel() < qbytes:
                self._low4 = torch.empty((qbytes,), dtype=torch.uint8, device=self.dev)
            if getattr(self, "_mv4", None) is None or self._mv4.numel() < n * qbw * qbh:
                self._mv4 = torch.empty((n * qbw * qbh,), dtype=torch.int32, device=self.dev)
                self._cost4 = torch.empty((n, 2), dtype=torch.int64, device=self.dev)
            low4, mv4, cost4 = self._low4.data_ptr(), self._mv4.data_ptr(), self._cost4.data_ptr()
        args = (y.data_ptr(), w, h, y.stride(1), n, F, low.data_ptr(), cost.data_ptr(),
                blk.data_ptr() if blk is not None else 0, self.range, torch.cuda.current_stream(self.dev).cuda_stream,
                mv.data_ptr() if mv is not None else 0, low4, mv4, cost4)
        self._any_weighted = False
        if self.weighted:
            # planes and weights first; the weighted cost kernels (more registers) only when some
            # picture is weighted -- steady content runs the plain ones (one host sync, on the
            # lookahead's own stream / thread)
            self._wt = torch.empty((B, F, 8, 2), dtype=torch.float32, device=self.dev)
            self._wst = torch.empty((n, 2), dtype=torch.int64, device=self.dev)
            self.last_weights = self._wt
            self.hip.lookahead(*args, self._wt.data_ptr(), self._wst.data_ptr(), self.wt_min_mean, self.wt_min_scale, 1)
            self._any_weighted = bool((self._wt[..., 0] > 0).any().item())
            self.hip.lookahead(*args, self._wt.data_ptr() if self._any_weighted else 0, 0, self.wt_min_mean,
                               self.wt_min_scale, 2)
        else:
            self.hip.lookahead(*args, 0, 0, self.wt_min_mean, self.wt_min_scale, 3)
        out = cost.view(B, F, 2)
        if block_mvs:
            return out, blk, mv
        return (out, blk) if block_costs else out


    @torch.no_grad()
    def multi_costs(self, y: torch.Tensor, blk: torch.Tensor, mv: torch.Tensor, max_dist: int,
                    search_range: int = 2) -> torch.Tensor:
        """x264 --b-adapt costs (lookahead.hip la_multi) of the batch whose lowres planes, block
        costs and distance-1 vectors the last :meth:`frame_costs` call produced: [B, F, 8] int64,
        column d = 2..max_dist the P cost at distance d, column 0 the B cost between the
        neighbours (frame sums of min(intra, candidate)).  The number of lowres blocks that
        chose intra in each (x264's ``i_intra_mbs``, the b-adapt guards) is left in
        ``self.last_multi_intra`` ([B, F, 8] int64, same columns)."""
        B, F, h, w = y.shape
        if self._low is None or blk is None or mv is None:
            raise ValueError("multi_costs needs a preceding frame_costs(block_costs=True, block_mvs=True)")
        if not 2 <= int(max_dist) <= 7:
            raise ValueError("max_dist in 2..7 (bframes 1..6)")
        out = torch.empty((B * F, 8), dtype=torch.int64, device=self.dev)
        wt = self._wt.data_ptr() if (self.weighted and getattr(self, "_any_weighted", False)
                                     and self._wt.shape[:2] == (B, F)) else 0
        self.hip.lookahead_multi(self._low.data_ptr(), w, h, B * F, F, blk.data_ptr(), mv.data_ptr(), int(max_dist),
                                 int(search_range), out.data_ptr(), torch.cuda.current_stream(self.dev).cuda_stream,
                                 wt)
        out = out.view(B, F, 8)
        self.last_multi_intra = out >> INTRA_SHIFT
        return out & ((1 << INTRA_SHIFT) - 1)


def lowres_weights(y: np.ndarray, min_mean: float = 2.0, min_scale: float = 0.08) -> np.ndarray:
    """numpy model of la_stats / la_weights: [B, F, 8, 2] float32 (w, o) of every picture
    against the picture d back (column d = 1..7, within the segment); w = 0: not weighted."""
    B, F, h, w = y.shape
    lw, lh = w // 2, h // 2
    yy = y.astype(np.int64)
    s = (yy[..., 0::2, 0::2][..., :lh, :lw] + yy[..., 0::2, 1::2][..., :lh, :lw] +
         yy[..., 1::2, 0::2][..., :lh, :lw] + yy[..., 1::2, 1::2][..., :lh, :lw] + 2) >> 2
    cnt = float(lw * lh)
    mean = s.sum(axis=(2, 3)).astype(np.float64) / cnt
    var = np.maximum((s * s).sum(axis=(2, 3)).astype(np.float64) / cnt - mean * mean, 0.0)
    out = np.zeros((B, F, 8, 2), np.float32)
    for b in range(B):
        for f in range(F):
            for d in range(1, min(8, f + 1)):
                mc, mr, vc, vr = mean[b, f], mean[b, f - d], var[b, f], var[b, f - d]
                wv = np.sqrt(vc / vr) if vr > 1e-3 else 1.0
                if (abs(mc - mr) >= min_mean or abs(wv - 1.0) >= min_scale) and wv > 1.0 / 64:
                    out[b, f, d] = (np.float32(wv), np.float32(mc - wv * mr))
    return out


def _inv_weight(S: np.ndarray, wv: np.float32, o: np.float32) -> np.ndarray:
    """la_inv_weight4: clamp(rint((s - o) * (1 / w)), 0, 255) in float32."""
    inv = np.float32(1.0) / wv
    v = (S.astype(np.float32) - o) * inv
    return np.clip(np.rint(v), 0, 255).astype(np.int64)


def lookahead_reference(y: np.ndarray, search_range: int = 6, weights: np.ndarray | None = None
                        ) -> tuple[np.ndarray, np.ndarray]:
    """Plain numpy model of ``lookahead.hip`` (the numerics-test oracle).

    y: [B, F, h, w] uint8.  Returns (frame costs [B, F, 2] int64, block costs
    [B, F, 2, lbh, lbw] int64).  SATD = (sum |H64 . vec(S - P)| + 2) >> 2 with
    H64[i, k] = (-1)^popcount(i & k) and vec index k = 8 * row + col.  ``weights``
    (:func:`lowres_weights`): the weighted inter cost -- search and SATD on the inverse-weighted
    source, SATD scaled back by w.
    """
    B, F, h, w = y.shape
    R, pad = search_range, 16
    lw, lh = w // 2, h // 2
    lbw, lbh = (lw + 7) // 8, (lh + 7) // 8
    ls, lr = lbw * 8 + 2 * pad, lbh * 8 + 2 * pad
    px = np.clip(np.arange(ls) - pad, 0, lw - 1)
    py = np.clip(np.arange(lr) - pad, 0, lh - 1)
    yy = y.astype(np.int64)
    s = (yy[..., 0::2, 0::2][..., :lh, :lw] + yy[..., 0::2, 1::2][..., :lh, :lw] +
         yy[..., 1::2, 0::2][..., :lh, :lw] + yy[..., 1::2, 1::2][..., :lh, :lw] + 2) >> 2
    low = s[..., py, :][..., :, px]  # [B, F, lr, ls]
    idx = np.arange(64)
    pc = np.vectorize(lambda v: bin(v).count("1"))(idx[:, None] & idx[None, :])
    H = np.where(pc % 2 == 1, -1, 1).astype(np.int64)

    def satd(res: np.ndarray) -> int:
        return int((np.abs(H @ res.reshape(64)).sum() + 2) >> 2)

    blk = np.zeros((B, F, 2, lbh, lbw), dtype=np.int64)
    side = 2 * R + 1
    for b in range(B):
        for f in range(F):
            cur = low[b, f]
            ref = low[b, f - 1] if f > 0 else None
            for by in range(lbh):
                for bx in range(lbw):
                    X0, Y0 = pad + 8 * bx, pad + 8 * by
                    S = cur[Y0:Y0 + 8, X0:X0 + 8]
                    top = cur[Y0 - 1, X0:X0 + 8]
                    left = cur[Y0:Y0 + 8, X0 - 1]
                    dc = (int(top.sum()) + int(left.sum()) + 8) >> 4
                    intra = min(satd(S - dc), satd(S - left[:, None]), satd(S - top[None, :])) + 5
                    inter = intra
                    if ref is not None:
                        wv = weights[b, f, 1, 0] if weights is not None else np.float32(0)
                        Sw = _inv_weight(S, wv, weights[b, f, 1, 1]) if wv > 0 else S
                        best = None
                        for dy in range(-R, R + 1):
                            for dx in range(-R, R + 1):
                                P = ref[Y0 + dy:Y0 + dy + 8, X0 + dx:X0 + dx + 8]
                                key = (int(np.abs(Sw - P).sum()) + 2 * (abs(dx) + abs(dy)), (dy + R) * side + dx + R)
                                if best is None or key < best[0]:
                                    best = (key, dx, dy)
                        _, mdx, mdy = best
                        P = ref[Y0 + mdy:Y0 + mdy + 8, X0 + mdx:X0 + mdx + 8]
                        sv = satd(Sw - P)
                        if wv > 0:
                            sv = int(np.rint(np.float32(wv) * np.float32(sv)))
                        inter = sv + 2 * (abs(mdx) + abs(mdy))
                    blk[b, f, 0, by, bx] = intra
                    blk[b, f, 1, by, bx] = inter
    frame = np.stack([blk[:, :, 0].sum(axis=(2, 3)), np.minimum(blk[:, :, 0], blk[:, :, 1]).sum(axis=(2, 3))], axis=-1)
    return frame, blk


def multi_reference(y: np.ndarray, search_range: int = 6, max_dist: int = 4, multi_range: int = 2,
                    with_intra: bool = False):
    """Plain numpy model of ``la_multi`` (lookahead.hip): [B, F, 8] int64, column d = 2..max_dist
    the P cost at distance d, column 0 the B cost between the neighbours (frame sums of
    min(intra, candidate) over the lowres 8x8 blocks), from the same lowres planes, intra costs
    and distance-1 vectors as :func:`lookahead_reference`.  with_intra: also the intra block
    counts of each (``GpuLookahead.last_multi_intra``), returned as a second array."""
    B, F, h, w = y.shape
    R, pad, MR = search_range, 16, multi_range
    lw, lh = w // 2, h // 2
    lbw, lbh = (lw + 7) // 8, (lh + 7) // 8
    ls, lr = lbw * 8 + 2 * pad, lbh * 8 + 2 * pad
    px = np.clip(np.arange(ls) - pad, 0, lw - 1)
    py = np.clip(np.arange(lr) - pad, 0, lh - 1)
    yy = y.astype(np.int64)
    s = (yy[..., 0::2, 0::2][..., :lh, :lw] + yy[..., 0::2, 1::2][..., :lh, :lw] +
         yy[..., 1::2, 0::2][..., :lh, :lw] + yy[..., 1::2, 1::2][..., :lh, :lw] + 2) >> 2
    low = s[..., py, :][..., :, px]
    idx = np.arange(64)
    pc = np.vectorize(lambda v: bin(v).count("1"))(idx[:, None] & idx[None, :])
    Hm = np.where(pc % 2 == 1, -1, 1).astype(np.int64)

    def satd(res: np.ndarray) -> int:
        return int((np.abs(Hm @ res.reshape(64)).sum() + 2) >> 2)

    def search(ref, S, X0, Y0, cx, cy, r):
        side = 2 * r + 1
        cx = min(max(cx, r - X0), ls - 28 - X0 + r)
        cy = min(max(cy, r - Y0), lr - 8 - r - Y0)
        best = None
        for dy in range(-r, r + 1):
            for dx in range(-r, r + 1):
                P = ref[Y0 + cy + dy:Y0 + cy + dy + 8, X0 + cx + dx:X0 + cx + dx + 8]
                key = (int(np.abs(S - P).sum()) + 2 * (abs(dx) + abs(dy)), (dy + r) * side + dx + r)
                if best is None or key < best[0]:
                    best = (key, cx + dx, cy + dy)
        return best[1], best[2]

    _, blk = lookahead_reference(y, search_range)
    out = np.zeros((B, F, 8), dtype=np.int64)
    cnt = np.zeros((B, F, 8), dtype=np.int64)
    for b in range(B):
        for f in range(1, F):
            cur = low[b, f]
            for by in range(lbh):
                for bx in range(lbw):
                    X0, Y0 = pad + 8 * bx, pad + 8 * by
                    S = cur[Y0:Y0 + 8, X0:X0 + 8]
                    intra, inter1 = int(blk[b, f, 0, by, bx]), int(blk[b, f, 1, by, bx])
                    # the distance-1 vector of la_cost (same search and tie-break)
                    ref1 = low[b, f - 1]
                    v1 = None
                    side = 2 * R + 1
                    for dy in range(-R, R + 1):
                        for dx in range(-R, R + 1):
                            P = ref1[Y0 + dy:Y0 + dy + 8, X0 + dx:X0 + dx + 8]
                            key = (int(np.abs(S - P).sum()) + 2 * (abs(dx) + abs(dy)), (dy + R) * side + dx + R)
                            if v1 is None or key < v1[0]:
                                v1 = (key, dx, dy)
                    vx, vy = v1[1], v1[2]
                    for d in range(2, min(max_dist, f) + 1):
                        ref = low[b, f - d]
                        mx, my = search(ref, S, X0, Y0, d * vx, d * vy, MR)
                        P = ref[Y0 + my:Y0 + my + 8, X0 + mx:X0 + mx + 8]
                        cst = satd(S - P) + 2 * (abs(mx - d * vx) + abs(my - d * vy)) + 2 * (abs(vx) + abs(vy))
                        out[b, f, d] += min(intra, cst)
                        cnt[b, f, d] += intra < cst
                    if f + 1 < F:
                        r1 = low[b, f + 1]
                        mx, my = search(r1, S, X0, Y0, -vx, -vy, MR)
                        P1 = r1[Y0 + my:Y0 + my + 8, X0 + mx:X0 + mx + 8]
                        c1 = satd(S - P1) + 2 * (abs(mx) + abs(my))
                        cx0, cy0 = min(max(vx, -8), 8), min(max(vy, -8), 8)
                        P0 = ref1[Y0 + cy0:Y0 + cy0 + 8, X0 + cx0:X0 + cx0 + 8]
                        Pb = (P0 + P1 + 1) >> 1
                        cbi = satd(S - Pb) + 2 * (abs(mx) + abs(my) + abs(vx) + abs(vy))
                        out[b, f, 0] += min(min(intra, inter1), min(c1, cbi))
                        cnt[b, f, 0] += intra < min(inter1, c1, cbi)
    return (out, cnt) if with_intra else out
