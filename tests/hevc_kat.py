"""Known-answer HEVC streams for tests/test_hevc_kat.py, written without any of the codec's
own C++ (csrc/host/hevc_dec*.cc, hevc_writer.cc, hevc_exerciser.cc and its context tables).

Pieces, all typed from ITU-T H.265 here:

* a bit writer with ue(v) / se(v) and NAL emulation prevention (7.3.1, 7.4.2);
* the CABAC encoder of 9.3.4 (EncodeDecision / EncodeBypass / EncodeTerminate / EncodeFlush,
  context initialisation 9.3.2.2) and the init values of the few contexts these streams use
  (Tables 9-5 .. 9-37).  Only the arithmetic coder's rangeTabLPS / transIdxLPS -- the same
  constants in H.264 and H.265 -- are read from csrc/common/h264_cabac_tables.h;
* VPS / SPS / PPS / slice-header syntax (7.3.2 .. 7.3.6) including st_ref_pic_set,
  pred_weight_table and scaling_list_data;
* slice data for the constructions the tests need: I pictures made of PCM CUs (exactly known
  samples), P pictures of skip CUs, 2Nx2N AMVP CUs (the first CU's AMVP list is all zero, so
  its motion is the coded mvd), asymmetric partitions with an AMVP PU and a merge PU, and
  2Nx2N CUs carrying one DC coefficient per transform block.

The expected pictures are computed in the tests from the clause formulas, so a misreading of
8.5 / 8.6 shared by the decoder and the repo's writers fails there.
"""
from __future__ import annotations

import os
import re

_HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc", "common",
                    "h264_cabac_tables.h")


def _arith_tables():
    txt = open(_HDR).read()
    rng = re.search(r"kCabacRangeLPS\[64\]\[4\]\s*=\s*\{(.*?)\};", txt, re.S).group(1)
    vals = [int(x) for x in re.findall(r"\d+", rng)]
    trans = re.search(r"kCabacTransLPS\[64\]\s*=\s*\{(.*?)\};", txt, re.S).group(1)
    tl = [int(x) for x in re.findall(r"\d+", trans)]
    assert len(vals) == 256 and len(tl) == 64
    return [vals[4 * i:4 * i + 4] for i in range(64)], tl


RANGE_LPS, TRANS_LPS = _arith_tables()

# initValue per context, Tables 9-5 .. 9-37; key -> {initType: [values by ctxInc]}
# (initType 0 = I slices, 1 = P slices without cabac_init_flag)
INIT = {
    "split_cu_flag": {0: [139, 141, 157], 1: [107, 139, 126]},
    "cu_skip_flag": {1: [197, 185, 201]},
    "pred_mode_flag": {1: [149]},
    "part_mode": {0: [184], 1: [154, 139, 154, 154]},
    "merge_flag": {1: [110]},
    "merge_idx": {1: [122]},
    "mvp_flag": {1: [168]},
    "rqt_root_cbf": {1: [79]},
    "abs_mvd_greater0": {1: [140]},
    "abs_mvd_greater1": {1: [198]},
    "cbf_luma": {1: [153, 111]},
    "cbf_chroma": {1: [149, 107, 167, 154]},
    "last_x_prefix": {1: [125, 110, 94, 110, 95, 79, 125, 111, 110, 78, 110, 111, 111, 95, 94, 108, 123, 108]},
    "last_y_prefix": {1: [125, 110, 94, 110, 95, 79, 125, 111, 110, 78, 110, 111, 111, 95, 94, 108, 123, 108]},
    "greater1": {1: [154, 196, 196, 167, 154, 152, 167, 182, 182, 134, 149, 136, 153, 121, 136, 137, 169, 194,
                     166, 167, 154, 167, 137, 182]},
    "greater2": {1: [107, 167, 91, 122, 107, 167]},
}

# Table 7-6: default 8x8 scaling lists (up-right diagonal order), intra (matrixId 0..2), inter (3..5)
DEFAULT_8x8_INTRA = [16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 17, 16, 17, 16, 17, 18, 17, 18, 18, 17, 18, 21, 19, 20,
                     21, 20, 19, 21, 24, 22, 22, 24, 24, 22, 22, 24, 25, 25, 27, 30, 27, 25, 25, 29, 31, 35, 35, 31,
                     29, 36, 41, 44, 41, 36, 47, 54, 54, 47, 65, 70, 65, 88, 88, 115]
DEFAULT_8x8_INTER = [16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 17, 17, 17, 17, 17, 18, 18, 18, 18, 18, 18, 20, 20, 20,
                     20, 20, 20, 20, 24, 24, 24, 24, 24, 24, 24, 24, 25, 25, 25, 25, 25, 25, 25, 28, 28, 28, 28, 28,
                     28, 33, 33, 33, 33, 33, 41, 41, 41, 41, 54, 54, 54, 71, 71, 91]


class Bits:
    def __init__(self):
        self.b: list[int] = []
        self.ue_sites: list[int] = []   # bit index of every ue(v) / se(v) code (for the range tests)

    def u(self, v: int, n: int):
        for k in range(n - 1, -1, -1):
            self.b.append((v >> k) & 1)

    def ue(self, v: int):
        self.ue_sites.append(len(self.b))
        v += 1
        n = v.bit_length()
        self.u(0, n - 1)
        self.u(v, n)

    def se(self, v: int):
        self.ue(2 * v - 1 if v > 0 else -2 * v)

    def with_ue(self, site: int, value: int) -> "Bits":
        """A copy whose ``site``-th Exp-Golomb code carries ``value`` instead (any size up to
        2^33 - 2, i.e. up to 32 leading zeros): the rest of the bits follow unchanged."""
        start = self.ue_sites[site]
        lz = 0
        while self.b[start + lz] == 0:
            lz += 1
        out = Bits()
        out.b = self.b[:start]
        v = value + 1
        n = v.bit_length()
        out.u(0, n - 1)
        out.u(v, n)
        out.b += self.b[start + 2 * lz + 1:]
        out.align_zero()
        return out

    def align_zero(self):
        while len(self.b) % 8:
            self.b.append(0)

    def trailing(self):
        self.b.append(1)
        self.align_zero()

    def bytes(self) -> bytes:
        assert len(self.b) % 8 == 0
        return bytes(int("".join(map(str, self.b[i:i + 8])), 2) for i in range(0, len(self.b), 8))


def nal(ntype: int, rbsp: bytes) -> bytes:
    out = bytearray(b"\x00\x00\x00\x01")
    out += bytes([(ntype << 1) & 0x7E, 1])
    zeros = 0
    for x in rbsp:
        if zeros >= 2 and x <= 3:
            out.append(3)
            zeros = 0
        out.append(x)
        zeros = zeros + 1 if x == 0 else 0
    return bytes(out)


class Cabac:
    """9.3.4 encoder side, writing into a Bits."""

    def __init__(self, bits: Bits, qp: int, init_type: int):
        self.w = bits
        self.ctx: dict[str, list[list[int]]] = {}
        for k, t in INIT.items():
            if init_type in t:
                self.ctx[k] = [self._init(v, qp) for v in t[init_type]]
        self.start()

    @staticmethod
    def _init(v: int, qp: int) -> list[int]:
        m, n = (v >> 4) * 5 - 45, ((v & 15) << 3) - 16
        pre = min(max(((m * min(max(qp, 0), 51)) >> 4) + n, 1), 126)
        return [pre - 64, 1] if pre > 63 else [63 - pre, 0]

    def start(self):
        self.low, self.range, self.first, self.outstanding = 0, 510, True, 0

    def _put(self, b: int):
        if self.first:
            self.first = False
        else:
            self.w.b.append(b)
        while self.outstanding:
            self.w.b.append(1 - b)
            self.outstanding -= 1

    def _renorm(self):
        while self.range < 256:
            if self.low < 256:
                self._put(0)
            elif self.low >= 512:
                self.low -= 512
                self._put(1)
            else:
                self.low -= 256
                self.outstanding += 1
            self.range <<= 1
            self.low <<= 1

    def bin(self, name: str, inc: int, b: int):
        st = self.ctx[name][inc]
        lps = RANGE_LPS[st[0]][(self.range >> 6) & 3]
        self.range -= lps
        if b != st[1]:
            self.low += self.range
            self.range = lps
            if st[0] == 0:
                st[1] = 1 - st[1]
            st[0] = TRANS_LPS[st[0]]
        else:
            st[0] = min(st[0] + 1, 62)
        self._renorm()

    def bypass(self, b: int):
        self.low <<= 1
        if b:
            self.low += self.range
        if self.low >= 1024:
            self._put(1)
            self.low -= 1024
        elif self.low < 512:
            self._put(0)
        else:
            self.low -= 512
            self.outstanding += 1

    def bypass_bits(self, v: int, n: int):
        for k in range(n - 1, -1, -1):
            self.bypass((v >> k) & 1)

    def terminate(self, b: int):
        self.range -= 2
        if b:
            self.low += self.range
            self.range = 2
            self._renorm()
            self._put((self.low >> 9) & 1)
            self.w.u(((self.low >> 7) & 3) | 1, 2)
        else:
            self._renorm()

    def eg(self, v: int, k: int):
        """k-th order Exp-Golomb bypass bins (9.3.3.5)."""
        while True:
            if v >= (1 << k):
                self.bypass(1)
                v -= 1 << k
                k += 1
            else:
                self.bypass(0)
                while k:
                    k -= 1
                    self.bypass((v >> k) & 1)
                return


def _ptl(b: Bits, bit_depth: int):
    b.u(0, 2)
    b.u(0, 1)
    prof = 1 if bit_depth == 8 else 2
    b.u(prof, 5)
    b.u((1 << (31 - prof)) | (1 << 29 if prof == 1 else 0), 32)
    b.u(0b1001, 4)  # progressive, not interlaced, not non-packed, frame only
    b.u(0, 43)
    b.u(0, 1)
    b.u(93, 8)  # level 3.1


def _scaling_data(b: Bits, lists: dict):
    """lists: (sizeId, matrixId) -> (coefs in diagonal order, dc or None); others default."""
    for size in range(4):
        for mid in range(0, 6, 3 if size == 3 else 1):
            if (size, mid) not in lists:
                b.u(0, 1)   # scaling_list_pred_mode_flag: predicted ...
                b.ue(0)     # ... from the default list
                continue
            coefs, dc = lists[(size, mid)]
            b.u(1, 1)
            nxt = 8
            if size > 1:
                b.se(dc - 8)
                nxt = dc
            assert len(coefs) == min(64, 1 << (4 + 2 * size))
            for c in coefs:
                d = (c - nxt) % 256
                d = d - 256 if d > 127 else d
                b.se(d)
                nxt = c


class KatStream:
    """One coded video sequence: an IDR of PCM CUs, then P pictures built CTU by CTU."""

    def __init__(self, w: int, h: int, bit_depth: int = 8, ctb_log2: int = 4, max_tb_log2: int | None = None,
                 weighted: bool = False, scaling: dict | None = None, max_merge: int = 1, sps_st_rps: int = 0):
        self.w, self.h, self.bd, self.ctb = w, h, bit_depth, ctb_log2
        self.max_tb = max_tb_log2 if max_tb_log2 is not None else min(5, ctb_log2)
        self.weighted, self.scaling, self.max_merge = weighted, scaling, max_merge
        self.sps_st_rps = sps_st_rps
        assert w % (1 << ctb_log2) == 0 and h % (1 << ctb_log2) == 0
        self.out = bytearray()
        self.units: list[tuple[int, Bits]] = []
        self._params()

    def _emit(self, ntype: int, b: Bits):
        self.units.append((ntype, b))
        self.out += nal(ntype, b.bytes())

    def ue_sites(self) -> list[tuple[int, int]]:
        """(unit, site) of every Exp-Golomb code written so far."""
        return [(k, j) for k, (_, b) in enumerate(self.units) for j in range(len(b.ue_sites))]

    def with_ue(self, unit: int, site: int, value: int) -> bytes:
        """The stream with one Exp-Golomb code replaced (parser range / wrap tests)."""
        out = bytearray()
        for k, (t, b) in enumerate(self.units):
            out += nal(t, (b.with_ue(site, value) if k == unit else b).bytes())
        return bytes(out)

    # ------------------------------------------------------------ parameter sets
    def _params(self):
        b = Bits()
        b.u(0, 4)
        b.u(3, 2)
        b.u(0, 6)
        b.u(0, 3)
        b.u(1, 1)
        b.u(0xFFFF, 16)
        _ptl(b, self.bd)
        b.u(1, 1)
        b.ue(4)
        b.ue(0)
        b.ue(0)
        b.u(0, 6)
        b.ue(0)
        b.u(0, 1)
        b.u(0, 1)
        b.trailing()
        self._emit(32, b)

        b = Bits()
        b.u(0, 4)
        b.u(0, 3)
        b.u(1, 1)
        _ptl(b, self.bd)
        b.ue(0)            # sps id
        b.ue(1)            # 4:2:0
        b.ue(self.w)
        b.ue(self.h)
        b.u(0, 1)          # conformance window
        b.ue(self.bd - 8)
        b.ue(self.bd - 8)
        b.ue(4)            # log2_max_pic_order_cnt_lsb_minus4: 8-bit POC lsb
        b.u(1, 1)
        b.ue(4)
        b.ue(0)
        b.ue(0)
        b.ue(0)            # min CB 8
        b.ue(self.ctb - 3)
        b.ue(0)            # min TB 4
        b.ue(self.max_tb - 2)
        b.ue(0)            # max_transform_hierarchy_depth_inter
        b.ue(0)            # ... intra
        b.u(1 if self.scaling is not None else 0, 1)
        if self.scaling is not None:
            b.u(1, 1)      # sps_scaling_list_data_present_flag
            _scaling_data(b, self.scaling)
        b.u(1, 1)          # amp_enabled_flag
        b.u(0, 1)          # SAO off
        b.u(1, 1)          # pcm_enabled_flag
        b.u(self.bd - 1, 4)
        b.u(self.bd - 1, 4)
        b.ue(0)            # min PCM CB 8
        b.ue(min(self.ctb, 5) - 3)
        b.u(1, 1)          # pcm_loop_filter_disabled_flag
        # num_short_term_ref_pic_sets (0: every RPS in the slice header); SPS sets are {-1}
        b.ue(self.sps_st_rps)
        for i in range(self.sps_st_rps):
            if i:
                b.u(0, 1)  # inter_ref_pic_set_prediction_flag
            b.ue(1)
            b.ue(0)
            b.ue(0)
            b.u(1, 1)
        b.u(0, 1)          # long_term_ref_pics_present_flag
        b.u(1, 1)          # sps_temporal_mvp_enabled_flag
        b.u(0, 1)          # strong intra smoothing
        b.u(0, 1)          # vui
        b.u(0, 1)          # extensions
        b.trailing()
        self._emit(33, b)

        b = Bits()
        b.ue(0)
        b.ue(0)
        b.u(0, 1)          # dependent slices
        b.u(0, 1)          # output_flag_present
        b.u(0, 3)
        b.u(0, 1)          # sign hiding
        b.u(0, 1)          # cabac_init_present
        b.ue(0)
        b.ue(0)
        b.se(0)            # init_qp 26
        b.u(0, 1)          # constrained intra
        b.u(0, 1)          # transform skip
        b.u(0, 1)          # cu_qp_delta
        b.se(0)
        b.se(0)
        b.u(0, 1)
        b.u(1 if self.weighted else 0, 1)
        b.u(0, 1)          # weighted bipred
        b.u(0, 1)          # transquant bypass
        b.u(0, 1)          # tiles
        b.u(0, 1)          # WPP
        b.u(0, 1)          # loop filter across slices
        b.u(1, 1)          # deblocking_filter_control_present_flag
        b.u(0, 1)          # override enabled
        b.u(1, 1)          # pps_deblocking_filter_disabled_flag
        b.u(0, 1)          # pps scaling lists
        b.u(0, 1)          # lists modification
        b.ue(0)
        b.u(0, 1)
        b.u(0, 1)
        b.trailing()
        self._emit(34, b)

    # ------------------------------------------------------------ pictures
    def idr_pcm(self, y, u, v, qp: int = 26):
        """IDR picture, every CTU one PCM CU of CTB size: decodes to exactly (y, u, v)."""
        b = Bits()
        b.u(1, 1)
        b.u(0, 1)          # no_output_of_prior_pics_flag
        b.ue(0)
        b.ue(2)            # I
        b.se(qp - 26)
        b.trailing()       # byte_alignment()
        c = Cabac(b, qp, 0)
        n = 1 << self.ctb
        ctus = [(x, yy) for yy in range(0, self.h, n) for x in range(0, self.w, n)]
        # PCM CUs are at most 32x32: a 64x64 CTB splits once (CtDepth 1 everywhere, so the
        # depth-0 split flag's ctxInc counts the available left / above CTBs, 9.3.4.2.2)
        pn = min(n, 32)
        for k, (x0, y0) in enumerate(ctus):
            if pn < n:
                c.bin("split_cu_flag", int(x0 > 0) + int(y0 > 0), 1)
            for cy in range(y0, y0 + n, pn):
                for cx in range(x0, x0 + n, pn):
                    c.bin("split_cu_flag", 0, 0)
                    c.terminate(1)     # pcm_flag
                    b.align_zero()     # pcm_alignment_zero_bit
                    for yy in range(cy, cy + pn):
                        for xx in range(cx, cx + pn):
                            b.u(int(y[yy, xx]), self.bd)
                    for pl in (u, v):
                        for yy in range(cy // 2, (cy + pn) // 2):
                            for xx in range(cx // 2, (cx + pn) // 2):
                                b.u(int(pl[yy, xx]), self.bd)
                    c.start()
            c.terminate(1 if k == len(ctus) - 1 else 0)  # end_of_slice_segment_flag
        b.align_zero()
        self._emit(19, b)

    def p_picture(self, poc: int, refs: list[int], cus: list[dict], tmvp: bool = False, qp: int = 26,
                  wp: dict | None = None, nref: int | None = None, inter_rps: bool = False):
        """TRAIL_R P picture.  ``refs``: POCs of the RPS (all used by the current picture, the
        first is RefPicList0[0]; ordered by decreasing POC as 8.3.2 builds StCurrBefore);
        ``cus``: one dict per CTU in raster order, each one CU of CTB size:

        * ``{"skip": True}``                              -- merge candidate 0;
        * ``{"mvd": (x, y)}``                             -- 2Nx2N AMVP PU;
        * ``{"part": "nLx2N", "pus": [("mvd", (x, y)), ("merge",)]}`` -- AMP / symmetric parts;
        * ``{"mvd": (x, y), "dc": [level per TB]}``       -- plus one DC coefficient per luma TB.

        ``wp``: {"denom", "w", "o", "cdenom_delta", "cw": [(w, o)] * 2} (delta-coded by the
        writer the way pred_weight_table codes them) or None.  ``nref``: code
        num_ref_idx_l0_active_minus1 (skip CUs only when > 1: no ref_idx is written).
        ``inter_rps``: predict the slice RPS from the last SPS set (needs ``sps_st_rps`` >= 1;
        delta_rps -1 on the set {-1}: gives {-1, -2})."""
        b = Bits()
        b.u(1, 1)
        b.ue(0)
        b.ue(1)            # P
        b.u(poc & 255, 8)
        b.u(0, 1)          # short_term_ref_pic_set_sps_flag
        assert all(r < poc for r in refs) and refs == sorted(refs, reverse=True)
        if inter_rps:
            assert self.sps_st_rps and refs == [poc - 1, poc - 2]
            b.u(1, 1)      # inter_ref_pic_set_prediction_flag
            b.ue(0)        # delta_idx_minus1
            b.u(1, 1)      # delta_rps_sign: negative
            b.ue(0)        # abs_delta_rps_minus1
            b.u(1, 1)      # used_by_curr_pic_flag[0]
            b.u(1, 1)      # used_by_curr_pic_flag[1]
        else:
            if self.sps_st_rps:
                b.u(0, 1)  # inter_ref_pic_set_prediction_flag (stRpsIdx > 0)
            b.ue(len(refs))
            b.ue(0)
            prev = poc
            for r in refs:
                b.ue(prev - r - 1)
                b.u(1, 1)
                prev = r
        b.u(1 if tmvp else 0, 1)
        b.u(1 if nref else 0, 1)  # num_ref_idx_active_override_flag
        if nref:
            assert all(cu.get("skip") for cu in cus)
            b.ue(nref - 1)
        if tmvp and nref and nref > 1:
            b.ue(0)        # collocated_ref_idx
        if self.weighted:
            self._pred_weight_table(b, wp)
        b.ue(5 - self.max_merge)
        b.se(qp - 26)
        b.trailing()
        c = Cabac(b, qp, 1)
        n = 1 << self.ctb
        ctus = [(x, yy) for yy in range(0, self.h, n) for x in range(0, self.w, n)]
        assert len(cus) == len(ctus)
        skip = {}
        for k, ((x0, y0), cu) in enumerate(zip(ctus, cus)):
            c.bin("split_cu_flag", 0, 0)
            inc = int(skip.get((x0 - n, y0), False)) + int(skip.get((x0, y0 - n), False))
            sk = bool(cu.get("skip"))
            skip[(x0, y0)] = sk
            c.bin("cu_skip_flag", inc, int(sk))
            if sk:
                if self.max_merge > 1:
                    c.bin("merge_idx", 0, 0)
            else:
                c.bin("pred_mode_flag", 0, 0)  # MODE_INTER
                part = cu.get("part", "2Nx2N")
                self._part_mode(c, part)
                pus = cu.get("pus", [("mvd", cu.get("mvd", (0, 0)))])
                for pu in pus:
                    if pu[0] == "merge":
                        c.bin("merge_flag", 0, 1)
                        if self.max_merge > 1:
                            c.bin("merge_idx", 0, 0)
                    else:
                        c.bin("merge_flag", 0, 0)
                        self._mvd(c, pu[1])
                        c.bin("mvp_flag", 0, 0)
                dc = cu.get("dc")
                if not (part == "2Nx2N" and pus[0][0] == "merge"):
                    c.bin("rqt_root_cbf", 0, 1 if dc else 0)
                if dc:
                    assert part == "2Nx2N"
                    self._transform_tree(c, self.ctb, dc)
            c.terminate(1 if k == len(ctus) - 1 else 0)
        b.align_zero()
        self._emit(1, b)

    def _pred_weight_table(self, b: Bits, wp: dict | None):
        wp = wp or {}
        denom = wp.get("denom", 0)
        b.ue(denom)
        cd = wp.get("cdenom_delta", 0)
        b.se(cd)
        has_l, has_c = "w" in wp, "cw" in wp
        b.u(int(has_l), 1)
        b.u(int(has_c), 1)
        if has_l:
            b.se(wp["w"] - (1 << denom))
            b.se(wp["o"])
        if has_c:
            cden = denom + cd
            for cw, delta_off in wp["cw"]:   # chroma offsets are coded as deltas (7.4.7.3)
                b.se(cw - (1 << cden))
                b.se(delta_off)

    @staticmethod
    def _part_mode(c: Cabac, part: str):
        bins = {"2Nx2N": "1", "2NxN": "011", "Nx2N": "001", "2NxnU": "0100", "2NxnD": "0101",
                "nLx2N": "0000", "nRx2N": "0001"}[part]
        for i, ch in enumerate(bins):
            if i < 2:
                c.bin("part_mode", i, int(ch))
            elif i == 2:
                c.bin("part_mode", 3, int(ch))  # log2CbSize > MinCbLog2SizeY with AMP
            else:
                c.bypass(int(ch))

    @staticmethod
    def _mvd(c: Cabac, mvd):
        ax, ay = abs(mvd[0]), abs(mvd[1])
        c.bin("abs_mvd_greater0", 0, int(ax > 0))
        c.bin("abs_mvd_greater0", 0, int(ay > 0))
        if ax:
            c.bin("abs_mvd_greater1", 0, int(ax > 1))
        if ay:
            c.bin("abs_mvd_greater1", 0, int(ay > 1))
        for a, s in ((ax, mvd[0] < 0), (ay, mvd[1] < 0)):
            if a:
                if a > 1:
                    c.eg(a - 2, 1)
                c.bypass(int(s))

    def _transform_tree(self, c: Cabac, log2: int, dc: list[int]):
        """Inter 2Nx2N CU of size 2^log2: transform blocks of min(log2, max_tb) (a CU above the
        maximum splits implicitly), chroma cbfs 0, one DC level per luma TB."""
        tbs = iter(dc)

        def node(l2: int, depth: int, parent_chroma: bool):
            # split_transform_flag is never coded here (max_transform_hierarchy_depth_inter 0)
            split = l2 > self.max_tb
            if l2 > 2 and (depth == 0 or parent_chroma):
                c.bin("cbf_chroma", depth, 0)
                c.bin("cbf_chroma", depth, 0)
            if split:
                for _ in range(4):
                    node(l2 - 1, depth + 1, False)
                return
            if depth != 0:
                c.bin("cbf_luma", 1 if depth == 0 else 0, 1)
            self._residual_dc(c, l2, next(tbs))

        node(log2, 0, True)

    @staticmethod
    def _residual_dc(c: Cabac, log2: int, level: int):
        assert level != 0 and abs(level) <= 6
        off = 3 * (log2 - 2) + ((log2 - 1) >> 2)
        c.bin("last_x_prefix", off, 0)
        c.bin("last_y_prefix", off, 0)
        a = abs(level)
        c.bin("greater1", 1, int(a > 1))
        if a > 1:
            c.bin("greater2", 0, int(a > 2))
        c.bypass(int(level < 0))
        if a > 2:
            rem = a - 3           # cRiceParam 0, below the escape (prefix TR of 4)
            for _ in range(rem):
                c.bypass(1)
            c.bypass(0)

    def bytes(self) -> bytes:
        return bytes(self.out)


def sample_streams(content) -> list[bytes]:
    """A few KAT constructions (fractional motion, weighted prediction at 8 / 10 bits, TMVP
    scaling, an AMP merge PU, scaling lists with a 16x16 DC entry) for the GPU decoder test;
    ``content(w, h, bd, seed)`` -> (y, u, v) int arrays."""
    out = []
    for bd in (8, 10):
        s = KatStream(32, 32, bit_depth=bd, ctb_log2=4, weighted=True)
        s.idr_pcm(*content(32, 32, bd, 40 + bd))
        s.p_picture(1, [0], [{"mvd": (-9, 14)}] + [{"skip": True}] * 3,
                    wp={"denom": 5, "w": 40, "o": -7, "cdenom_delta": 1, "cw": [(70, 3), (50, -20)]})
        s.p_picture(2, [1], [{"mvd": (3, -5)}, {"skip": True}, {"mvd": (6, 1), "dc": None}, {"skip": True}],
                    wp={"denom": 0, "w": 1, "o": 3})
        out.append(s.bytes())
    s = KatStream(64, 32, ctb_log2=5)
    s.idr_pcm(*content(64, 32, 8, 50))
    s.p_picture(3, [0], [{"mvd": (-7, 21)}, {"part": "nLx2N", "pus": [("mvd", (5, -6)), ("merge",)]}])
    s.p_picture(8, [3], [{"skip": True}, {"part": "2NxnU", "pus": [("mvd", (-4, 2)), ("merge",)]}], tmvp=True)
    out.append(s.bytes())
    s = KatStream(32, 16, ctb_log2=4, scaling={(2, 3): ([(8 + 3 * i) % 97 + 9 for i in range(64)], 37)})
    s.idr_pcm(*content(32, 16, 8, 51))
    s.p_picture(1, [0], [{"mvd": (0, 0), "dc": [-4]}, {"mvd": (2, 3), "dc": [5]}], qp=31)
    out.append(s.bytes())
    return out
