"""Random H.264 decision-record streams (test / benchmark inputs for the decoders).

A stream is written from random per-MB records through the host CAVLC writer
(``_host.write_slice``): I pictures mix Intra16x16 and Intra4x4 MBs with random
*legal* prediction modes; P pictures mix P_Skip, P_L0_16x16, 16x8, 8x16, 8x8
(8x8 sub-blocks) and intra MBs with random motion vectors, per-MB QP deltas and
sparse random levels.  The result exercises every syntax path the GPU decoder
reconstructs, which encoder-produced streams (16x16 motion only) do not.
"""
from __future__ import annotations

import numpy as np

from .. import ops  # noqa: F401  (package import order)

# MbHeader byte offsets (csrc/common/h264_mb.h)
_KIND, _CBP, _QP, _I16, _CHROMA, _FLAGS, _REF, _MV, _I4 = 0, 1, 2, 3, 4, 5, 8, 16, 48
HDR_BYTES = 64
I4x4, I16x16, P16x16, PSKIP, IPCM, P16x8, P8x16, P8x8, I8x8 = 0, 1, 2, 3, 4, 5, 6, 7, 8
MBF_T8x8 = 2
_ZZ8 = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14,
        21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53,
        60, 61, 54, 47, 55, 62, 63]

_BLK_X = [0, 1, 0, 1, 2, 3, 2, 3, 0, 1, 0, 1, 2, 3, 2, 3]
_BLK_Y = [0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3]


def _i4_modes_ok(rng, mx: int, my: int) -> list[int]:
    out = []
    for b in range(16):
        bx, by = _BLK_X[b], _BLK_Y[b]
        left = bx > 0 or mx > 0
        top = by > 0 or my > 0
        ok = [2]
        if top:
            ok += [0, 3, 7]
        if left:
            ok += [1, 8]
        if top and left:
            ok += [4, 5, 6]
        out.append(int(rng.choice(ok)))
    return out


def _i8_modes_ok(rng, mx: int, my: int) -> list[int]:
    """Legal Intra8x8 modes per 8x8 block (8.3.2.2): availability of top / left / top-left."""
    out = []
    for b8 in range(4):
        top = b8 >= 2 or my > 0
        left = (b8 & 1) == 1 or mx > 0
        tl = (b8 == 3) or (b8 == 0 and mx > 0 and my > 0) or (b8 == 1 and my > 0) or (b8 == 2 and mx > 0)
        ok = [2]
        if top:
            ok += [0, 3, 7]
        if left:
            ok += [1, 8]
        if top and left and tl:
            ok += [4, 5, 6]
        out.append(int(rng.choice(ok)))
    return out


def _i16_mode(rng, mx: int, my: int) -> int:
    ok = [2] + ([0] if my > 0 else []) + ([1] if mx > 0 else []) + ([3] if mx > 0 and my > 0 else [])
    return int(rng.choice(ok))


def _chroma_mode(rng, mx: int, my: int) -> int:
    ok = [0] + ([1] if mx > 0 else []) + ([2] if my > 0 else []) + ([3] if mx > 0 and my > 0 else [])
    return int(rng.choice(ok))


def _levels(rng, n: int, density: float, start: int = 0) -> np.ndarray:
    v = np.zeros(n, np.int16)
    pos = np.arange(start, n)
    keep = pos[rng.random(len(pos)) < density]
    v[keep] = rng.integers(-4, 5, len(keep))
    return v


def _intra_record(rng, h, c, mx, my, qp, density, allow_i4=True, t8x8=False, dc_only=False, pcm=0.0, bit_depth=8):
    qp &= 0xFF  # int8 QP_Y (negative below QP 0 at High 10)
    if pcm and rng.random() < pcm:
        h[_KIND] = IPCM
        c[:384] = rng.integers(0, 1 << bit_depth, 384)
        h[_QP] = qp
        return
    if dc_only:  # constrained intra in P pictures: DC modes are legal with any availability
        h[_KIND] = I4x4 if rng.random() < 0.5 else I16x16
        h[_I16] = 2
        h[_I4:_I4 + 16] = 2
        for b in range(16):
            c[b * 16:(b + 1) * 16] = _levels(rng, 16, density, start=int(h[_KIND] == I16x16))
        if h[_KIND] == I16x16:
            c[256:272] = _levels(rng, 16, density * 2)
        h[_CHROMA] = 0
        h[_QP] = qp
        c[272:280] = _levels(rng, 8, density)
        for b in range(8):
            c[280 + b * 16:280 + (b + 1) * 16] = _levels(rng, 16, density / 2, start=1)
        return
    if t8x8 and rng.random() < 0.35:
        h[_KIND] = I8x8
        modes = _i8_modes_ok(rng, mx, my)
        h[_I4:_I4 + 16] = np.repeat(modes, 4)
        for b8 in range(4):
            c[b8 * 64:(b8 + 1) * 64] = _levels(rng, 64, density / 2) if rng.random() < 0.7 else 0
    elif allow_i4 and rng.random() < 0.5:
        h[_KIND] = I4x4
        h[_I4:_I4 + 16] = _i4_modes_ok(rng, mx, my)
        for b in range(16):
            c[b * 16:(b + 1) * 16] = _levels(rng, 16, density)
    else:
        h[_KIND] = I16x16
        h[_I16] = _i16_mode(rng, mx, my)
        for b in range(16):
            c[b * 16:(b + 1) * 16] = _levels(rng, 16, density, start=1) if rng.random() < 0.5 else 0
        c[256:272] = _levels(rng, 16, density * 2)
        h[_I4:_I4 + 16] = 2
    h[_CHROMA] = _chroma_mode(rng, mx, my)
    h[_QP] = qp
    c[272:280] = _levels(rng, 8, density)
    for b in range(8):
        c[280 + b * 16:280 + (b + 1) * 16] = _levels(rng, 16, density / 2, start=1)


def random_stream(host, width: int, height: int, frames: int, seed: int = 0, qp: int = 28,
                  density: float = 0.15, intra_in_p: float = 0.1, mv_range: int = 48, keyint: int = 0,
                  cabac: bool = False, t8x8: bool = False, records: list | None = None, refs: int = 1,
                  slice_rows: int = 0, pcm: float = 0.0, constrained_intra: bool = False,
                  cqm: dict | None = None, bit_depth: int = 8) -> bytes:
    """Annex-B stream of ``frames`` pictures (IDR + P) from random decision records.

    cabac / t8x8 select the entropy coder and the High-profile 8x8 transform (I8x8 MBs and
    8x8-transformed inter MBs).  ``records``, if given, receives (hdr, coef) per picture.
    ``slice_rows`` > 0: every picture is coded as several slices of that many MB rows (intra
    modes then treat each slice's first row as having no row above).  ``pcm``: share of I_PCM
    macroblocks (CAVLC); ``constrained_intra``: constrained_intra_pred_flag (CAVLC; intra MBs of
    P pictures use DC modes); ``cqm``: scaling-matrix keys of the writer config (cqm, cqm4,
    cqm8, cqm_coded; needs t8x8); ``bit_depth`` > 8: a High 10 stream (PCM samples of that many
    bits, QPs down to -6 * (bit_depth - 8))."""
    rng = np.random.default_rng(seed)
    cfg = dict(width=width, height=height, qp=qp, cabac=int(cabac), t8x8=int(t8x8), refs=int(refs),
               constrained_intra=int(constrained_intra), bit_depth=int(bit_depth), **(cqm or {}))
    qmin = -6 * (int(bit_depth) - 8)
    wmb, hmb = (width + 15) // 16, (height + 15) // 16
    nmb = wmb * hmb
    out = [host.parameter_sets(cfg)]
    fn = 0
    idr_id = 0
    since_idr = 0
    for t in range(frames):
        idr = t == 0 or (keyint > 0 and t % keyint == 0)
        if idr:
            fn = 0
            since_idr = 0
        nref = max(1, min(int(refs), since_idr))  # references held by the sliding window
        sqp = int(np.clip(qp + rng.integers(-2, 3), max(10 + qmin, qmin), 48))
        hdr = np.zeros((nmb, HDR_BYTES), np.uint8)
        hdr[:, _REF:_REF + 8] = 0xFF
        coef = np.zeros((nmb, 408), np.int16)
        for mb in range(nmb):
            mx, my = mb % wmb, mb // wmb
            h, c = hdr[mb], coef[mb]
            mqp = int(np.clip(sqp + rng.integers(-3, 4), qmin, 51))
            if idr or rng.random() < intra_in_p:
                r0 = (my // slice_rows) * slice_rows if slice_rows else 0
                _intra_record(rng, h, c, mx, my - r0, mqp, density, t8x8=t8x8, dc_only=constrained_intra and not idr,
                              pcm=pcm, bit_depth=bit_depth)
                continue
            r = rng.random()
            kind = PSKIP if r < 0.25 else (P16x16 if r < 0.5 else (P16x8 if r < 0.65 else (P8x16 if r < 0.8 else P8x8)))
            mv = rng.integers(-mv_range, mv_range + 1, (4, 2))
            if kind in (PSKIP, P16x16):
                mv[:] = mv[0]
            elif kind == P16x8:
                mv[1], mv[3] = mv[0], mv[2]
            elif kind == P8x16:
                mv[2], mv[3] = mv[0], mv[1]
            h[_KIND] = kind
            h[_QP] = mqp & 0xFF
            h[_MV:_MV + 16] = np.frombuffer(mv.astype(np.int16).tobytes(), np.uint8)
            rf = rng.integers(0, nref, 4) if kind != PSKIP else np.zeros(4, np.int64)
            if kind == P16x16:
                rf[:] = rf[0]
            elif kind == P16x8:
                rf[1], rf[3] = rf[0], rf[2]
            elif kind == P8x16:
                rf[2], rf[3] = rf[0], rf[1]
            h[_REF:_REF + 4] = rf.astype(np.uint8)
            if kind != PSKIP:
                if t8x8 and rng.random() < 0.5:
                    h[_FLAGS] = MBF_T8x8
                    for b8 in range(4):
                        c[b8 * 64:(b8 + 1) * 64] = _levels(rng, 64, density / 2) if rng.random() < 0.6 else 0
                else:
                    for b in range(16):
                        c[b * 16:(b + 1) * 16] = _levels(rng, 16, density) if rng.random() < 0.6 else 0
                c[272:280] = _levels(rng, 8, density)
                for b in range(8):
                    c[280 + b * 16:280 + (b + 1) * 16] = _levels(rng, 16, density / 2, start=1)
        fp = dict(idr=int(idr), qp=sqp, frame_num=fn, idr_pic_id=idr_id)
        if not idr and refs > 1:
            fp["num_ref_l0"] = nref
        if slice_rows:
            for r0 in range(0, hmb, slice_rows):
                n_mbs = min(slice_rows, hmb - r0) * wmb
                nal, _ = host.write_slice(cfg, dict(fp, first_mb=r0 * wmb, num_mbs=n_mbs), hdr, coef)
                out.append(nal)
        else:
            nal, _ = host.write_slice(cfg, fp, hdr, coef)
            out.append(nal)
        if records is not None:
            records.append((hdr, coef))
        if idr:
            idr_id += 1
        since_idr += 1
        fn = (fn + 1) % 16
    return b"".join(out)


def unpack_levels(seg: dict, t: int) -> np.ndarray:
    """Dense [nmb, 408] levels of picture t of a ``_host.parse`` segment (inverse of the
    packed block format; used by the round-trip tests)."""
    mask, off = seg["mask"][t], seg["off"][t]
    base = int(seg["pic_off"][t])
    coef = seg["coef"]
    nmb = mask.shape[0]
    out = np.zeros((nmb, 408), np.int16)
    for mb in range(nmb):
        m = int(mask[mb])
        k = base + int(off[mb])
        for bit in range(26):
            if not (m >> bit) & 1:
                continue
            blk = coef[k * 16:(k + 1) * 16]
            k += 1
            if bit < 16:
                out[mb, bit * 16:(bit + 1) * 16] = blk
            elif bit == 16:
                out[mb, 256:272] = blk
            elif bit == 17:
                out[mb, 272:280] = blk[:8]
            else:
                j = bit - 18
                out[mb, 280 + j * 16:280 + (j + 1) * 16] = blk
    return out


# ---------------------------------------------------------------- B pictures (temporal direct)
B16x16, BDIRECT = 9, 13


def _trunc_div(a: int, b: int) -> int:
    """C integer division (rounds toward zero), as the spec's "/" operator."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def temporal_direct(col_hdr: np.ndarray, poc_cur: int, poc_l0: int, poc_l1: int):
    """Temporal direct motion (clause 8.4.1.2.3, frame MBs, direct_8x8_inference_flag = 1)
    for every MB of a B picture whose RefPicList1[0] is the P picture ``col_hdr``
    ([nmb, 64] MbHeader bytes) and whose RefPicList0[0] is that picture's own reference.

    Returns (mvL0, mvL1) as int [nmb, 4, 2] per 8x8 quadrant; refIdxL0 = refIdxL1 = 0.
    Co-located intra MBs give mvCol = 0; with direct_8x8_inference the corner 4x4 block of
    each co-located quadrant supplies mvCol, i.e. that quadrant's MV."""
    nmb = col_hdr.shape[0]
    kinds = col_hdr[:, _KIND]
    mv_col = np.frombuffer(np.ascontiguousarray(col_hdr[:, _MV:_MV + 16]).tobytes(), np.int16).reshape(nmb, 4, 2)
    mv_col = mv_col.astype(np.int64)
    intra = np.isin(kinds, [I4x4, I16x16, 4, I8x8])
    mv_col = np.where(intra[:, None, None], 0, mv_col)
    tb = int(np.clip(poc_cur - poc_l0, -128, 127))
    td = int(np.clip(poc_l1 - poc_l0, -128, 127))
    if td == 0:
        return mv_col.copy(), np.zeros_like(mv_col)
    tx = _trunc_div(16384 + abs(_trunc_div(td, 2)), td)
    dsf = int(np.clip((tb * tx + 32) >> 6, -1024, 1023))
    mv_l0 = (dsf * mv_col + 128) >> 8
    mv_l1 = mv_l0 - mv_col
    return mv_l0, mv_l1
