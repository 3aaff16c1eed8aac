"""Random HEVC decision-record streams (test inputs for the HEVC writer/decoder pair).

Records follow csrc/common/hevc_tables.h: a 32-byte ``CtuInfo`` per 32x32 CTB, an
8-byte ``CuInfo`` per 8x8 granule (z-order, replicated over each CU) and level planes
shaped like the picture.  Pictures mix every CU size, all 35 intra modes, inter CUs
with random motion (skip / merge / AMVP chosen by the writer), sparse random levels
with occasional large magnitudes (escape codes) and random SAO parameters.
"""
from __future__ import annotations

import numpy as np

CTB = 32


def _zorder8(gx: int, gy: int) -> int:
    return (gx & 1) | ((gy & 1) << 1) | ((gx & 2) << 1) | ((gy & 2) << 2)


def _cu_list(split: int):
    """(x, y, size) of the CUs of a CTB in coding order for a split byte."""
    if not split & 1:
        return [(0, 0, 32)]
    out = []
    for q in range(4):
        x1, y1 = (q & 1) * 16, (q >> 1) * 16
        if (split >> (1 + q)) & 1:
            out += [(x1 + (r & 1) * 8, y1 + (r >> 1) * 8, 8) for r in range(4)]
        else:
            out.append((x1, y1, 16))
    return out


def _levels(rng, n: int, density: float) -> np.ndarray:
    blk = np.zeros((n, n), np.int16)
    if rng.random() < 0.3:
        return blk
    mask = rng.random((n, n)) < density * (1.0 + 3.0 * (np.add.outer(np.arange(n), np.arange(n)) < n // 2))
    vals = rng.integers(-3, 4, (n, n))
    big = rng.random((n, n)) < 0.03
    vals = np.where(big, rng.integers(-600, 601, (n, n)), vals)
    blk[mask] = vals[mask]
    return blk


def random_records(rng, width: int, height: int, pslice: bool, bit_depth: int = 8, density: float = 0.08,
                   intra_in_p: float = 0.2, mv_range: int = 64, sao: bool = True, ctb_qp: tuple | None = None,
                   nxn: float = 0.0, tu_split: float = 0.0, force_split: int | None = None, bslice: bool = False,
                   mv_pool: int = 0, uniform64: float = 0.0, nref: tuple = (1, 1)):
    """``ctb_qp = (qp, spread)``: per-CTB QPs qp + U[-spread, spread] (cu_qp_delta streams);
    ``nxn``: probability of an 8x8 intra CU being split into four 4x4 PUs; ``tu_split``: of a
    16x16 / 32x32 inter CU coding its residual as four quarter TUs (needs tu_inter_depth 1);
    ``bslice``: inter CUs predict from list 0, list 1 or both (CuInfo.dir, mv1); ``mv_pool`` > 0:
    vectors drawn from that many values, so merge candidates (spatial, temporal, combined
    bi-predictive, zero) match often; ``uniform64``: probability that a 64x64-aligned group of
    four blocks is one residual-free inter motion (the CTU-64 writer codes it as a 64x64 skip CU
    when the motion is a merge candidate); ``nref``: active pictures of list 0 / list 1 -- inter CUs
    draw a refIdx per used list (CuInfo pad[0] / pad[1], bytes 13 / 14)."""
    pool = rng.integers(-mv_range, mv_range + 1, (max(1, mv_pool), 2)).astype(np.int16) if mv_pool else None

    def rand_mv():
        if pool is not None:
            return pool[int(rng.integers(0, len(pool)))].copy()
        return rng.integers(-mv_range, mv_range + 1, 2).astype(np.int16)
    W, H = -(-width // CTB) * CTB, -(-height // CTB) * CTB
    wc, hc = W // CTB, H // CTB
    ctu = np.zeros((wc * hc, 32), np.uint8)
    cu = np.zeros((wc * hc * 16, 16), np.uint8)
    cy = np.zeros((H, W), np.int16)
    cb = np.zeros((H // 2, W // 2), np.int16)
    cr = np.zeros((H // 2, W // 2), np.int16)
    cmax = (1 << (min(bit_depth, 10) - 5)) - 1
    for i in range(wc * hc):
        rx, ry = i % wc, i // wc
        r = rng.random()
        split = 0 if r < 0.25 else (1 | (int(rng.integers(0, 16)) << 1))
        if force_split is not None:
            split = force_split
        ctu[i, 0] = split
        if ctb_qp is not None:
            ctu[i, 1] = np.int8(np.clip(ctb_qp[0] + rng.integers(-ctb_qp[1], ctb_qp[1] + 1), 0, 51)).view(np.uint8)
        if sao:
            t = ctu[i]
            for k in range(2):
                t[2 + k] = int(rng.integers(0, 3))
                t[4 + k] = int(rng.integers(0, 4))
            t[6:9] = rng.integers(0, 32, 3)
            off = np.zeros((3, 4), np.int8)
            for c in range(3):
                typ = t[2 + (1 if c else 0)]
                a = rng.integers(0, cmax + 1, 4)
                if typ == 1:
                    off[c] = a * rng.choice([-1, 1], 4)
                elif typ == 2:
                    off[c] = [a[0], a[1], -a[2], -a[3]]
            t[10:22] = off.reshape(-1).view(np.uint8)
            if rx > 0 and rng.random() < 0.2:   # exercise sao_merge_left
                t[2:22] = ctu[i - 1, 2:22]
        for (x, y, n) in _cu_list(split):
            intra = (not pslice) or rng.random() < intra_in_p
            rec = np.zeros(16, np.uint8)
            rec[0] = 0 if intra else 1
            if intra:
                rec[1] = int(rng.integers(0, 35))
                if n == 8 and rng.random() < nxn:   # PART_NxN: four 4x4 PUs (flags bit 3)
                    rec[3] |= 8
                    rec[4:8] = rng.integers(0, 35, 4)
                    rec[4] = rec[1]
            else:
                if n >= 16 and rng.random() < tu_split:   # residual quadtree split once (flags bit 4)
                    rec[3] |= 16
                mv = rand_mv()
                if rng.random() < 0.3:
                    mv[:] = 0
                if bslice:
                    d = int(rng.integers(1, 4))
                    mv1 = rand_mv()
                    if rng.random() < 0.3:
                        mv1[:] = 0
                    rec[12] = d
                    if d & 1:
                        rec[4:8] = mv.view(np.uint8)
                        rec[13] = int(rng.integers(0, nref[0]))
                    if d & 2:
                        rec[8:12] = mv1.view(np.uint8)
                        rec[14] = int(rng.integers(0, nref[1]))
                else:
                    rec[4:8] = mv.view(np.uint8)
                    rec[13] = int(rng.integers(0, nref[0]))
            for gy in range(y // 8, (y + n) // 8):
                for gx in range(x // 8, (x + n) // 8):
                    cu[i * 16 + _zorder8(gx, gy)] = rec
            X, Y = rx * CTB + x, ry * CTB + y
            cy[Y:Y + n, X:X + n] = _levels(rng, n, density)
            cb[Y // 2:(Y + n) // 2, X // 2:(X + n) // 2] = _levels(rng, n // 2, density)
            cr[Y // 2:(Y + n) // 2, X // 2:(X + n) // 2] = _levels(rng, n // 2, density)
    if uniform64 > 0 and pslice:
        for gy in range(0, hc - 1, 2):
            for gx in range(0, wc - 1, 2):
                if rng.random() >= uniform64:
                    continue
                rec = np.zeros(16, np.uint8)
                rec[0], rec[3] = 1, 2 << 1   # inter, 32x32 CU
                mv = rand_mv() if rng.random() < 0.5 else np.zeros(2, np.int16)
                rec[4:8] = mv.view(np.uint8)
                if bslice:
                    rec[12] = 1
                for by in (gy, gy + 1):
                    for bx in (gx, gx + 1):
                        i = by * wc + bx
                        ctu[i, 0] = 0
                        cu[i * 16:(i + 1) * 16] = rec
                Y, X = gy * CTB, gx * CTB
                cy[Y:Y + 64, X:X + 64] = 0
                cb[Y // 2:Y // 2 + 32, X // 2:X // 2 + 32] = 0
                cr[Y // 2:Y // 2 + 32, X // 2:X // 2 + 32] = 0
    return ctu, cu, cy, cb, cr


def random_stream(host, width: int, height: int, frames: int, seed: int = 0, qp: int = 30, bit_depth: int = 8,
                  host_cfg: dict | None = None, qp_spread: int = 0, **kw) -> tuple[bytes, list]:
    """Annex-B HEVC stream (IDR + P pictures) and the records it was written from.
    ``host_cfg`` adds writer options (e.g. ``wpp=1, threads=4``); ``qp_spread`` > 0 gives
    every CTB its own QP (needs ``cu_qp_delta=1`` in ``host_cfg``)."""
    rng = np.random.default_rng(seed)
    cfg = dict(width=width, height=height, bit_depth=bit_depth, **(host_cfg or {}))
    out = [host.hevc_parameter_sets(cfg)]
    recs = []
    for t in range(frames):
        fqp = int(np.clip(qp + rng.integers(-3, 4), 0, 51))
        r = random_records(rng, width, height, pslice=t > 0, bit_depth=bit_depth,
                           ctb_qp=(fqp, qp_spread) if qp_spread else None, **kw)
        nal, _ = host.hevc_write_slice(cfg, dict(idr=int(t == 0), poc=t, qp=fqp, slice_type=1 if t else 2), *r)
        out.append(nal)
        recs.append(r)
    return b"".join(out), recs


def random_gop_stream(host, width: int, height: int, frames: int, bframes: int = 3, seed: int = 0, qp: int = 30,
                      bit_depth: int = 8, tmvp: bool = True, pyramid: bool = False, host_cfg: dict | None = None,
                      refs: int = 1, **kw) -> tuple[bytes, list]:
    """Annex-B HEVC stream of one closed GOP with B pictures (models/gop.py hevc_gop_plan:
    I, P anchors, B pictures referencing the pictures on both sides; ``pyramid``: the middle
    B of a run is a reference picture) from random records, with each picture's RPS; TMVP
    takes the collocated picture's records.  Returns the stream and the records per
    *display* index (the decoder outputs pictures in POC order).  ``refs`` > 1: P pictures
    predict from up to that many earlier reference pictures (x265 --ref; refIdx per CU)."""
    from ..models.gop import hevc_gop_plan, hevc_ref_slots

    rng = np.random.default_rng(seed)
    cfg = dict(width=width, height=height, bit_depth=bit_depth, bframes=bframes, tmvp=int(tmvp), pyramid=int(pyramid),
               refs=int(refs), **(host_cfg or {}))
    out = [host.hevc_parameter_sets(cfg)]
    recs: list = [None] * frames
    nrefs = int(refs)
    held = {}    # display index -> (cu records or None for intra, its L0 / L1 references, its list 0)
    for pic in hevc_gop_plan(frames, bframes, pyramid, refs=nrefs, ref_slots=hevc_ref_slots(bframes, pyramid, nrefs)):
        fqp = int(np.clip(qp + rng.integers(-3, 4), 0, 51))
        r = random_records(rng, width, height, pslice=pic.kind != "I", bit_depth=bit_depth, bslice=pic.kind == "B",
                           nref=(max(1, len(pic.refs0)), 1), **kw)
        fp = dict(idr=int(pic.kind == "I"), poc=pic.d, qp=fqp, slice_type={"I": 2, "P": 1, "B": 0}[pic.kind],
                  nal_ref=int(pic.ref), rps=[(d, int(u)) for d, u in pic.rps])
        if pic.kind != "I":
            fp["ref_poc0"] = pic.l0
            fp["refs0"] = list(pic.refs0)
            col = pic.l1 if pic.kind == "B" else pic.l0
            if pic.kind == "B":
                fp["ref_poc1"] = pic.l1
            ccu, c0, c1, cl0 = held[col]
            fp.update(col_poc=col, col_ref_poc0=c0, col_ref_poc1=c1, col_cu=ccu, col_refs0=cl0)
        nal, _ = host.hevc_write_slice(cfg, fp, *r)
        if pic.ref:
            held[pic.d] = (None if pic.kind == "I" else r[1].copy(), pic.l0, pic.l1, list(pic.refs0) or None)
        out.append(nal)
        recs[pic.d] = r
    return b"".join(out), recs


def expected_ctb_qps(ctu: np.ndarray, cy: np.ndarray, cb: np.ndarray, cr: np.ndarray, slice_qp: int,
                     wpp: bool) -> np.ndarray:
    """QpY per CTB a decoder derives from cu_qp_delta records (8.6.1, one quantization
    group per CTB): the CTB's own QP when any block of it has a coded level, else the
    prediction (the previous CTB's QpY; the slice QP at the slice start and, with WPP,
    at every CTB row)."""
    H, W = cy.shape
    wc = W // CTB
    out = np.zeros(len(ctu), np.int32)
    prev = slice_qp
    for i in range(len(ctu)):
        rx, ry = i % wc, i // wc
        if wpp and rx == 0:
            prev = slice_qp
        X, Y = rx * CTB, ry * CTB
        coded = (cy[Y:Y + CTB, X:X + CTB].any() or cb[Y // 2:Y // 2 + 16, X // 2:X // 2 + 16].any()
                 or cr[Y // 2:Y // 2 + 16, X // 2:X // 2 + 16].any())
        q = int(ctu[i, 1].view(np.int8)) if coded else prev
        out[i] = q
        prev = q
    return out


def pack_levels(cy: np.ndarray, cb: np.ndarray, cr: np.ndarray):
    """Level planes -> the GPU encoder's packed form (hevc::PackedLevels, numpy model of
    hevc_nz_map / hevc_nz_pack): per CTB sub-block maps, first-block offsets, and the
    non-zero 4x4 blocks in luma, Cb, Cr bit order."""
    H, W = cy.shape
    wc, hc = W // CTB, H // CTB
    nz = np.zeros((wc * hc, 2), np.uint64)
    off = np.zeros(wc * hc, np.uint32)
    blocks = []
    n = 0
    for ci in range(wc * hc):
        rx, ry = ci % wc, ci // wc
        off[ci] = n
        lm = cm = 0
        for by in range(8):
            for bx in range(8):
                b = cy[ry * 32 + by * 4:ry * 32 + by * 4 + 4, rx * 32 + bx * 4:rx * 32 + bx * 4 + 4]
                if b.any():
                    lm |= 1 << (by * 8 + bx)
                    blocks.append(b.copy())
        for c, pl in enumerate((cb, cr)):
            for by in range(4):
                for bx in range(4):
                    b = pl[ry * 16 + by * 4:ry * 16 + by * 4 + 4, rx * 16 + bx * 4:rx * 16 + bx * 4 + 4]
                    if b.any():
                        cm |= 1 << (16 * c + by * 4 + bx)
                        blocks.append(b.copy())
        nz[ci] = (lm, cm)
        n = len(blocks)
    lv = np.stack(blocks).reshape(-1) if blocks else np.zeros(16, np.int16)
    return nz, off, lv.astype(np.int16)


def unpack_levels(nz: np.ndarray, off: np.ndarray, lv: np.ndarray, W: int, H: int):
    """Inverse of :func:`pack_levels`: packed non-zero 4x4 blocks -> level planes."""
    wc = W // CTB
    cy = np.zeros((H, W), np.int16)
    cb = np.zeros((H // 2, W // 2), np.int16)
    cr = np.zeros((H // 2, W // 2), np.int16)
    blocks = lv.reshape(-1, 4, 4)
    for ci in range(len(off)):
        rx, ry = ci % wc, ci // wc
        k = int(off[ci])
        lm, cm = int(nz[ci, 0]), int(nz[ci, 1])
        for bit in range(64):
            if lm >> bit & 1:
                by, bx = divmod(bit, 8)
                cy[ry * 32 + by * 4:ry * 32 + by * 4 + 4, rx * 32 + bx * 4:rx * 32 + bx * 4 + 4] = blocks[k]
                k += 1
        for bit in range(32):
            if cm >> bit & 1:
                pl = cb if bit < 16 else cr
                by, bx = divmod(bit & 15, 4)
                pl[ry * 16 + by * 4:ry * 16 + by * 4 + 4, rx * 16 + bx * 4:rx * 16 + bx * 4 + 4] = blocks[k]
                k += 1
    return cy, cb, cr


def _diag4():
    """(x, y) of the 16 positions of a 4x4 diagonal up-right scan (6.5.3)."""
    out = []
    for d in range(7):
        for y in range(d, -1, -1):
            x = d - y
            if x < 4 and y < 4:
                out.append((x, y))
    return out


def hide_signs_diag(blk: np.ndarray) -> np.ndarray:
    """Make a TU's levels sign-data-hiding consistent for the diagonal scan (the test model
    of an encoder's parity fix): in every 4x4 group whose significant span exceeds 3 scan
    positions, negate the first significant coefficient when the parity of the group's
    absolute sum disagrees with its sign."""
    out = blk.copy()
    sc = _diag4()
    n = blk.shape[0]
    for gy in range(0, n, 4):
        for gx in range(0, n, 4):
            v = [int(out[gy + y, gx + x]) for x, y in sc]
            nzp = [p for p in range(16) if v[p] != 0]
            if nzp and nzp[-1] - nzp[0] > 3:
                if (sum(abs(t) for t in v) & 1) != (v[nzp[0]] < 0):
                    x, y = sc[nzp[0]]
                    out[gy + y, gx + x] = -out[gy + y, gx + x]
    return out
