// H.264 CABAC entropy coder (clause 9.3) shared by the host slice writer and the
// gfx950 slice-coding kernel (csrc/kernels/cabac.hip): one implementation, compiled for
// both, so the GPU bitstream is byte-identical to the host one by construction and the
// host build is what the CPU tests exercise.
//
// Reference parity: x264's default entropy coder behind the reference's `264` preset
// (`-threads 4 -vcodec libx264`, server.go:69-70, executed at client.go:115).
//
// * CabacEncoder: the arithmetic coder of clause 9.3.4.2 in byte-oriented form.  The
//   10-bit codILow register is kept together with the not-yet-emitted bits above it;
//   whole bytes leave as soon as 8 are pending, and the outstanding-bit mechanism of the
//   spec becomes carry propagation into a pending byte followed by a run of 0xFF bytes.
//   The first bit the spec suppresses (firstBitFlag) is always 0 and is dropped as the
//   carry position of the first byte.
// * CabacMbCoder: macroblock_layer() / residual() binarisation and context selection
//   (clauses 9.3.2, 9.3.3.1) from MbHeader records (h264_mb.h), for I, P and B slices,
//   4x4 and 8x8 transforms, partitions at 8x8 granularity.  All context selection is
//   derived from the records (cabac_prepare_mb + cabac_qp_chain), never from the coder,
//   so every macroblock can be binarised independently: the GPU binarises a whole
//   picture in parallel into 16-bit symbols and runs only the arithmetic coder serially.
#pragma once
#include <cstddef>
#include <cstdint>

#include "h264_cabac_tables.h"
#include "h264_mb.h"
#include "h264_tables.h"

namespace mivc {
namespace h264 {

#if defined(__HIPCC__) && defined(__HIP_DEVICE_COMPILE__)
MIVC_HD int cabac_clz32(uint32_t v) { return __clz(static_cast<int>(v)); }
#else
MIVC_HD int cabac_clz32(uint32_t v) { return v ? __builtin_clz(v) : 32; }
#endif

// Output sink over a caller-owned buffer (host vector storage or device memory).
struct CabacBuf {
  uint8_t* p;
  size_t cap;
  size_t n;
  int overflow;
  MIVC_HD void put(int b) {
    if (n < cap) p[n] = static_cast<uint8_t>(b);
    else overflow = 1;
    ++n;
  }
};

struct CabacEncoder {
  uint32_t low;
  uint32_t range;
  int nbits;  // output bits held above the 10-bit register (-1 before the first)
  int pend;   // last byte that may still receive a carry (-1: none yet)
  int nff;    // 0xFF bytes following it
  int bad;    // carry past the start of the stream (cannot happen for a valid coder)
  uint8_t* st;
  CabacBuf* out;

  MIVC_HD void init(uint8_t* states, CabacBuf* o) {
    low = 0;
    range = 510;
    nbits = -1;
    pend = -1;
    nff = 0;
    bad = 0;
    st = states;
    out = o;
  }
  MIVC_HD void put_byte(uint32_t v) {
    const int b = static_cast<int>(v & 0xFFu);
    if (v >> 8) {
      if (pend < 0) bad = 1;
      if (nff > 0) {
        out->put(pend + 1);
        for (int k = 0; k < nff - 1; ++k) out->put(0);
        pend = 0;
        nff = 0;
      } else {
        pend += 1;
      }
    }
    if (b == 0xFF) {
      ++nff;
    } else {
      if (pend >= 0) {
        out->put(pend);
        for (int k = 0; k < nff; ++k) out->put(0xFF);
      }
      pend = b;
      nff = 0;
    }
  }
  MIVC_HD void drain() {
    while (nbits >= 8) {
      const int sh = nbits + 2;
      const uint32_t v = low >> sh;
      low &= (1u << sh) - 1u;
      nbits -= 8;
      put_byte(v);
    }
  }
  MIVC_HD void shift(int s) {
    low <<= s;
    nbits += s;
    if (nbits >= 8) drain();
  }
  // EncodeDecision (9.3.4.2)
  MIVC_HD void decision(int ctx, int bin) {
    const int s = st[ctx];
    int pst = s >> 1, mps = s & 1;
    const uint32_t rlps = kCabacRangeLPS[pst][(range >> 6) & 3];
    range -= rlps;
    if (bin != mps) {
      low += range;
      range = rlps;
      if (pst == 0) mps ^= 1;
      pst = kCabacTransLPS[pst];
    } else {
      pst = pst < 62 ? pst + 1 : 62;
    }
    st[ctx] = static_cast<uint8_t>((pst << 1) | mps);
    if (range < 256) {
      const int sh = cabac_clz32(range) - 23;
      range <<= sh;
      shift(sh);
    }
  }
  // EncodeBypass (9.3.4.4)
  MIVC_HD void bypass(int bin) {
    low <<= 1;
    if (bin) low += range;
    ++nbits;
    if (nbits >= 8) drain();
  }
  // n (1..10) bypass bins at once, the first in bit n-1 of `bits`: each EncodeBypass is
  // low = 2 * low + b * range, so n of them are low * 2^n + range * bits
  MIVC_HD void bypass_bits(uint32_t bits, int n) {
    low = (low << n) + range * bits;
    nbits += n;
    if (nbits >= 8) drain();
  }
  // EncodeTerminate (9.3.4.5); bin = 1 also flushes (EncodeFlush) and writes the
  // rbsp_stop_one_bit plus zero alignment, i.e. the slice data is complete.
  MIVC_HD void terminate(int bin) {
    range -= 2;
    if (!bin) {
      if (range < 256) {
        range <<= 1;
        shift(1);
      }
      return;
    }
    low += range;
    // EncodeFlush: codIRange = 2, RenormE (7 bits), then PutBit(low bit 9) and
    // WriteBits(((low >> 7) & 3) | 1, 2): bits 9, 8 and a forced 1 at bit 7
    range = 2;
    shift(7);
    low |= 0x80u;
    shift(3);
    if (nbits > 0) shift(8 - nbits);  // zero-pad to the byte boundary
    if (pend >= 0) out->put(pend);
    for (int k = 0; k < nff; ++k) out->put(0xFF);
    pend = -1;
    nff = 0;
  }
  // unary / exp-Golomb helpers
  MIVC_HD void bypass_eg(uint32_t v, int k) {
    while (v >= (1u << k)) {
      bypass(1);
      v -= 1u << k;
      ++k;
    }
    bypass(0);
    while (k--) bypass((v >> k) & 1);
  }
};

// ---------------------------------------------------------------- symbol sinks
// The macroblock binariser (CabacMbCoder) writes into a sink with the engine's interface:
// decision(ctx, bin), bypass(bin), terminate(bin), bypass_eg(v, k).  CabacEncoder codes
// directly (host writer); the symbol sinks below record 16-bit symbols instead, so the
// GPU binarises every macroblock in parallel and only the arithmetic coding is serial:
//   regular    0 b ccccccccc          bin b with context c (< 512)
//   bypass     10 nnnn bbbbbbbbbb     n (1..10) bypass bins, first bin in bit n-1
//   terminate  11 ............ b      end_of_slice / I_PCM terminate bin
template <class Emit>
struct CabacSymbolPacker {
  Emit out;
  int nb = 0;        // pending bypass bins
  uint32_t bits = 0;
  MIVC_HD void flush_bypass() {
    if (nb) out.emit(static_cast<uint16_t>(0x8000u | (static_cast<uint32_t>(nb) << 10) | bits));
    nb = 0;
    bits = 0;
  }
  MIVC_HD void decision(int ctx, int bin) {
    flush_bypass();
    out.emit(static_cast<uint16_t>((bin ? 0x200u : 0u) | static_cast<uint32_t>(ctx)));
  }
  MIVC_HD void bypass(int bin) {
    bits = (bits << 1) | (bin ? 1u : 0u);
    if (++nb == 10) flush_bypass();
  }
  MIVC_HD void terminate(int bin) {
    flush_bypass();
    out.emit(static_cast<uint16_t>(0xC000u | (bin ? 1u : 0u)));
  }
  MIVC_HD void bypass_eg(uint32_t v, int k) {
    while (v >= (1u << k)) {
      bypass(1);
      v -= 1u << k;
      ++k;
    }
    bypass(0);
    while (k--) bypass((v >> k) & 1);
  }
};
struct CabacCountEmit {
  int n = 0;
  MIVC_HD void emit(uint16_t) { ++n; }
};
struct CabacStoreEmit {
  uint16_t* p;
  int n = 0;
  MIVC_HD void emit(uint16_t s) { p[n++] = s; }
};

// ---------------------------------------------------------------- per-MB coding state
// Everything the binarisation of an MB and of its later neighbours needs, computed from
// the decision records alone (cabac_prepare_mb) plus the mb_qp_delta chain
// (cabac_qp_chain).  Because nothing here depends on the arithmetic coder, every MB of a
// slice can be binarised independently.
struct alignas(8) CabacNb {
  uint8_t avail;       // coded in this slice (set by prepare)
  uint8_t kind;        // MbKind as coded (MBK_PSKIP for P_Skip, MBK_BDIRECT for B_Skip / B_Direct_16x16)
  uint8_t skip;        // mb_skip_flag
  uint8_t cbp;         // luma bits 0-3 | chroma << 4 (I_PCM: 0x2F)
  uint8_t t8x8;        // transform_size_8x8_flag as coded (0 when not coded)
  uint8_t chroma_mode; // intra_chroma_pred_mode (0 for inter / I_PCM)
  uint8_t direct;      // bit q: quadrant q predicted in direct mode
  uint8_t cbf_dc;      // bit0 luma DC, bit1 Cb DC, bit2 Cr DC
  uint16_t cbf_luma;   // raster 4x4 (x + 4y): coded_block_flag as seen by neighbours
  uint8_t cbf_cac[2];  // chroma AC, bit = raster 2x2 block
  int8_t ref[2][4];    // per quadrant and list (-1: list unused / intra)
  int16_t mv[2][4][2];
  int16_t mvd[2][4][2];  // mvd per quadrant, list, component (0 where none is coded)
  uint8_t i4[16];      // Intra4x4/8x8 pred mode per raster 4x4 (2 = DC for non-NxN)
  uint8_t i16_mode;
  uint8_t b_code;      // B mb_type (Table 7-14)
  int8_t dqp;          // mb_qp_delta (if coded)
  uint8_t prev_dqp_nz; // the previous MB in decoding order coded a non-zero mb_qp_delta
  int8_t qp;           // QP_Y of the record
  uint8_t pad[3];
  uint32_t mask;       // non-zero block mask (cabac_block_mask)
};

struct CabacSliceInfo {
  int slice_type;        // SLICE_P / SLICE_B / SLICE_I
  int wmb, hmb;
  int first_mb;
  int num_ref[2];        // num_ref_idx_lX_active
  int t8x8_mode;         // pps transform_8x8_mode_flag
  int slice_qp;
  int chroma_qp_offset;  // unused by the syntax, kept for the records
};

MIVC_HD int cabac_med3(int a, int b, int c) {
  const int mx = a > b ? a : b, mn = a < b ? a : b;
  return c > mx ? mx : (c < mn ? mn : c);
}

// Non-zero block mask of a record: bits 0-15 luma 4x4 blocks (blkIdx; I16x16: AC levels
// 1..15 only; 8x8 transform: 16-level chunk k of 8x8 block b8 at bit b8 * 4 + k), bit 16
// luma DC, bits 17 / 18 Cb / Cr DC, bits 19-26 chroma AC (comp * 4 + blk, levels 1..15).
enum : uint32_t { NZ_LUMA_DC = 1u << 16, NZ_CDC = 3u << 17, NZ_CAC = 0xFFu << 19 };
MIVC_HD uint32_t cabac_block_mask(const MbHeader& h, const int16_t* c) {
  uint32_t m = 0;
  const bool i16 = h.kind == MBK_I16x16;
  for (int b = 0; b < 16; ++b)
    for (int i = (i16 ? 1 : 0); i < 16; ++i)
      if (c[COEF_LUMA + b * 16 + i]) {
        m |= 1u << b;
        break;
      }
  for (int i = 0; i < 16; ++i)
    if (i16 && c[COEF_LUMA_DC + i]) m |= NZ_LUMA_DC;
  for (int k = 0; k < 2; ++k)
    for (int i = 0; i < 4; ++i)
      if (c[COEF_CHROMA_DC + k * 4 + i]) m |= 1u << (17 + k);
  for (int b = 0; b < 8; ++b)
    for (int i = 1; i < 16; ++i)
      if (c[COEF_CHROMA_AC + b * 16 + i]) {
        m |= 1u << (19 + b);
        break;
      }
  return m;
}

// Cbp of a record as the syntax codes it (luma bits of 8x8 blocks with non-zero levels,
// chroma 0/1/2; I16x16: luma 0 or 15), from its block mask.
MIVC_HD int cabac_mask_cbp(const MbHeader& h, uint32_t m) {
  if (h.kind == MBK_IPCM) return 0x2F;
  int luma = 0;
  for (int b8 = 0; b8 < 4; ++b8)
    if ((m >> (b8 * 4)) & 15u) luma |= 1 << b8;
  if (h.kind == MBK_I16x16 && luma) luma = 15;
  const int chroma = (m & NZ_CAC) ? 2 : ((m & NZ_CDC) ? 1 : 0);
  return luma | (chroma << 4);
}

MIVC_HD int cabac_record_cbp(const MbHeader& h, const int16_t* c) { return cabac_mask_cbp(h, cabac_block_mask(h, c)); }

// B mb_type value (Table 7-14) of an inter record (B16x16 / B16x8 / B8x16 / B8x8; the
// prediction list(s) of each partition are the lists with ref >= 0)
MIVC_HD int cabac_b_code(const MbHeader& h) {
  auto pred = [&](int q) { return (h.ref[0][q] >= 0 ? 1 : 0) | (h.ref[1][q] >= 0 ? 2 : 0); };
  if (h.kind == MBK_BDIRECT) return 0;
  if (h.kind == MBK_B8x8) return 22;
  if (h.kind == MBK_B16x16) return pred(0);
  const int p0 = pred(0), p1 = h.kind == MBK_B16x8 ? pred(2) : pred(1);
  // pair index (Table 7-14 order): (1,1) 0, (2,2) 1, (1,2) 2, (2,1) 3, (1,3) 4, (2,3) 5,
  // (3,1) 6, (3,2) 7, (3,3) 8 -- one nibble per (p0 * 4 + p1)
  const int idx = static_cast<int>((0x8760513042000000ull >> (4 * (p0 * 4 + p1))) & 15u);
  return 4 + 2 * idx + (h.kind == MBK_B16x8 ? 0 : 1);
}

// Partition layout of an inter MB kind: np partitions starting at quadrants qfirst[],
// width w4[] (4x4 units), shape 0 generic / 1 16x8 / 2 8x16, quadrant masks pm[].
// Partitions of an inter MB: np partitions of one shape (0: 16x16 when np == 1, else 8x8
// quadrants; 1: 16x8; 2: 8x16).  Per-partition values are computed, not tabulated: an array
// indexed by the partition loop counter made the GPU coder keep the struct in scratch memory.
struct CabacParts {
  int np, shape;
  MIVC_HD int qfirst(int p) const { return shape == 1 ? 2 * p : p; }  // first quadrant
  MIVC_HD int w4(int p) const { (void)p; return np == 1 || shape == 1 ? 4 : 2; }  // width in 4x4 blocks
  MIVC_HD int pm(int p) const {  // quadrant mask
    return np == 1 ? 0xF : (shape == 1 ? (p ? 0xC : 0x3) : (shape == 2 ? (p ? 0xA : 0x5) : 1 << p));
  }
};
MIVC_HD CabacParts cabac_parts(int kind) {
  CabacParts p{};
  if (kind == MBK_P16x16 || kind == MBK_B16x16 || kind == MBK_PSKIP) {
    p.np = 1; p.shape = 0;
  } else if (kind == MBK_P16x8 || kind == MBK_B16x8) {
    p.np = 2; p.shape = 1;
  } else if (kind == MBK_P8x16 || kind == MBK_B8x16) {
    p.np = 2; p.shape = 2;
  } else {
    p.np = 4; p.shape = 0;
  }
  return p;
}

// Neighbourhood of one MB inside a picture-sized table of records / states.
struct CabacView {
  int wmb, first_mb;
  int addr, mx, my;
  MIVC_HD void at(int a, int w, int first) {
    wmb = w;
    first_mb = first;
    addr = a;
    mx = a % w;
    my = a / w;
  }
  // address of the MB holding the 4x4 block (x4, y4) relative to this MB (-1..4), or -1
  MIVC_HD int mb_of(int x4, int y4) const {
    int n;
    if (y4 < 0) {
      if (my == 0) return -1;
      if (x4 < 0) n = mx > 0 ? addr - wmb - 1 : -1;
      else if (x4 < 4) n = addr - wmb;
      else n = mx + 1 < wmb ? addr - wmb + 1 : -1;
    } else if (y4 < 4) {
      if (x4 < 0) n = mx > 0 ? addr - 1 : -1;
      else if (x4 < 4) n = addr;
      else return -1;
    } else {
      return -1;
    }
    return n >= first_mb ? n : -1;
  }
  static MIVC_HD int quad_of(int x4, int y4) { return (((x4 + 4) & 3) >> 1) + 2 * (((y4 + 4) & 3) >> 1); }
  static MIVC_HD int rast_of(int x4, int y4) { return ((x4 + 4) & 3) + 4 * ((y4 + 4) & 3); }
};

// ---------------------------------------------------------------- motion vector prediction (8.4.1.3)
// From the records: partition with top-left 4x4 (bx, by), width w4, shape 0/1/2, part index;
// done = quadrants of MB v.addr already assigned (the record's own MVs count for them).
MIVC_HD void cabac_mvp(const CabacView& v, const MbHeader* hdr, int list, int ref, int bx, int by, int w4, int shape,
                       int part, int done, int out[2]) {
  struct N {
    bool avail;
    int ref;
    int mv[2];
  };
  auto get = [&](int x4, int y4) -> N {
    N n{false, -1, {0, 0}};
    const int a = v.mb_of(x4, y4);
    if (a < 0) return n;
    const int q = CabacView::quad_of(x4, y4);
    if (a == v.addr && !((done >> q) & 1)) return n;
    n.avail = true;
    const MbHeader& m = hdr[a];
    if (mbk_is_intra(m.kind)) return n;
    n.ref = m.ref[list][q];
    if (n.ref >= 0) {
      n.mv[0] = m.mv[list][q][0];
      n.mv[1] = m.mv[list][q][1];
    }
    return n;
  };
  N a = get(bx - 1, by), b = get(bx, by - 1), c = get(bx + w4, by - 1);
  if (!c.avail) c = get(bx - 1, by - 1);
  if (shape == 1) {
    if (part == 0 && b.ref == ref) { out[0] = b.mv[0]; out[1] = b.mv[1]; return; }
    if (part == 1 && a.ref == ref) { out[0] = a.mv[0]; out[1] = a.mv[1]; return; }
  } else if (shape == 2) {
    if (part == 0 && a.ref == ref) { out[0] = a.mv[0]; out[1] = a.mv[1]; return; }
    if (part == 1 && c.ref == ref) { out[0] = c.mv[0]; out[1] = c.mv[1]; return; }
  }
  if (!b.avail && !c.avail && a.avail) {
    b = a;
    c = a;
  }
  const int match = (a.ref == ref) + (b.ref == ref) + (c.ref == ref);
  if (match == 1) {
    const N& m = a.ref == ref ? a : (b.ref == ref ? b : c);
    out[0] = m.mv[0];
    out[1] = m.mv[1];
    return;
  }
  out[0] = cabac_med3(a.mv[0], b.mv[0], c.mv[0]);
  out[1] = cabac_med3(a.mv[1], b.mv[1], c.mv[1]);
}

// P_Skip motion (8.4.1.1) from the records
MIVC_HD void cabac_pskip_mv(const CabacView& v, const MbHeader* hdr, int out[2]) {
  out[0] = out[1] = 0;
  const int a = v.mb_of(-1, 0), b = v.mb_of(0, -1);
  if (a < 0 || b < 0) return;
  const MbHeader& A = hdr[a];
  const MbHeader& B = hdr[b];
  if (!mbk_is_intra(A.kind) && A.ref[0][1] == 0 && A.mv[0][1][0] == 0 && A.mv[0][1][1] == 0) return;
  if (!mbk_is_intra(B.kind) && B.ref[0][2] == 0 && B.mv[0][2][0] == 0 && B.mv[0][2][1] == 0) return;
  cabac_mvp(v, hdr, 0, 0, 0, 0, 4, 0, 0, 0, out);
}

// Coding state of MB addr from its record (and its neighbours' records).  mask: the
// record's non-zero block mask (cabac_block_mask).  dqp / prev_dqp_nz are set later by
// cabac_qp_chain.
MIVC_HD void cabac_prepare_mb(const CabacSliceInfo& si, const MbHeader* hdr, int addr, uint32_t mask, CabacNb& n) {
  CabacView v;
  v.at(addr, si.wmb, si.first_mb);
  const MbHeader& h = hdr[addr];
  const bool pslice = si.slice_type == SLICE_P, bslice = si.slice_type == SLICE_B;
  int kind = h.kind;
  const bool intra = mbk_is_intra(kind);
  const int cbp = cabac_mask_cbp(h, mask);
  n.avail = 1;
  n.skip = 0;
  n.cbp = static_cast<uint8_t>(cbp);
  n.t8x8 = 0;
  n.chroma_mode = 0;
  n.direct = 0;
  n.cbf_dc = 0;
  n.cbf_luma = 0;
  n.cbf_cac[0] = n.cbf_cac[1] = 0;
  n.i16_mode = h.i16_mode;
  n.qp = h.qp;
  n.mask = mask;
  n.dqp = 0;
  n.prev_dqp_nz = 0;
  n.b_code = 0;
  for (int l = 0; l < 2; ++l)
    for (int q = 0; q < 4; ++q) {
      n.ref[l][q] = intra ? -1 : h.ref[l][q];
      n.mv[l][q][0] = intra ? 0 : h.mv[l][q][0];
      n.mv[l][q][1] = intra ? 0 : h.mv[l][q][1];
      n.mvd[l][q][0] = n.mvd[l][q][1] = 0;
    }
  for (int i = 0; i < 16; ++i) n.i4[i] = 2;
  // ---- skip
  bool skip = false;
  if (pslice && (kind == MBK_P16x16 || kind == MBK_PSKIP) && cbp == 0 && h.ref[0][0] == 0) {
    int smv[2];
    cabac_pskip_mv(v, hdr, smv);
    skip = smv[0] == h.mv[0][0][0] && smv[1] == h.mv[0][0][1];
  } else if (bslice && kind == MBK_BDIRECT && cbp == 0) {
    skip = true;
  }
  if (skip) {
    n.skip = 1;
    n.kind = static_cast<uint8_t>(pslice ? MBK_PSKIP : MBK_BDIRECT);
    n.cbp = 0;
    if (bslice) n.direct = 0xF;
    return;
  }
  if (kind == MBK_PSKIP) kind = MBK_P16x16;
  n.kind = static_cast<uint8_t>(kind);
  if (bslice && !intra) n.b_code = static_cast<uint8_t>(cabac_b_code(h));
  // ---- intra modes
  if (kind == MBK_I4x4)
    for (int blk = 0; blk < 16; ++blk) n.i4[kBlkX[blk] + 4 * kBlkY[blk]] = h.i4_modes[blk];
  if (kind == MBK_I8x8)
    for (int b8 = 0; b8 < 4; ++b8)
      for (int k = 0; k < 4; ++k)
        n.i4[(b8 & 1) * 2 + (k & 1) + 4 * ((b8 >> 1) * 2 + (k >> 1))] = h.i4_modes[b8 * 4];
  if (intra) n.chroma_mode = h.chroma_mode;
  // ---- transform size as coded
  if (kind == MBK_I8x8) n.t8x8 = 1;
  else if (!intra && (cbp & 15) && si.t8x8_mode && (h.flags & MBF_T8x8)) n.t8x8 = 1;
  // ---- direct / mvd (partition order, list 0 then list 1)
  if (kind == MBK_BDIRECT) {
    n.direct = 0xF;
  } else if (!intra) {
    const CabacParts P = cabac_parts(kind);
    const int dir_mask = kind == MBK_B8x8 ? (h.sub_direct & 15) : 0;
    n.direct = static_cast<uint8_t>(dir_mask);
    for (int l = 0; l < 2; ++l) {
      int done = 0;
      for (int p = 0; p < P.np; ++p) {
        const int q = P.qfirst(p);
        if (((dir_mask >> q) & 1) || h.ref[l][q] < 0) {
          done |= P.pm(p);
          continue;
        }
        int pm[2];
        cabac_mvp(v, hdr, l, h.ref[l][q], (q & 1) * 2, (q >> 1) * 2, P.w4(p), P.shape, p, done, pm);
        const int dx = h.mv[l][q][0] - pm[0], dy = h.mv[l][q][1] - pm[1];
        for (int k = 0; k < 4; ++k)
          if ((P.pm(p) >> k) & 1) {
            n.mvd[l][k][0] = static_cast<int16_t>(dx);
            n.mvd[l][k][1] = static_cast<int16_t>(dy);
          }
        done |= P.pm(p);
      }
    }
  }
  // ---- coded_block_flags as neighbours see them
  const int cc = cbp >> 4;
  if (kind == MBK_I16x16 && (mask & NZ_LUMA_DC)) n.cbf_dc |= 1;
  if (cc) n.cbf_dc |= static_cast<uint8_t>(((mask >> 17) & 3u) << 1);
  if (cc == 2) {
    n.cbf_cac[0] = static_cast<uint8_t>((mask >> 19) & 15u);
    n.cbf_cac[1] = static_cast<uint8_t>((mask >> 23) & 15u);
  }
  for (int b8 = 0; b8 < 4; ++b8) {
    if (!((cbp >> b8) & 1)) continue;
    const int x4 = (b8 & 1) * 2, y4 = (b8 >> 1) * 2;
    if (n.t8x8) {
      n.cbf_luma |= static_cast<uint16_t>(0x33u << (x4 + 4 * y4));  // 8x8 blocks: flag inferred 1
      continue;
    }
    for (int b4 = 0; b4 < 4; ++b4) {
      const int blk = b8 * 4 + b4;
      if ((mask >> blk) & 1u) n.cbf_luma |= static_cast<uint16_t>(1u << (kBlkX[blk] + 4 * kBlkY[blk]));
    }
  }
}

// mb_qp_delta of every MB of a slice (QP_pred chain, 7.4.5) and the context flag of its
// first bin: nb[first_mb .. first_mb + n).  Serial; the GPU runs it as a scan.
MIVC_HD void cabac_qp_chain(const CabacSliceInfo& si, CabacNb* nb, int n) {
  int last_qp = si.slice_qp, last_nz = 0;
  for (int a = si.first_mb; a < si.first_mb + n; ++a) {
    CabacNb& m = nb[a];
    const bool has = !m.skip && (m.cbp != 0 || m.kind == MBK_I16x16);
    m.prev_dqp_nz = static_cast<uint8_t>(last_nz);
    if (has) {
      int d = m.qp - last_qp;
      if (d < -26) d += 52;
      if (d > 25) d -= 52;
      m.dqp = static_cast<int8_t>(d);
      last_qp = m.qp;
      last_nz = d != 0;
    } else {
      m.dqp = 0;
      last_nz = 0;
    }
  }
}

// ---------------------------------------------------------------- macroblock binariser
// Binarises MB addr (7.3.5 / 9.3.2 / 9.3.3.1) into sink E, followed by its
// end_of_slice_flag.  nb: prepared coding states of the whole picture.
template <class E>
struct CabacMbCoder {
  E& e;
  const CabacSliceInfo& si;
  const CabacNb* nb;
  CabacView v;
  const CabacNb* cur;

  MIVC_HD CabacMbCoder(E& e_, const CabacSliceInfo& s, const CabacNb* table) : e(e_), si(s), nb(table), cur(nullptr) {}

  MIVC_HD const CabacNb* nb_mb(int x4, int y4) const {
    const int a = v.mb_of(x4, y4);
    return a < 0 ? nullptr : &nb[a];
  }
  MIVC_HD const CabacNb* A() const { return nb_mb(-1, 0); }
  MIVC_HD const CabacNb* B() const { return nb_mb(0, -1); }

  // ---------------------------------------------------------------- syntax elements
  MIVC_HD void put_mb_skip(int skip) {
    const CabacNb* a = A();
    const CabacNb* b = B();
    const int inc = (a && !a->skip) + (b && !b->skip);
    e.decision((si.slice_type == SLICE_B ? CTX_MB_SKIP_B : CTX_MB_SKIP_P) + inc, skip);
  }

  // I mb_type (I slices: with the neighbour context of bin 0; P / B: the suffix)
  MIVC_HD void put_mb_type_i(int kind, int i16_mode, int cbp, bool islice) {
    if (islice) {
      const CabacNb* a = A();
      const CabacNb* b = B();
      const int inc = (a && a->kind != MBK_I4x4 && a->kind != MBK_I8x8) + (b && b->kind != MBK_I4x4 && b->kind != MBK_I8x8);
      e.decision(CTX_MB_TYPE_I + inc, kind == MBK_I4x4 || kind == MBK_I8x8 ? 0 : 1);
    } else {
      const int off = si.slice_type == SLICE_B ? CTX_MB_TYPE_B_INTRA : CTX_MB_TYPE_P_INTRA;
      e.decision(off, kind == MBK_I4x4 || kind == MBK_I8x8 ? 0 : 1);
    }
    if (kind == MBK_I4x4 || kind == MBK_I8x8) return;
    e.terminate(kind == MBK_IPCM ? 1 : 0);
    if (kind == MBK_IPCM) return;
    const int cl = (cbp & 15) ? 1 : 0, cc = cbp >> 4;
    if (islice) {
      e.decision(CTX_MB_TYPE_I + 3, cl);
      e.decision(CTX_MB_TYPE_I + 4, cc != 0);
      if (cc) e.decision(CTX_MB_TYPE_I + 5, cc == 2);
      e.decision(CTX_MB_TYPE_I + 6, (i16_mode >> 1) & 1);
      e.decision(CTX_MB_TYPE_I + 7, i16_mode & 1);
    } else {
      const int off = si.slice_type == SLICE_B ? CTX_MB_TYPE_B_INTRA : CTX_MB_TYPE_P_INTRA;
      e.decision(off + 1, cl);
      e.decision(off + 2, cc != 0);
      if (cc) e.decision(off + 2, cc == 2);
      e.decision(off + 3, (i16_mode >> 1) & 1);
      e.decision(off + 3, i16_mode & 1);
    }
  }

  MIVC_HD void put_mb_type_p(int kind, int i16_mode, int cbp) {
    switch (kind) {
      case MBK_P16x16: e.decision(14, 0); e.decision(15, 0); e.decision(16, 0); return;
      case MBK_P16x8:  e.decision(14, 0); e.decision(15, 1); e.decision(17, 1); return;
      case MBK_P8x16:  e.decision(14, 0); e.decision(15, 1); e.decision(17, 0); return;
      case MBK_P8x8:   e.decision(14, 0); e.decision(15, 0); e.decision(16, 1); return;
      default:
        e.decision(14, 1);
        put_mb_type_i(kind, i16_mode, cbp, false);
    }
  }

  // B mb_type (Table 9-37(b)); code: B mb_type value 0..22, 23 = intra prefix
  MIVC_HD void put_mb_type_b(int kind, int i16_mode, int cbp, int code) {
    const CabacNb* a = A();
    const CabacNb* b = B();
    const int inc = (a && !a->skip && a->kind != MBK_BDIRECT) + (b && !b->skip && b->kind != MBK_BDIRECT);
    if (code == 0) {
      e.decision(CTX_MB_TYPE_B + inc, 0);
      return;
    }
    e.decision(CTX_MB_TYPE_B + inc, 1);
    if (code <= 2) {  // B_L0_16x16 "100", B_L1_16x16 "101"
      e.decision(CTX_MB_TYPE_B + 3, 0);
      e.decision(CTX_MB_TYPE_B + 5, code - 1);
      return;
    }
    e.decision(CTX_MB_TYPE_B + 3, 1);
    if (code <= 10) {  // 1 1 0 b b b
      const int v3 = code - 3;
      e.decision(CTX_MB_TYPE_B + 4, 0);
      e.decision(CTX_MB_TYPE_B + 5, (v3 >> 2) & 1);
      e.decision(CTX_MB_TYPE_B + 5, (v3 >> 1) & 1);
      e.decision(CTX_MB_TYPE_B + 5, v3 & 1);
      return;
    }
    e.decision(CTX_MB_TYPE_B + 4, 1);
    if (code == 11 || code == 22 || code == 23) {  // 1 1 1 1 1 0 / 1 1 1 1 1 1 / 1 1 1 1 0 1
      e.decision(CTX_MB_TYPE_B + 5, 1);
      e.decision(CTX_MB_TYPE_B + 5, code == 23 ? 0 : 1);
      e.decision(CTX_MB_TYPE_B + 5, code == 11 ? 0 : 1);
      if (code == 23) put_mb_type_i(kind, i16_mode, cbp, false);
      return;
    }
    // 12..21: bins 3..6 = the 4-bit value code - 12
    const int v4 = code - 12;
    e.decision(CTX_MB_TYPE_B + 5, (v4 >> 3) & 1);
    e.decision(CTX_MB_TYPE_B + 5, (v4 >> 2) & 1);
    e.decision(CTX_MB_TYPE_B + 5, (v4 >> 1) & 1);
    e.decision(CTX_MB_TYPE_B + 5, v4 & 1);
  }

  MIVC_HD void put_sub_mb_type_b(int code) {
    // Table 9-38: 0 "0", 1 "100", 2 "101", 3..6 "110xx", 7..10 "1110xx", 11 "11110", 12 "11111"
    if (code == 0) { e.decision(CTX_SUB_MB_B, 0); return; }
    e.decision(CTX_SUB_MB_B, 1);
    if (code <= 2) {
      e.decision(CTX_SUB_MB_B + 1, 0);
      e.decision(CTX_SUB_MB_B + 3, code - 1);
      return;
    }
    e.decision(CTX_SUB_MB_B + 1, 1);
    if (code <= 6) {
      e.decision(CTX_SUB_MB_B + 2, 0);
      e.decision(CTX_SUB_MB_B + 3, ((code - 3) >> 1) & 1);
      e.decision(CTX_SUB_MB_B + 3, (code - 3) & 1);
      return;
    }
    e.decision(CTX_SUB_MB_B + 2, 1);
    if (code >= 11) {
      e.decision(CTX_SUB_MB_B + 3, 1);
      e.decision(CTX_SUB_MB_B + 3, code - 11);
      return;
    }
    e.decision(CTX_SUB_MB_B + 3, 0);
    e.decision(CTX_SUB_MB_B + 3, ((code - 7) >> 1) & 1);
    e.decision(CTX_SUB_MB_B + 3, (code - 7) & 1);
  }

  MIVC_HD void put_ref_idx(int list, int q, int ref) {
    const int x4 = (q & 1) * 2, y4 = (q >> 1) * 2;
    auto cond = [&](int xn, int yn) -> int {
      const CabacNb* m = nb_mb(xn, yn);
      if (!m || m->skip || mbk_is_intra(m->kind)) return 0;
      const int qn = CabacView::quad_of(xn, yn);
      if ((m->direct >> qn) & 1) return 0;
      return m->ref[list][qn] > 0;
    };
    const int inc = cond(x4 - 1, y4) + 2 * cond(x4, y4 - 1);
    e.decision(CTX_REF_IDX + inc, ref > 0);
    if (ref == 0) return;
    for (int k = 1; k < ref; ++k) e.decision(CTX_REF_IDX + (k == 1 ? 4 : 5), 1);
    e.decision(CTX_REF_IDX + (ref == 1 ? 4 : 5), 0);
  }

  MIVC_HD void put_mvd(int list, int q, int comp, int val) {
    const int x4 = (q & 1) * 2, y4 = (q >> 1) * 2;
    auto absn = [&](int xn, int yn) -> int {
      const CabacNb* m = nb_mb(xn, yn);
      if (!m) return 0;
      const int d = m->mvd[list][CabacView::quad_of(xn, yn)][comp];
      return d < 0 ? -d : d;
    };
    const int sum = absn(x4 - 1, y4) + absn(x4, y4 - 1);
    const int base = comp ? CTX_MVD_Y : CTX_MVD_X;
    const int inc0 = sum < 3 ? 0 : (sum > 32 ? 2 : 1);
    const int av = val < 0 ? -val : val;
    const int pre = av < 9 ? av : 9;
    e.decision(base + inc0, pre > 0);
    if (pre > 0) {
      for (int k = 1; k < pre; ++k) e.decision(base + (k < 4 ? k + 2 : 6), 1);
      if (pre < 9) e.decision(base + (pre < 4 ? pre + 2 : 6), 0);
      if (av >= 9) e.bypass_eg(static_cast<uint32_t>(av - 9), 3);
      e.bypass(val < 0);
    }
  }

  MIVC_HD void put_cbp(int cbp) {
    const CabacNb* a = A();
    const CabacNb* b = B();
    // unavailable neighbours and I_PCM count as "all luma blocks coded" / chroma 0 / 2
    const int la = a ? (a->kind == MBK_IPCM ? 0x2F : a->cbp) : 0x0F;
    const int lb = b ? (b->kind == MBK_IPCM ? 0x2F : b->cbp) : 0x0F;
    for (int b8 = 0; b8 < 4; ++b8) {
      const int ca = (b8 & 1) ? ((cbp >> (b8 - 1)) & 1) : ((la >> (b8 + 1)) & 1);
      const int cb = (b8 & 2) ? ((cbp >> (b8 - 2)) & 1) : ((lb >> (b8 + 2)) & 1);
      e.decision(CTX_CBP_LUMA + (ca ? 0 : 1) + 2 * (cb ? 0 : 1), (cbp >> b8) & 1);
    }
    const int ca = a ? (a->kind == MBK_IPCM ? 2 : (a->cbp >> 4)) : 0;
    const int cb = b ? (b->kind == MBK_IPCM ? 2 : (b->cbp >> 4)) : 0;
    const int cc = cbp >> 4;
    e.decision(CTX_CBP_CHROMA + (ca > 0) + 2 * (cb > 0), cc > 0);
    if (cc) e.decision(CTX_CBP_CHROMA + 4 + (ca == 2) + 2 * (cb == 2), cc == 2);
  }

  MIVC_HD void put_qp_delta(int d, int prev_nz) {
    const int m = d > 0 ? 2 * d - 1 : -2 * d;
    e.decision(CTX_QP_DELTA + (prev_nz ? 1 : 0), m > 0);
    if (m > 0) {
      for (int k = 1; k < m; ++k) e.decision(CTX_QP_DELTA + (k == 1 ? 2 : 3), 1);
      e.decision(CTX_QP_DELTA + (m == 1 ? 2 : 3), 0);
    }
  }

  MIVC_HD void put_chroma_mode(int mode) {
    const CabacNb* a = A();
    const CabacNb* b = B();
    const int inc = (a && mbk_is_intra(a->kind) && a->kind != MBK_IPCM && a->chroma_mode != 0) +
                    (b && mbk_is_intra(b->kind) && b->kind != MBK_IPCM && b->chroma_mode != 0);
    e.decision(CTX_CHROMA_PRED + inc, mode > 0);
    if (mode > 0) {
      e.decision(CTX_CHROMA_PRED + 3, mode > 1);
      if (mode > 1) e.decision(CTX_CHROMA_PRED + 3, mode > 2);
    }
  }

  // predIntraNxNPredMode of the 4x4 block at raster (x4, y4) (8.3.1.1 / 8.3.2.1)
  MIVC_HD int pred_intra_mode(int x4, int y4) const {
    const CabacNb* a = nb_mb(x4 - 1, y4);
    const CabacNb* b = nb_mb(x4, y4 - 1);
    if (!a || !b) return 2;
    const int ma = (a->kind == MBK_I4x4 || a->kind == MBK_I8x8) ? a->i4[CabacView::rast_of(x4 - 1, y4)] : 2;
    const int mb = (b->kind == MBK_I4x4 || b->kind == MBK_I8x8) ? b->i4[CabacView::rast_of(x4, y4 - 1)] : 2;
    return ma < mb ? ma : mb;
  }
  MIVC_HD void put_intra_mode(int mode, int pred) {
    if (mode == pred) {
      e.decision(CTX_PREV_INTRA, 1);
      return;
    }
    e.decision(CTX_PREV_INTRA, 0);
    const int rem = mode < pred ? mode : mode - 1;
    e.decision(CTX_REM_INTRA, rem & 1);
    e.decision(CTX_REM_INTRA, (rem >> 1) & 1);
    e.decision(CTX_REM_INTRA, (rem >> 2) & 1);
  }

  MIVC_HD void put_t8x8(int flag) {
    const CabacNb* a = A();
    const CabacNb* b = B();
    e.decision(CTX_T8x8 + (a && a->t8x8) + (b && b->t8x8), flag);
  }

  // ---------------------------------------------------------------- residual_block_cabac
  // c: n coefficients in scan order (levelListIdx order); cat 0..5; cbf_inc < 0: no flag;
  // nonzero = false: the block is known to be all zero (only coded_block_flag = 0)
  MIVC_HD void put_block(const int16_t* c, int n, int cat, int cbf_inc, bool nonzero) {
    if (!nonzero) {
      if (cbf_inc >= 0) e.decision(CTX_CBF + kCbfCatOffset[cat] + cbf_inc, 0);
      return;
    }
    // levels are read in place (no local copy: on the GPU a 64-entry array lives in scratch
    // memory -- 256 bytes per lane of cabac_bins / cabac_count)
    int last = -1;
    for (int i = 0; i < n; ++i)
      if (c[i]) last = i;
    if (cbf_inc >= 0) {
      e.decision(CTX_CBF + kCbfCatOffset[cat] + cbf_inc, last >= 0);
      if (last < 0) return;
    }
    for (int i = 0; i < n - 1; ++i) {
      const int sig = c[i] != 0;
      int sctx, lctx;
      if (cat == 5) {
        sctx = CTX_SIG8x8 + kSig8x8Frame[i];
        lctx = CTX_LAST8x8 + kLast8x8Frame[i];
      } else {
        const int inc = cat == 3 ? (i < 2 ? i : 2) : i;
        sctx = CTX_SIG + kSigCatOffset[cat] + inc;
        lctx = CTX_LAST + kSigCatOffset[cat] + inc;
      }
      e.decision(sctx, sig);
      if (sig) {
        e.decision(lctx, i == last);
        if (i == last) break;
      }
    }
    const int abase = cat == 5 ? CTX_ABS8x8 : CTX_ABS + kAbsCatOffset[cat];
    const int gmax = cat == 3 ? 3 : 4;
    int ngt1 = 0, neq1 = 0;
    for (int i = last; i >= 0; --i) {
      const int val = c[i];
      if (!val) continue;
      const int a1 = (val < 0 ? -val : val) - 1;
      e.decision(abase + (ngt1 ? 0 : (neq1 + 1 < 4 ? neq1 + 1 : 4)), a1 > 0);
      if (a1 > 0) {
        const int ctx1 = abase + 5 + (ngt1 < gmax ? ngt1 : gmax);
        const int pre = a1 < 14 ? a1 : 14;
        for (int k = 1; k < pre; ++k) e.decision(ctx1, 1);
        if (pre < 14) e.decision(ctx1, 0);
        else e.bypass_eg(static_cast<uint32_t>(a1 - 14), 0);
        ++ngt1;
      } else {
        ++neq1;
      }
      e.bypass(val < 0);
    }
  }

  // coded_block_flag ctxIdxInc of a luma 4x4 block at raster (x4, y4) of the current MB
  MIVC_HD int cbf_luma_inc(int x4, int y4, bool intra) const {
    auto cond = [&](int xn, int yn) -> int {
      const CabacNb* m = nb_mb(xn, yn);
      if (!m) return intra ? 1 : 0;
      if (m->kind == MBK_IPCM) return 1;
      return (m->cbf_luma >> CabacView::rast_of(xn, yn)) & 1;
    };
    return cond(x4 - 1, y4) + 2 * cond(x4, y4 - 1);
  }
  MIVC_HD int cbf_dc_inc(int bit, bool intra) const {  // bit 0 luma DC, 1 Cb, 2 Cr
    auto cond = [&](const CabacNb* m) -> int {
      if (!m) return intra ? 1 : 0;
      if (m->kind == MBK_IPCM) return 1;
      return (m->cbf_dc >> bit) & 1;
    };
    return cond(A()) + 2 * cond(B());
  }
  MIVC_HD int cbf_cac_inc(int comp, int cx, int cy, bool intra) const {
    auto cond = [&](const CabacNb* m, int blk) -> int {
      if (!m) return intra ? 1 : 0;
      if (m->kind == MBK_IPCM) return 1;
      return (m->cbf_cac[comp] >> blk) & 1;
    };
    const int a = cx > 0 ? cond(cur, cy * 2) : cond(A(), cy * 2 + 1);
    const int b = cy > 0 ? cond(cur, cx) : cond(B(), 2 + cx);
    return a + 2 * b;
  }

  MIVC_HD void put_inter_pred(const MbHeader& h, int kind) {
    if (kind == MBK_BDIRECT) return;  // B_Direct_16x16: no mb_pred (motion is derived)
    const bool bslice = si.slice_type == SLICE_B;
    const CabacParts P = cabac_parts(kind);
    const bool sub8 = P.np == 4;
    const int dir_mask = cur->direct;
    if (sub8) {
      if (bslice) {
        for (int s = 0; s < 4; ++s) {
          int code = 0;
          if (!((dir_mask >> s) & 1)) {
            const bool l0 = h.ref[0][s] >= 0, l1 = h.ref[1][s] >= 0;
            code = (l0 && l1) ? 3 : (l1 ? 2 : 1);
          }
          put_sub_mb_type_b(code);
        }
      } else {
        for (int s = 0; s < 4; ++s) e.decision(CTX_SUB_MB_P, 1);  // P_L0_8x8
      }
    }
    for (int l = 0; l < 2; ++l) {
      if (si.num_ref[l] <= 1) continue;
      for (int p = 0; p < P.np; ++p) {
        const int q = P.qfirst(p);
        if (((dir_mask >> q) & 1) || h.ref[l][q] < 0) continue;
        put_ref_idx(l, q, h.ref[l][q]);
      }
    }
    for (int l = 0; l < 2; ++l)
      for (int p = 0; p < P.np; ++p) {
        const int q = P.qfirst(p);
        if (((dir_mask >> q) & 1) || h.ref[l][q] < 0) continue;
        put_mvd(l, q, 0, cur->mvd[l][q][0]);
        put_mvd(l, q, 1, cur->mvd[l][q][1]);
      }
  }

  // ---------------------------------------------------------------- one macroblock
  MIVC_HD void code_mb(int addr, const MbHeader& h, const int16_t* c, bool last_in_slice) {
    v.at(addr, si.wmb, si.first_mb);
    cur = &nb[addr];
    const bool pslice = si.slice_type == SLICE_P, bslice = si.slice_type == SLICE_B;
    if (pslice || bslice) put_mb_skip(cur->skip);
    if (!cur->skip) code_mb_layer(h, c);
    e.terminate(last_in_slice ? 1 : 0);
  }

  MIVC_HD void code_mb_layer(const MbHeader& h, const int16_t* c) {
    const bool pslice = si.slice_type == SLICE_P, bslice = si.slice_type == SLICE_B;
    const int kind = cur->kind;
    const int cbp = cur->cbp;
    const uint32_t mask = cur->mask;
    const bool intra = mbk_is_intra(kind);
    // ---- mb_type
    if (pslice) put_mb_type_p(kind, h.i16_mode, cbp);
    else if (bslice) put_mb_type_b(kind, h.i16_mode, cbp, intra ? 23 : cur->b_code);
    else put_mb_type_i(kind, h.i16_mode, cbp, true);
    // ---- prediction
    if (kind == MBK_I4x4 || kind == MBK_I8x8) {
      if (si.t8x8_mode) put_t8x8(kind == MBK_I8x8);
      if (kind == MBK_I4x4) {
        for (int blk = 0; blk < 16; ++blk) {
          const int x4 = kBlkX[blk], y4 = kBlkY[blk];
          put_intra_mode(h.i4_modes[blk], pred_intra_mode(x4, y4));
        }
      } else {
        for (int b8 = 0; b8 < 4; ++b8) put_intra_mode(h.i4_modes[b8 * 4], pred_intra_mode((b8 & 1) * 2, (b8 >> 1) * 2));
      }
    }
    if (intra) put_chroma_mode(h.chroma_mode);
    else put_inter_pred(h, kind);
    // ---- coded_block_pattern, transform size
    if (kind != MBK_I16x16) {
      put_cbp(cbp);
      if ((cbp & 15) && si.t8x8_mode && !intra) put_t8x8(cur->t8x8);
    }
    if (cbp == 0 && kind != MBK_I16x16) return;
    put_qp_delta(cur->dqp, cur->prev_dqp_nz);
    // ---- residual: luma
    if (kind == MBK_I16x16) put_block(c + COEF_LUMA_DC, 16, 0, cbf_dc_inc(0, true), (mask & NZ_LUMA_DC) != 0);
    for (int b8 = 0; b8 < 4; ++b8) {
      if (!((cbp >> b8) & 1)) continue;
      if (cur->t8x8) {
        put_block(c + COEF_LUMA + b8 * 64, 64, 5, -1, true);
        continue;
      }
      for (int b4 = 0; b4 < 4; ++b4) {
        const int blk = b8 * 4 + b4;
        const int inc = cbf_luma_inc(kBlkX[blk], kBlkY[blk], intra);
        const bool nzb = (mask >> blk) & 1u;
        if (kind == MBK_I16x16) put_block(c + COEF_LUMA + blk * 16 + 1, 15, 1, inc, nzb);
        else put_block(c + COEF_LUMA + blk * 16, 16, 2, inc, nzb);
      }
    }
    // ---- chroma
    const int cc = cbp >> 4;
    if (cc)
      for (int comp = 0; comp < 2; ++comp)
        put_block(c + COEF_CHROMA_DC + comp * 4, 4, 3, cbf_dc_inc(1 + comp, intra), ((mask >> (17 + comp)) & 1u) != 0);
    if (cc == 2)
      for (int comp = 0; comp < 2; ++comp)
        for (int b = 0; b < 4; ++b)
          put_block(c + COEF_CHROMA_AC + (comp * 4 + b) * 16 + 1, 15, 4, cbf_cac_inc(comp, b & 1, b >> 1, intra),
                    ((mask >> (19 + comp * 4 + b)) & 1u) != 0);
  }
};

// One recorded symbol through the arithmetic coder.
MIVC_HD void cabac_code_symbol(CabacEncoder& e, uint16_t s) {
  if (!(s & 0x8000u)) e.decision(s & 0x1FF, (s >> 9) & 1);
  else if (!(s & 0x4000u)) e.bypass_bits(s & 0x3FFu, (s >> 10) & 15);
  else e.terminate(s & 1);
}

// The GPU's serial stage: CabacEncoder over recorded symbols with one branch-free update
// for the three common symbol kinds, so the 64 slices of a wave (one per lane) do not
// serialise on divergent paths.  Decision, bypass batch and terminate(0) (= the MPS path
// with rLPS 2 and no context) share
//     low' = (low + add) << n + range * bypass_bits,  range' = new_range << n;
// terminate(1), the last symbol of every slice, is finish().  Context states are read
// at st[ctx * stride] (the GPU keeps one LDS column per lane); lps / trans are the
// flattened Table 9-44 / transIdxLPS.
//
// `low` is 64-bit so bytes can be drained lazily: a symbol adds at most 10 bits, so after
// a drain (nbits < 8) four more symbols fit (< 48 + 10 bits) before the next one.  A wave
// then takes the divergent byte-output path once per 4 symbols instead of once per symbol.
// Out: byte9(v) takes one output byte whose bit 8 is a carry into the bytes before it
// (false: a carry with no byte to take it); finish() ends the byte stream.
template <class Out>
struct CabacSymbolCoder {
  uint64_t low;
  uint32_t range;
  int nbits, bad;
  Out out;

  MIVC_HD void init() {
    low = 0;
    range = 510;
    nbits = -1;
    bad = 0;
  }
  MIVC_HD void drain() {
    while (nbits >= 8) {
      const int sh = nbits + 2;
      const uint32_t v = static_cast<uint32_t>(low >> sh);
      low &= (1ull << sh) - 1ull;
      nbits -= 8;
      if (!out.byte9(v)) bad = 1;
    }
  }
  MIVC_HD void step_nodrain(uint32_t sym, uint8_t* st, int stride, const uint8_t* lps, const uint8_t* trans) {
    const bool dec = !(sym & 0x8000u);
    const bool byp = (sym & 0xC000u) == 0x8000u;
    uint8_t* sp = st + (dec ? (sym & 0x1FFu) : 0u) * static_cast<uint32_t>(stride);
    const int sv = dec ? *sp : 0;
    int pst = sv >> 1, mps = sv & 1;
    const uint32_t rlps = dec ? lps[pst * 4 + ((range >> 6) & 3)] : 2u;
    const uint32_t r1 = range - rlps;
    const bool lpsb = dec && static_cast<int>((sym >> 9) & 1u) != mps;
    const uint32_t nr = lpsb ? rlps : r1;
    const uint32_t add = lpsb ? r1 : 0u;
    if (dec) {
      const int up = pst < 62 ? pst + 1 : 62;
      const int dn = trans[pst];
      mps ^= (lpsb && pst == 0) ? 1 : 0;
      *sp = static_cast<uint8_t>(((lpsb ? dn : up) << 1) | mps);
    }
    const int shd = cabac_clz32(nr) - 23;
    const int n = byp ? static_cast<int>((sym >> 10) & 15u) : (shd > 0 ? shd : 0);
    low = ((low + add) << n) + (byp ? static_cast<uint64_t>(range) * (sym & 0x3FFu) : 0ull);
    range = byp ? range : (nr << n);
    nbits += n;
  }
  MIVC_HD void step(uint32_t sym, uint8_t* st, int stride, const uint8_t* lps, const uint8_t* trans) {
    step_nodrain(sym, st, stride, lps, trans);
    if (nbits >= 8) drain();
  }
  // EncodeTerminate(1) + EncodeFlush + rbsp_stop_one_bit + alignment (CabacEncoder::terminate)
  MIVC_HD void finish() {
    drain();
    range -= 2;
    low += range;
    range = 2;
    low <<= 7;
    nbits += 7;
    drain();
    low |= 0x80u;
    low <<= 3;
    nbits += 3;
    drain();
    if (nbits > 0) {
      low <<= 8 - nbits;
      nbits = 8;
      drain();
    }
    out.finish();
  }
};

// Byte output with x264-style carry resolution: the last non-0xFF byte is held back with
// a count of 0xFF bytes after it until a later byte shows whether a carry reaches them.
template <class Sink>
struct CabacPendingOut {
  Sink sink;  // put(int byte)
  int pend = -1, nff = 0;
  MIVC_HD bool byte9(uint32_t v) {
    const int b = static_cast<int>(v & 0xFFu);
    bool ok = true;
    if (v >> 8) {
      if (pend < 0) ok = false;
      if (nff > 0) {
        sink.put(pend + 1);
        for (int k = 0; k < nff - 1; ++k) sink.put(0);
        pend = 0;
        nff = 0;
      } else {
        pend += 1;
      }
    }
    if (b == 0xFF) {
      ++nff;
    } else {
      if (pend >= 0) {
        sink.put(pend);
        for (int k = 0; k < nff; ++k) sink.put(0xFF);
      }
      pend = b;
      nff = 0;
    }
    return ok;
  }
  MIVC_HD void finish() {
    if (pend >= 0) sink.put(pend);
    for (int k = 0; k < nff; ++k) sink.put(0xFF);
    pend = -1;
    nff = 0;
  }
};

struct CabacBufRef {
  CabacBuf* b;
  MIVC_HD void put(int v) { b->put(v); }
};

// ---------------------------------------------------------------- serial slice writer (host)
struct CabacSliceStats {
  int skipped = 0, intra = 0, inter = 0;
};

// Code MB records [first_mb, first_mb + n) of one picture as slice data into `out`
// (the caller writes the byte-aligned slice header and the NAL framing).  nb: scratch
// of width_mbs * height_mbs entries; masks: optional precomputed block masks.
MIVC_HD size_t cabac_write_slice_data(const CabacSliceInfo& si, CabacNb* nb, uint8_t* states, CabacBuf* out,
                                      const MbHeader* hdr, const int16_t* coef, int n, CabacEncoder* enc_out = nullptr,
                                      CabacSliceStats* st = nullptr) {
  const int end = si.first_mb + n;
  for (int a = si.first_mb; a < end; ++a)
    cabac_prepare_mb(si, hdr, a, cabac_block_mask(hdr[a], coef + static_cast<size_t>(a) * kCoefPerMb), nb[a]);
  cabac_qp_chain(si, nb, n);
  CabacEncoder e;
  cabac_init_contexts(states, si.slice_type == SLICE_I ? 0 : 1 /* cabac_init_idc 0 */, si.slice_qp);
  e.init(states, out);
  CabacMbCoder<CabacEncoder> coder(e, si, nb);
  for (int a = si.first_mb; a < end; ++a) {
    coder.code_mb(a, hdr[a], coef + static_cast<size_t>(a) * kCoefPerMb, a == end - 1);
    if (st) {
      if (nb[a].skip) ++st->skipped;
      else if (mbk_is_intra(nb[a].kind)) ++st->intra;
      else ++st->inter;
    }
  }
  if (enc_out) *enc_out = e;
  return out->n;
}

// The same slice data through the GPU decomposition: every MB binarised on its own into
// symbols (any order), then the symbols arithmetic-coded in MB order.  Must produce the
// bytes of cabac_write_slice_data (a CPU test pins it).  syms: scratch >= total symbols.
inline size_t cabac_write_slice_data_symbols(const CabacSliceInfo& si, CabacNb* nb, uint8_t* states, CabacBuf* out,
                                             const MbHeader* hdr, const int16_t* coef, int n, uint16_t* syms,
                                             size_t cap_syms, int* nsyms_out) {
  const int end = si.first_mb + n;
  for (int a = end - 1; a >= si.first_mb; --a)  // reverse order: nothing depends on coding order
    cabac_prepare_mb(si, hdr, a, cabac_block_mask(hdr[a], coef + static_cast<size_t>(a) * kCoefPerMb), nb[a]);
  cabac_qp_chain(si, nb, n);
  size_t total = 0;
  for (int a = si.first_mb; a < end; ++a) {
    CabacSymbolPacker<CabacCountEmit> cnt;
    CabacMbCoder<CabacSymbolPacker<CabacCountEmit>> c1(cnt, si, nb);
    c1.code_mb(a, hdr[a], coef + static_cast<size_t>(a) * kCoefPerMb, a == end - 1);
    cnt.flush_bypass();
    if (total + cnt.out.n > cap_syms) return 0;
    CabacSymbolPacker<CabacStoreEmit> st;
    st.out.p = syms + total;
    CabacMbCoder<CabacSymbolPacker<CabacStoreEmit>> c2(st, si, nb);
    c2.code_mb(a, hdr[a], coef + static_cast<size_t>(a) * kCoefPerMb, a == end - 1);
    st.flush_bypass();
    total += st.out.n;
  }
  if (nsyms_out) *nsyms_out = static_cast<int>(total);
  if (total == 0 || syms[total - 1] != 0xC001u) return 0;  // slices end in end_of_slice_flag = 1
  cabac_init_contexts(states, si.slice_type == SLICE_I ? 0 : 1, si.slice_qp);
  CabacSymbolCoder<CabacPendingOut<CabacBufRef>> e;
  e.out.sink.b = out;
  e.init();
  for (size_t i = 0; i + 1 < total; ++i) {  // drained every 4 symbols, as the GPU coder does
    e.step_nodrain(syms[i], states, 1, &kCabacRangeLPS[0][0], kCabacTransLPS);
    if ((i & 3) == 3) e.drain();
  }
  e.finish();
  return e.bad ? 0 : out->n;
}

}  // namespace h264
}  // namespace mivc
