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
// * CabacMbWriter: macroblock_layer() / residual() binarisation and context selection
//   (clauses 9.3.2, 9.3.3.1) from MbHeader records (h264_mb.h), for I, P and B slices,
//   4x4 and 8x8 transforms, partitions at 8x8 granularity.
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

// ---------------------------------------------------------------- neighbour context
// What later macroblocks need to know about a coded one (kept per MB in a row buffer).
struct alignas(8) CabacNb {
  uint8_t avail;       // coded in this slice
  uint8_t kind;        // MbKind as coded (MBK_PSKIP for P_Skip)
  uint8_t skip;        // mb_skip_flag
  uint8_t cbp;         // luma bits 0-3 | chroma << 4 (I_PCM: 0x2F)
  uint8_t t8x8;
  uint8_t chroma_mode; // intra_chroma_pred_mode (0 for inter / I_PCM)
  uint8_t direct;      // bit q: quadrant q predicted in direct mode
  uint8_t cbf_dc;      // bit0 luma DC, bit1 Cb DC, bit2 Cr DC
  uint16_t cbf_luma;   // raster 4x4 (x + 4y): coded_block_flag as seen by neighbours
  uint8_t cbf_cac[2];  // chroma AC, bit = raster 2x2 block
  int8_t ref[2][4];    // per quadrant and list (-1: list unused / intra)
  int16_t mv[2][4][2];
  uint8_t mvd[2][4][2];  // min(|mvd|, 255) per quadrant, list, component
  uint8_t i4[16];      // Intra4x4/8x8 pred mode per raster 4x4 (2 = DC for non-NxN)
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

// Macroblock-layer writer.  The caller owns the row buffer (wmb CabacNb entries) and
// codes MBs of one slice in raster order; see cabac_write_slice_data for the loop.
struct CabacMbWriter {
  CabacEncoder e;
  CabacSliceInfo si;
  CabacNb* row;        // [wmb]: entry mx is MB (mx, my-1) before MB (mx, my) is coded
  CabacNb tl;          // MB (mx-1, my-1), saved before row[mx-1] was overwritten
  CabacNb cur;         // the MB being coded
  int last_qp;         // QP_Y of the previous MB in decoding order
  int last_dqp;        // that MB coded a non-zero mb_qp_delta
  int mx, my;
  uint32_t mbmask;     // non-zero block mask of the MB being coded
  // statistics
  int n_skip, n_intra, n_inter;

  // states_ready: the caller already initialised the contexts (the GPU kernel does it
  // with all lanes); row_ready: the row buffer is already marked unavailable
  MIVC_HD void begin(const CabacSliceInfo& s, CabacNb* rowbuf, uint8_t* states, CabacBuf* out,
                     bool states_ready = false, bool row_ready = false) {
    si = s;
    row = rowbuf;
    if (!row_ready)
      for (int i = 0; i < s.wmb; ++i) row[i].avail = 0;
    tl.avail = 0;
    if (!states_ready) cabac_init_contexts(states, s.slice_type == SLICE_I ? 0 : 1 /* cabac_init_idc 0 */, s.slice_qp);
    e.init(states, out);
    last_qp = s.slice_qp;
    last_dqp = 0;
    n_skip = n_intra = n_inter = 0;
  }

  // ---------------------------------------------------------------- neighbour access
  // MB holding the 4x4 block at (x4, y4) relative to the current MB (x4, y4 in -1..4);
  // nullptr when unavailable.  Blocks inside the current MB return &cur.
  MIVC_HD const CabacNb* nb_mb(int x4, int y4) const {
    if (y4 < 0) {
      if (x4 < 0) return (mx > 0 && tl.avail) ? &tl : nullptr;
      if (x4 < 4) return row[mx].avail ? &row[mx] : nullptr;
      return (mx + 1 < si.wmb && row[mx + 1].avail) ? &row[mx + 1] : nullptr;
    }
    if (y4 > 3) return nullptr;
    if (x4 < 0) return (mx > 0 && row[mx - 1].avail) ? &row[mx - 1] : nullptr;
    if (x4 > 3) return nullptr;
    return &cur;
  }
  MIVC_HD bool top_avail() const { return row[mx].avail != 0; }
  MIVC_HD bool left_avail() const { return mx > 0 && row[mx - 1].avail; }
  MIVC_HD const CabacNb* A() const { return left_avail() ? &row[mx - 1] : nullptr; }
  MIVC_HD const CabacNb* B() const { return top_avail() ? &row[mx] : nullptr; }

  static MIVC_HD int quad_of(int x4, int y4) { return (((x4 + 4) & 3) >> 1) + 2 * (((y4 + 4) & 3) >> 1); }
  static MIVC_HD int rast_of(int x4, int y4) { return ((x4 + 4) & 3) + 4 * ((y4 + 4) & 3); }

  // ---------------------------------------------------------------- motion vector prediction (8.4.1.3)
  // partition with top-left 4x4 (bx, by), width w4 (4x4 units), shape 0 generic, 1 16x8,
  // 2 8x16; done = quadrants of the current MB already assigned (bit mask).
  MIVC_HD void mvp(int list, int ref, int bx, int by, int w4, int shape, int part, int done, int out[2]) const {
    struct N {
      bool avail;
      int ref;
      int mv[2];
    };
    auto get = [&](int x4, int y4) -> N {
      N n{false, -1, {0, 0}};
      const CabacNb* m = nb_mb(x4, y4);
      if (!m) return n;
      const int q = quad_of(x4, y4);
      if (m == &cur && !((done >> q) & 1)) return n;
      n.avail = true;
      if (mbk_is_intra(m->kind)) return n;
      n.ref = m->ref[list][q];
      if (n.ref >= 0) {
        n.mv[0] = m->mv[list][q][0];
        n.mv[1] = m->mv[list][q][1];
      }
      return n;
    };
    N a = get(bx - 1, by), b = get(bx, by - 1), c = get(bx + w4, by - 1);
    // C inside the current MB below-right of a finished partition is "not yet decoded";
    // a C to the right of the MB below the top row is unavailable (nb_mb returns null)
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

  // P_Skip motion (8.4.1.1)
  MIVC_HD void pskip_mv(int out[2]) const {
    out[0] = out[1] = 0;
    const CabacNb* a = A();
    const CabacNb* b = B();
    if (!a || !b) return;
    if (!mbk_is_intra(a->kind) && a->ref[0][1] == 0 && a->mv[0][1][0] == 0 && a->mv[0][1][1] == 0) return;
    if (!mbk_is_intra(b->kind) && b->ref[0][2] == 0 && b->mv[0][2][0] == 0 && b->mv[0][2][1] == 0) return;
    mvp(0, 0, 0, 0, 4, 0, 0, 0, out);
  }

  // ---------------------------------------------------------------- syntax elements
  MIVC_HD void put_mb_skip(int skip) {
    const CabacNb* a = A();
    const CabacNb* b = B();
    const int inc = (a && !a->skip) + (b && !b->skip);
    e.decision((si.slice_type == SLICE_B ? CTX_MB_SKIP_B : CTX_MB_SKIP_P) + inc, skip);
  }

  // I mb_type bins after the prefix: offset = first context of the I binarisation
  // (3 in I slices with neighbour ctx for bin 0; 17 / 32 suffix in P / B slices)
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

  // B mb_type (Table 9-37(b)); bits = the bin string after bin 0, MSB first, nb bins
  MIVC_HD void put_mb_type_b(int kind, int i16_mode, int cbp, int code) {
    const CabacNb* a = A();
    const CabacNb* b = B();
    const int inc = (a && !a->skip && a->kind != MBK_BDIRECT) + (b && !b->skip && b->kind != MBK_BDIRECT);
    if (kind == MBK_BDIRECT) {
      e.decision(CTX_MB_TYPE_B + inc, 0);
      return;
    }
    e.decision(CTX_MB_TYPE_B + inc, 1);
    // code: B mb_type value 1..22 (Table 7-14), 23 = intra prefix
    if (code <= 2) {  // B_L0_16x16 "100", B_L1_16x16 "101"
      e.decision(CTX_MB_TYPE_B + 3, 0);
      e.decision(CTX_MB_TYPE_B + 5, code - 1);
      return;
    }
    e.decision(CTX_MB_TYPE_B + 3, 1);
    int bits, nb;
    if (code <= 10) { bits = code - 3; nb = 4; }                // 1 1 0 xxx: 3..10 -> 0000..0111 (4 bins incl. the 0)
    else if (code == 11) { bits = 0x3E; nb = 0; }               // handled below
    else if (code == 22) { bits = 0x1F; nb = 0; }
    else if (code == 23) { bits = 0x1D; nb = 0; }
    else { bits = code - 12 + 0x10; nb = 5; }                   // 12..21: 1 1 1 0 xxx / 1 1 1 1 0 xx
    if (code <= 10) {
      // bins 2..5: 0 b b b
      e.decision(CTX_MB_TYPE_B + 4, 0);
      e.decision(CTX_MB_TYPE_B + 5, (bits >> 2) & 1);
      e.decision(CTX_MB_TYPE_B + 5, (bits >> 1) & 1);
      e.decision(CTX_MB_TYPE_B + 5, bits & 1);
      return;
    }
    e.decision(CTX_MB_TYPE_B + 4, 1);
    if (code == 11) {  // 1 1 1 1 1 0
      e.decision(CTX_MB_TYPE_B + 5, 1);
      e.decision(CTX_MB_TYPE_B + 5, 1);
      e.decision(CTX_MB_TYPE_B + 5, 0);
      return;
    }
    if (code == 22) {  // B_8x8: 1 1 1 1 1 1
      e.decision(CTX_MB_TYPE_B + 5, 1);
      e.decision(CTX_MB_TYPE_B + 5, 1);
      e.decision(CTX_MB_TYPE_B + 5, 1);
      return;
    }
    if (code == 23) {  // intra prefix: 1 1 1 1 0 1
      e.decision(CTX_MB_TYPE_B + 5, 1);
      e.decision(CTX_MB_TYPE_B + 5, 0);
      e.decision(CTX_MB_TYPE_B + 5, 1);
      put_mb_type_i(kind, i16_mode, cbp, false);
      return;
    }
    // 12..21 -> bins 3..6 = 4-bit value (code - 12) with 12..19 = 0xxx, 20..21 = 100x
    const int v = code - 12;
    e.decision(CTX_MB_TYPE_B + 5, (v >> 3) & 1);
    e.decision(CTX_MB_TYPE_B + 5, (v >> 2) & 1);
    e.decision(CTX_MB_TYPE_B + 5, (v >> 1) & 1);
    e.decision(CTX_MB_TYPE_B + 5, v & 1);
    (void)nb;
  }

  MIVC_HD void put_sub_mb_type_b(int code) {
    // Table 9-38: 0 direct "0", 1 "100", 2 "101", 3 "11000", 4 "11001", 5 "11010", 6 "11011",
    // 7 "111000", 8 "111001", 9 "111010", 10 "111011", 11 "11110", 12 "11111"
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
    // neighbours A / B of the partition's top-left 4x4 (quadrant granularity)
    const int x4 = (q & 1) * 2, y4 = (q >> 1) * 2;
    auto cond = [&](const CabacNb* m, int qn) -> int {
      if (!m || m->skip || mbk_is_intra(m->kind)) return 0;
      if ((m->direct >> qn) & 1) return 0;
      return m->ref[list][qn] > 0;
    };
    const CabacNb* a = nb_mb(x4 - 1, y4);
    const CabacNb* b = nb_mb(x4, y4 - 1);
    const int inc = cond(a, quad_of(x4 - 1, y4)) + 2 * cond(b, quad_of(x4, y4 - 1));
    e.decision(CTX_REF_IDX + inc, ref > 0);
    if (ref == 0) return;
    for (int k = 1; k < ref; ++k) e.decision(CTX_REF_IDX + (k == 1 ? 4 : 5), 1);
    e.decision(CTX_REF_IDX + (ref == 1 ? 4 : 5), 0);
  }

  MIVC_HD void put_mvd(int list, int q, int comp, int v) {
    const int x4 = (q & 1) * 2, y4 = (q >> 1) * 2;
    auto absn = [&](const CabacNb* m, int qn) -> int {
      if (!m) return 0;
      return m->mvd[list][qn][comp];
    };
    const int sum = absn(nb_mb(x4 - 1, y4), quad_of(x4 - 1, y4)) + absn(nb_mb(x4, y4 - 1), quad_of(x4, y4 - 1));
    const int base = comp ? CTX_MVD_Y : CTX_MVD_X;
    const int inc0 = sum < 3 ? 0 : (sum > 32 ? 2 : 1);
    const int av = v < 0 ? -v : v;
    const int pre = av < 9 ? av : 9;
    e.decision(base + inc0, pre > 0);
    if (pre > 0) {
      for (int k = 1; k < pre; ++k) e.decision(base + (k < 4 ? k + 2 : 6), 1);
      if (pre < 9) e.decision(base + (pre < 4 ? pre + 2 : 6), 0);
      if (av >= 9) e.bypass_eg(static_cast<uint32_t>(av - 9), 3);
      e.bypass(v < 0);
    }
  }

  MIVC_HD void put_cbp(int cbp, bool intra_cur) {
    (void)intra_cur;
    const CabacNb* a = A();
    const CabacNb* b = B();
    // unavailable neighbours and I_PCM count as "all blocks coded"
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

  MIVC_HD void put_qp_delta(int d) {
    const int m = d > 0 ? 2 * d - 1 : -2 * d;
    e.decision(CTX_QP_DELTA + (last_dqp ? 1 : 0), m > 0);
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
    const int ma = (a->kind == MBK_I4x4 || a->kind == MBK_I8x8) ? a->i4[rast_of(x4 - 1, y4)] : 2;
    const int mb = (b->kind == MBK_I4x4 || b->kind == MBK_I8x8) ? b->i4[rast_of(x4, y4 - 1)] : 2;
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
  MIVC_HD int put_block(const int16_t* c, int n, int cat, int cbf_inc, bool nonzero = true) {
    if (!nonzero) {
      if (cbf_inc >= 0) e.decision(CTX_CBF + kCbfCatOffset[cat] + cbf_inc, 0);
      return 0;
    }
    int last = -1;
    for (int i = n - 1; i >= 0; --i)
      if (c[i]) {
        last = i;
        break;
      }
    if (cbf_inc >= 0) {
      e.decision(CTX_CBF + kCbfCatOffset[cat] + cbf_inc, last >= 0);
      if (last < 0) return 0;
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
      const int v = c[i];
      if (!v) continue;
      const int a1 = (v < 0 ? -v : v) - 1;
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
      e.bypass(v < 0);
    }
    return 1;
  }

  // coded_block_flag ctxIdxInc of a luma 4x4 block at raster (x4, y4) of the current MB
  MIVC_HD int cbf_luma_inc(int x4, int y4, bool intra) const {
    auto cond = [&](int xn, int yn) -> int {
      const CabacNb* m = nb_mb(xn, yn);
      if (!m) return intra ? 1 : 0;
      if (m->kind == MBK_IPCM) return 1;
      return (m->cbf_luma >> rast_of(xn, yn)) & 1;
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
    const int a = cx > 0 ? cond(&cur, cy * 2) : cond(A(), cy * 2 + 1);
    const int b = cy > 0 ? cond(&cur, cx) : cond(B(), 2 + cx);
    return a + 2 * b;
  }

  // ---------------------------------------------------------------- one macroblock
  // h / c: the record; skip_ok: the encoder's motion equals the skip / direct motion
  // (P: derived here; B: the caller's direct derivation).  b_code: B mb_type value.
  MIVC_HD void code_mb(int mbx, int mby, const MbHeader& h, const int16_t* c, int b_code = 0, const int8_t* b_sub = nullptr,
                       const uint32_t* mask_in = nullptr) {
    mx = mbx;
    my = mby;
    const bool pslice = si.slice_type == SLICE_P, bslice = si.slice_type == SLICE_B;
    int kind = h.kind;
    mbmask = mask_in ? *mask_in : cabac_block_mask(h, c);
    const int cbp = cabac_mask_cbp(h, mbmask);
    const bool intra = mbk_is_intra(kind);
    // ---- reset the current MB context
    cur.avail = 1;
    cur.skip = 0;
    cur.cbp = static_cast<uint8_t>(cbp);
    cur.t8x8 = 0;
    cur.chroma_mode = 0;
    cur.direct = 0;
    cur.cbf_dc = 0;
    cur.cbf_luma = 0;
    cur.cbf_cac[0] = cur.cbf_cac[1] = 0;
    for (int l = 0; l < 2; ++l)
      for (int q = 0; q < 4; ++q) {
        cur.ref[l][q] = intra ? -1 : h.ref[l][q];
        cur.mv[l][q][0] = intra ? 0 : h.mv[l][q][0];
        cur.mv[l][q][1] = intra ? 0 : h.mv[l][q][1];
        cur.mvd[l][q][0] = cur.mvd[l][q][1] = 0;
      }
    for (int i = 0; i < 16; ++i) cur.i4[i] = 2;
    cur.kind = static_cast<uint8_t>(kind == MBK_PSKIP ? MBK_P16x16 : kind);
    // ---- skip
    bool skip = false;
    if (pslice && (kind == MBK_P16x16 || kind == MBK_PSKIP) && cbp == 0 && h.ref[0][0] == 0) {
      int smv[2];
      pskip_mv(smv);
      skip = smv[0] == h.mv[0][0][0] && smv[1] == h.mv[0][0][1];
    } else if (bslice && kind == MBK_BDIRECT && cbp == 0) {
      skip = true;
    }
    if (pslice || bslice) put_mb_skip(skip ? 1 : 0);
    if (skip) {
      cur.skip = 1;
      cur.kind = static_cast<uint8_t>(pslice ? MBK_PSKIP : MBK_BDIRECT);
      cur.cbp = 0;
      if (bslice) cur.direct = 0xF;
      last_dqp = 0;
      ++n_skip;
      finish_mb();
      return;
    }
    if (kind == MBK_PSKIP) kind = MBK_P16x16;
    cur.kind = static_cast<uint8_t>(kind);
    const bool t8 = (h.flags & MBF_T8x8) != 0 && si.t8x8_mode;
    // ---- mb_type
    if (pslice) put_mb_type_p(kind, h.i16_mode, cbp);
    else if (bslice) put_mb_type_b(kind, h.i16_mode, cbp, intra ? 23 : (b_code ? b_code : cabac_b_code(h)));
    else put_mb_type_i(kind, h.i16_mode, cbp, true);
    if (intra) ++n_intra; else ++n_inter;
    // ---- prediction
    if (kind == MBK_I4x4 || kind == MBK_I8x8) {
      if (si.t8x8_mode) put_t8x8(kind == MBK_I8x8);
      cur.t8x8 = kind == MBK_I8x8;
      if (kind == MBK_I4x4) {
        for (int blk = 0; blk < 16; ++blk) {
          const int x4 = kBlkX[blk], y4 = kBlkY[blk];
          const int mode = h.i4_modes[blk];
          put_intra_mode(mode, pred_intra_mode(x4, y4));
          cur.i4[x4 + 4 * y4] = static_cast<uint8_t>(mode);
        }
      } else {
        for (int b8 = 0; b8 < 4; ++b8) {
          const int x4 = (b8 & 1) * 2, y4 = (b8 >> 1) * 2;
          const int mode = h.i4_modes[b8 * 4];
          put_intra_mode(mode, pred_intra_mode(x4, y4));
          for (int k = 0; k < 4; ++k) cur.i4[x4 + (k & 1) + 4 * (y4 + (k >> 1))] = static_cast<uint8_t>(mode);
        }
      }
    }
    if (intra) {
      put_chroma_mode(h.chroma_mode);
      cur.chroma_mode = h.chroma_mode;
    } else {
      code_inter_pred(h, kind, b_code, b_sub);
    }
    // ---- coded_block_pattern, transform size
    if (kind != MBK_I16x16) {
      put_cbp(cbp, intra);
      if ((cbp & 15) && si.t8x8_mode && !intra && kind != MBK_I8x8) {
        bool ok = true;
        if (kind == MBK_B8x8) ok = true;  // sub-blocks are 8x8 or direct (direct_8x8_inference = 1)
        if (ok) {
          put_t8x8(t8 ? 1 : 0);
          cur.t8x8 = t8;
        }
      }
    }
    const bool t8_res = cur.t8x8 != 0;
    // ---- mb_qp_delta + residual
    if (cbp == 0 && kind != MBK_I16x16) {
      last_dqp = 0;
      finish_mb();
      return;
    }
    int d = h.qp - last_qp;
    if (d < -26) d += 52;
    if (d > 25) d -= 52;
    put_qp_delta(d);
    last_dqp = d != 0;
    last_qp = h.qp;
    // luma
    if (kind == MBK_I16x16) {
      const int f = put_block(c + COEF_LUMA_DC, 16, 0, cbf_dc_inc(0, true), (mbmask & NZ_LUMA_DC) != 0);
      cur.cbf_dc |= f;
    }
    for (int b8 = 0; b8 < 4; ++b8) {
      if (!((cbp >> b8) & 1)) continue;
      if (t8_res) {
        put_block(c + COEF_LUMA + b8 * 64, 64, 5, -1);
        const int x4 = (b8 & 1) * 2, y4 = (b8 >> 1) * 2;
        cur.cbf_luma |= static_cast<uint16_t>(0x33u << (x4 + 4 * y4));
        continue;
      }
      for (int b4 = 0; b4 < 4; ++b4) {
        const int blk = b8 * 4 + b4;
        const int x4 = kBlkX[blk], y4 = kBlkY[blk];
        const int inc = cbf_luma_inc(x4, y4, intra);
        int f;
        const bool nzb = (mbmask >> blk) & 1u;
        if (kind == MBK_I16x16) f = put_block(c + COEF_LUMA + blk * 16 + 1, 15, 1, inc, nzb);
        else f = put_block(c + COEF_LUMA + blk * 16, 16, 2, inc, nzb);
        if (f) cur.cbf_luma |= static_cast<uint16_t>(1u << (x4 + 4 * y4));
      }
    }
    // chroma
    const int cc = cbp >> 4;
    if (cc) {
      for (int comp = 0; comp < 2; ++comp) {
        const int f = put_block(c + COEF_CHROMA_DC + comp * 4, 4, 3, cbf_dc_inc(1 + comp, intra),
                                ((mbmask >> (17 + comp)) & 1u) != 0);
        cur.cbf_dc |= static_cast<uint8_t>(f << (1 + comp));
      }
    }
    if (cc == 2) {
      for (int comp = 0; comp < 2; ++comp)
        for (int b = 0; b < 4; ++b) {
          const int f = put_block(c + COEF_CHROMA_AC + (comp * 4 + b) * 16 + 1, 15, 4,
                                  cbf_cac_inc(comp, b & 1, b >> 1, intra), ((mbmask >> (19 + comp * 4 + b)) & 1u) != 0);
          cur.cbf_cac[comp] |= static_cast<uint8_t>(f << b);
        }
    }
    finish_mb();
  }

  MIVC_HD void code_inter_pred(const MbHeader& h, int kind, int b_code, const int8_t* b_sub) {
    const bool bslice = si.slice_type == SLICE_B;
    // partitions (quadrant masks): 16x16: {0xF}; 16x8: {0x3, 0xC}; 8x16: {0x5, 0xA}; 8x8: 4
    int np, qfirst[4], w4[4], shape;
    if (kind == MBK_P16x16 || kind == MBK_B16x16) { np = 1; qfirst[0] = 0; w4[0] = 4; shape = 0; }
    else if (kind == MBK_P16x8 || kind == MBK_B16x8) { np = 2; qfirst[0] = 0; qfirst[1] = 2; w4[0] = w4[1] = 4; shape = 1; }
    else if (kind == MBK_P8x16 || kind == MBK_B8x16) { np = 2; qfirst[0] = 0; qfirst[1] = 1; w4[0] = w4[1] = 2; shape = 2; }
    else { np = 4; for (int q = 0; q < 4; ++q) { qfirst[q] = q; w4[q] = 2; } shape = 0; }
    const bool sub8 = np == 4;
    const int dir_mask = kind == MBK_B8x8 ? (h.sub_direct & 15) : 0;
    auto pmask = [&](int p) -> int {
      if (!sub8) return shape == 0 ? 0xF : (shape == 1 ? (p ? 0xC : 0x3) : (p ? 0xA : 0x5));
      return 1 << p;
    };
    (void)b_code;
    if (sub8) {
      if (bslice) {
        for (int s = 0; s < 4; ++s) {
          int code = 0;
          if (!((dir_mask >> s) & 1)) {
            const bool l0 = h.ref[0][s] >= 0, l1 = h.ref[1][s] >= 0;
            code = (l0 && l1) ? 3 : (l1 ? 2 : 1);
          }
          put_sub_mb_type_b(b_sub ? b_sub[s] : code);
        }
        cur.direct = static_cast<uint8_t>(dir_mask);
      } else {
        for (int s = 0; s < 4; ++s) e.decision(CTX_SUB_MB_P, 1);  // P_L0_8x8
      }
    }
    // ref_idx, all partitions of list 0 then list 1
    for (int l = 0; l < 2; ++l) {
      if (si.num_ref[l] <= 1) continue;
      for (int p = 0; p < np; ++p) {
        const int q = qfirst[p];
        if (sub8 && ((dir_mask >> q) & 1)) continue;
        if (h.ref[l][q] < 0) continue;
        put_ref_idx(l, q, h.ref[l][q]);
      }
    }
    // mvd, list 0 then list 1; the MVs of earlier partitions are visible to later ones
    int done = 0;
    for (int l = 0; l < 2; ++l) {
      done = 0;
      for (int p = 0; p < np; ++p) {
        const int q = qfirst[p];
        const int m = pmask(p);
        if (sub8 && ((dir_mask >> q) & 1)) {
          done |= m;
          continue;
        }
        if (h.ref[l][q] < 0) {
          done |= m;
          continue;
        }
        int pm[2];
        mvp(l, h.ref[l][q], (q & 1) * 2, (q >> 1) * 2, w4[p], shape, p, done, pm);
        const int dx = h.mv[l][q][0] - pm[0], dy = h.mv[l][q][1] - pm[1];
        put_mvd(l, q, 0, dx);
        put_mvd(l, q, 1, dy);
        const int ax = dx < 0 ? -dx : dx, ay = dy < 0 ? -dy : dy;
        for (int k = 0; k < 4; ++k)
          if ((m >> k) & 1) {
            cur.mvd[l][k][0] = static_cast<uint8_t>(ax > 255 ? 255 : ax);
            cur.mvd[l][k][1] = static_cast<uint8_t>(ay > 255 ? 255 : ay);
          }
        done |= m;
      }
    }
  }

  MIVC_HD void finish_mb() { row[mx] = cur; }
};

// Code MB records [first_mb, first_mb + n) of one picture as slice data; returns the
// number of bytes written (slice_data only: the caller writes the slice header, which
// ends byte-aligned with cabac_alignment_one_bits, and the NAL framing).
// b_codes / b_subs: optional per-MB B mb_type value and sub_mb_types (B slices).
MIVC_HD size_t cabac_write_slice_data(CabacMbWriter& w, const CabacSliceInfo& si, CabacNb* rowbuf, uint8_t* states,
                                      CabacBuf* out, const MbHeader* hdr, const int16_t* coef, int n,
                                      const uint8_t* b_codes = nullptr, const int8_t* b_subs = nullptr,
                                      const uint32_t* masks = nullptr, bool states_ready = false,
                                      bool row_ready = false) {
  w.begin(si, rowbuf, states, out, states_ready, row_ready);
  const int end = si.first_mb + n;
  for (int addr = si.first_mb; addr < end; ++addr) {
    const int mx = addr % si.wmb, my = addr / si.wmb;
    if (mx == 0) w.tl.avail = 0;
    CabacNb top_old = rowbuf[mx];
    w.code_mb(mx, my, hdr[addr], coef + static_cast<size_t>(addr) * kCoefPerMb, b_codes ? b_codes[addr] : 0,
              b_subs ? b_subs + static_cast<size_t>(addr) * 4 : nullptr, masks ? masks + addr : nullptr);
    w.tl = top_old;  // MB (mx, my-1) is the top-left of MB (mx+1, my)
    w.e.terminate(addr == end - 1 ? 1 : 0);
  }
  return out->n;
}

}  // namespace h264
}  // namespace mivc
