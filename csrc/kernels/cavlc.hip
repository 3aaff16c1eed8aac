// CAVLC entropy coding on the GPU (SURVEY.md K-C10 "optionally a GPU CAVLC").
//
// Produces the slice RBSP (slice header + slice_data + trailing bits) of every
// (slot) frame directly in HBM, so only the compressed bytes cross PCIe (the
// host keeps NAL framing / emulation prevention).  Byte-exact with the host
// writer (csrc/host/cavlc_writer.cc), which is the test oracle.
//
// Why it parallelises: with one MV per 16x16 P macroblock the motion field is
// fixed by the encoder, and P_Skip is only a *coding* choice (taken when
// mv == mvp_skip and cbp == 0) that never changes a vector -- so every MB's
// predictors, skip flag, nC contexts and most-probable intra modes depend only
// on the decision records, not on other MBs' coding.  The remaining serial
// quantities (mb_skip_run, QP_pred for mb_qp_delta, bit offsets) are prefix
// scans.
//
// Kernels, all batched over B slots:
//   cavlc_analyze   (nmb x B, wave64 per MB)  cbp, TotalCoeff per block, skip, mvd, i4 mode codes
//   cavlc_scan      (B, 1024)                 skip runs, QP_pred / mb_qp_delta, trailing run
//   cavlc_length    (nmb x B, wave64 per MB)  bit length of every coded MB
//   cavlc_offsets   (B, 1024)                 prefix sum of lengths, header + trailer bits
//   cavlc_write     (nmb x B, wave64 per MB)  emit bits (lanes own disjoint bit ranges)
//   cavlc_compact   (B, 256)                  big-endian words -> bytes, packed slot after slot
#include "kcommon.h"

namespace mivc {
namespace gpu {

using h264::MbHeader;

struct alignas(16) CavlcMb {
  uint8_t coded;      // 0: P_Skip
  uint8_t kind;       // coded MbKind
  uint8_t cbp;
  uint8_t has_delta;  // mb_qp_delta present
  int16_t mvd[2];
  int16_t run;        // mb_skip_run preceding this MB (P slices)
  int8_t qp_delta;
  uint8_t pad[7];
  uint8_t tc[24];     // TotalCoeff: luma blocks (blkIdx order), Cb[4], Cr[4]
  uint8_t i4code[16]; // 0x80 = prev_intra4x4_pred_mode_flag, else rem_intra4x4_pred_mode
  uint8_t pad2[8];
};
static_assert(sizeof(CavlcMb) == 72 || sizeof(CavlcMb) == 80, "CavlcMb layout");

struct CavlcArgs {
  Geom g;
  const MbHeader* hdr;
  const int16_t* coef;
  CavlcMb* mbs;
  int* len;              // [B, nmb] bits per MB (0 if skipped)
  uint16_t* blen;        // [B, nmb, 28] bits per syntax slot (header + residual blocks)
  long long* off;        // [B, nmb] bit offset of each MB
  int* trail;            // [B] trailing skip run
  long long* total_bits; // [B]
  int* slot_bytes;       // [B]
  uint32_t* words;       // [B, cap_words]
  long long cap_words;
  const uint32_t* hdr_bits;  // [B, 16] slice header bits (big-endian bit order words)
  const int* hdr_nbits;      // [B]
  int pslice;
  int slice_qp;
  const int* slot_qp;    // [B] per-slot slice QP (null: slice_qp for every slot)
  uint8_t* out;          // compacted bytes
  long long* out_off;    // [B] byte offset of every slot in `out`
  const uint8_t* nz;     // [B, nmb, 16] raster luma non-zero flags from the encoder (nullable):
                         // all-zero blocks of inter MBs are not loaded
};

// ---------------------------------------------------------------- bit sinks
struct LenSink {
  int n = 0;
  __device__ __forceinline__ void put(uint32_t, int bits) { n += bits; }
};

// Writes a contiguous bit range owned by one lane.  Words fully inside the range are
// stored plainly; the (possibly shared) first and last words are OR-ed atomically.
struct WordSink {
  uint32_t* buf;
  long long w;     // current word index
  uint64_t acc;    // pending bits, left-aligned
  int nacc;        // pending bit count (< 32 after each put)
  bool first;
  __device__ __forceinline__ WordSink(uint32_t* b, long long bitpos) : buf(b), w(bitpos >> 5), acc(0), nacc(static_cast<int>(bitpos & 31)), first(true) {}
  __device__ __forceinline__ void put(uint32_t v, int bits) {
    if (bits <= 0) return;
    uint64_t x = bits >= 32 ? v : (v & ((1u << bits) - 1u));
    acc |= x << (64 - nacc - bits);
    nacc += bits;
    while (nacc >= 32) {
      uint32_t word = static_cast<uint32_t>(acc >> 32);
      if (first) atomicOr(buf + w, word); else buf[w] = word;
      first = false;
      ++w;
      acc <<= 32;
      nacc -= 32;
    }
  }
  __device__ __forceinline__ void flush() {
    if (nacc > 0) atomicOr(buf + w, static_cast<uint32_t>(acc >> 32));
    nacc = 0;
  }
};

template <class S>
__device__ __forceinline__ void put_ue(S& s, uint32_t v) {
  uint32_t x = v + 1;
  int n = 31 - __clz(x);
  s.put(x, 2 * n + 1);
}
template <class S>
__device__ __forceinline__ void put_se(S& s, int v) {
  put_ue(s, v <= 0 ? static_cast<uint32_t>(-2 * v) : static_cast<uint32_t>(2 * v - 1));
}

// ---------------------------------------------------------------- residual_block_cavlc
template <class S>
__device__ __forceinline__ void put_level(S& s, int level_code, int sl) {
  if (sl == 0) {
    if (level_code < 14) { s.put(1, level_code + 1); return; }
    if (level_code < 30) { s.put(1, 15); s.put(static_cast<uint32_t>(level_code - 14), 4); return; }
    int rem = level_code - 30;
    if (rem < 4096) { s.put(1, 16); s.put(static_cast<uint32_t>(rem), 12); return; }
    int prefix = 16;
    while (true) {
      int r = rem - ((1 << (prefix - 3)) - 4096);
      if (r < (1 << (prefix - 3))) { s.put(0, prefix); s.put(1, 1); s.put(static_cast<uint32_t>(r), prefix - 3); return; }
      ++prefix;
    }
  }
  if (level_code < (15 << sl)) {
    s.put(1, (level_code >> sl) + 1);
    s.put(static_cast<uint32_t>(level_code & ((1 << sl) - 1)), sl);
    return;
  }
  int rem = level_code - (15 << sl);
  if (rem < 4096) { s.put(1, 16); s.put(static_cast<uint32_t>(rem), 12); return; }
  int prefix = 16;
  while (true) {
    int r = rem - ((1 << (prefix - 3)) - 4096);
    if (r < (1 << (prefix - 3))) { s.put(0, prefix); s.put(1, 1); s.put(static_cast<uint32_t>(r), prefix - 3); return; }
    ++prefix;
  }
}

// c: 16 coefficients in scan order (a register array: every loop below is fully
// unrolled so no index is dynamic and nothing spills to scratch).  Returns TotalCoeff.
template <class S>
__device__ __forceinline__ int cavlc_block(S& s, const int (&c)[16], int start, int end, int maxnum, int nc) {
  uint32_t nz = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) nz |= (i >= start && i <= end && c[i] != 0) ? (1u << i) : 0u;
  const int total = __popc(nz);
  // trailing ones: leading run (from the highest frequency) of |level| == 1, at most 3
  int t1 = 0;
  bool t1open = true;
#pragma unroll
  for (int i = 15; i >= 0; --i) {
    if (nz & (1u << i)) {
      bool one = c[i] == 1 || c[i] == -1;
      if (t1open && one && t1 < 3) ++t1; else t1open = false;
    }
  }
  if (nc == -1) {
    s.put(h264::kChromaDcCoeffTokenBits[total * 4 + t1], h264::kChromaDcCoeffTokenLen[total * 4 + t1]);
  } else {
    int t = nc < 2 ? 0 : (nc < 4 ? 1 : (nc < 8 ? 2 : 3));
    s.put(h264::kCoeffTokenBits[t][total * 4 + t1], h264::kCoeffTokenLen[t][total * 4 + t1]);
  }
  if (total == 0) return 0;
  const int last = 31 - __clz(nz);
  const int total_zeros = (last - start + 1) - total;
  int k = 0;
  int sl = (total > 10 && t1 < 3) ? 1 : 0;
#pragma unroll
  for (int i = 15; i >= 0; --i) {
    if (nz & (1u << i)) {
      int lv = c[i];
      if (k < t1) {
        s.put(lv < 0 ? 1u : 0u, 1);
      } else {
        int code = lv > 0 ? 2 * lv - 2 : -2 * lv - 1;
        if (k == t1 && t1 < 3) code -= 2;
        put_level(s, code, sl);
        if (sl == 0) sl = 1;
        int al = lv < 0 ? -lv : lv;
        if (al > (3 << (sl - 1)) && sl < 6) ++sl;
      }
      ++k;
    }
  }
  if (total < end - start + 1) {
    if (maxnum == 4) s.put(h264::kChromaDcTotalZerosBits[total - 1][total_zeros], h264::kChromaDcTotalZerosLen[total - 1][total_zeros]);
    else s.put(h264::kTotalZerosBits[total - 1][total_zeros], h264::kTotalZerosLen[total - 1][total_zeros]);
  }
  int zl = total_zeros;
#pragma unroll
  for (int i = 15; i >= 1; --i) {
    uint32_t lower = nz & ((1u << i) - 1u);
    if ((nz & (1u << i)) && lower != 0 && zl > 0) {
      int run = i - (31 - __clz(lower)) - 1;
      int t = (zl < 7 ? zl : 7) - 1;
      s.put(h264::kRunBeforeBits[t][run], h264::kRunBeforeLen[t][run]);
      zl -= run;
    }
  }
  return total;
}

// 16 int16 coefficients (32 contiguous bytes) -> registers with two 16-byte loads
__device__ __forceinline__ void load16(const int16_t* p, int (&v)[16]) {
  const uint4 q0 = reinterpret_cast<const uint4*>(p)[0];
  const uint4 q1 = reinterpret_cast<const uint4*>(p)[1];
  const uint32_t w[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    v[2 * i] = static_cast<int16_t>(w[i] & 0xFFFFu);
    v[2 * i + 1] = static_cast<int16_t>(w[i] >> 16);
  }
}

// ---------------------------------------------------------------- helpers
__device__ __forceinline__ int med3(int a, int b, int c) { return max(min(a, b), min(max(a, b), c)); }

struct NbMv {
  bool avail;
  int ref;
  int mv[2];
};

__device__ __forceinline__ NbMv nb_mv(const MbHeader* hdr, size_t base, int wmb, int hmb, int x, int y, int quad) {
  NbMv r{false, -1, {0, 0}};
  if (x < 0 || y < 0 || x >= wmb || y >= hmb) return r;
  r.avail = true;
  const MbHeader& h = hdr[base + y * wmb + x];
  if (h264::mbk_is_intra(h.kind)) return r;
  r.ref = 0;
  r.mv[0] = h.mv[0][quad][0];
  r.mv[1] = h.mv[0][quad][1];
  return r;
}

// (tc of the neighbouring luma 4x4 block, availability) for block (bx, by) of MB (mx, my)
__device__ __forceinline__ int nc_luma(const CavlcMb* mbs, size_t base, int wmb, int mx, int my, const uint8_t* own_tc,
                                       int bx, int by) {
  bool ha, hb;
  int na = 0, nb = 0;
  if (bx > 0) { ha = true; na = own_tc[h264::kRasterToBlk[(bx - 1) + 4 * by]]; }
  else { ha = mx > 0; if (ha) na = mbs[base + my * wmb + mx - 1].tc[h264::kRasterToBlk[3 + 4 * by]]; }
  if (by > 0) { hb = true; nb = own_tc[h264::kRasterToBlk[bx + 4 * (by - 1)]]; }
  else { hb = my > 0; if (hb) nb = mbs[base + (my - 1) * wmb + mx].tc[h264::kRasterToBlk[bx + 12]]; }
  if (ha && hb) return (na + nb + 1) >> 1;
  return ha ? na : (hb ? nb : 0);
}

__device__ __forceinline__ int nc_chroma(const CavlcMb* mbs, size_t base, int wmb, int mx, int my, const uint8_t* own_tc,
                                         int comp, int cx, int cy) {
  bool ha, hb;
  int na = 0, nb = 0;
  if (cx > 0) { ha = true; na = own_tc[16 + comp * 4 + cy * 2 + cx - 1]; }
  else { ha = mx > 0; if (ha) na = mbs[base + my * wmb + mx - 1].tc[16 + comp * 4 + cy * 2 + 1]; }
  if (cy > 0) { hb = true; nb = own_tc[16 + comp * 4 + (cy - 1) * 2 + cx]; }
  else { hb = my > 0; if (hb) nb = mbs[base + (my - 1) * wmb + mx].tc[16 + comp * 4 + 2 + cx]; }
  if (ha && hb) return (na + nb + 1) >> 1;
  return ha ? na : (hb ? nb : 0);
}

// ---------------------------------------------------------------- K1: analyze
// Two MBs per wave (lanes 0-31 and 32-63).  Per half: lanes 0-15 count the non-zero
// coefficients of the 16 luma blocks, 16-23 the chroma AC blocks (two 16-byte loads
// each), lane 24 the 8 chroma DC levels; then lane 0 derives cbp / skip / mvd and lanes
// 0-15 the Intra4x4 mode codes.
__global__ __launch_bounds__(64) void cavlc_analyze(CavlcArgs a) {
  const Geom& g = a.g;
  const int lane = threadIdx.x, sub = lane & 31, half = lane >> 5;
  const int mb = blockIdx.x * 2 + half, slot = blockIdx.y;
  __shared__ int s_tc[2][24];
  __shared__ int s_dc[2];
  const bool active = mb < g.nmb();
  const int mbc = active ? mb : 0;
  const int mx = mbc % g.wmb, my = mbc / g.wmb;
  const size_t base = static_cast<size_t>(slot) * g.nmb();
  const size_t o = base + mbc;
  const MbHeader& h = a.hdr[o];
  const int16_t* c = a.coef + o * h264::kCoefPerMb;
  CavlcMb& m = a.mbs[o];
  const int kind0 = h.kind;
  int n = 0;
  if (sub < 24) {
    int v[16];
    load16(c + (sub < 16 ? h264::COEF_LUMA + sub * 16 : h264::COEF_CHROMA_AC + (sub - 16) * 16), v);
    const int start = sub >= 16 ? 1 : (kind0 == h264::MBK_I16x16 ? 1 : 0);
#pragma unroll
    for (int i = 0; i < 16; ++i) n += (i >= start && v[i] != 0) ? 1 : 0;
  } else if (sub == 24) {
    const uint4 q = *reinterpret_cast<const uint4*>(c + h264::COEF_CHROMA_DC);
    n = (q.x | q.y | q.z | q.w) != 0;
  }
  if (sub < 24) s_tc[half][sub] = n;
  else if (sub == 24) s_dc[half] = n;
  __syncthreads();
  if (!active) return;
  if (sub < 24) m.tc[sub] = static_cast<uint8_t>(n);
  if (sub == 0) {
    const int* tc = s_tc[half];
    int luma = 0;
    for (int b8 = 0; b8 < 4; ++b8)
      if (tc[b8 * 4] | tc[b8 * 4 + 1] | tc[b8 * 4 + 2] | tc[b8 * 4 + 3]) luma |= 1 << b8;
    const bool i16 = kind0 == h264::MBK_I16x16;
    if (i16 && luma) luma = 15;
    int chroma = 0;
    for (int i = 16; i < 24; ++i)
      if (tc[i]) chroma = 2;
    if (!chroma && s_dc[half]) chroma = 1;
    int cbp = luma | (chroma << 4);
    m.cbp = static_cast<uint8_t>(cbp);
    const bool inter = !h264::mbk_is_intra(kind0);
    int kind = kind0 == h264::MBK_PSKIP ? h264::MBK_P16x16 : kind0;
    m.kind = static_cast<uint8_t>(kind);
    m.has_delta = (cbp != 0 || i16) ? 1 : 0;
    m.coded = 1;
    m.mvd[0] = m.mvd[1] = 0;
    if (inter) {
      // neighbours: A = left MB block (3,0) -> quadrant 1; B = top block (0,3) -> quadrant 2;
      // C = top-right block (0,3) -> quadrant 2; D = top-left block (3,3) -> quadrant 3
      NbMv A = nb_mv(a.hdr, base, g.wmb, g.hmb, mx - 1, my, 1);
      NbMv B = nb_mv(a.hdr, base, g.wmb, g.hmb, mx, my - 1, 2);
      NbMv C = nb_mv(a.hdr, base, g.wmb, g.hmb, mx + 1, my - 1, 2);
      NbMv D = nb_mv(a.hdr, base, g.wmb, g.hmb, mx - 1, my - 1, 3);
      if (!C.avail) C = D;
      // P_Skip predictor
      int smv[2] = {0, 0};
      bool zero = !A.avail || !B.avail || (A.ref == 0 && A.mv[0] == 0 && A.mv[1] == 0) ||
                  (B.ref == 0 && B.mv[0] == 0 && B.mv[1] == 0);
      NbMv Bm = B, Cm = C;
      if (!Bm.avail && !Cm.avail && A.avail) { Bm = A; Cm = A; }
      int match = (A.ref == 0) + (Bm.ref == 0) + (Cm.ref == 0);
      int pmv[2];
      if (match == 1) {
        const NbMv& q = A.ref == 0 ? A : (Bm.ref == 0 ? Bm : Cm);
        pmv[0] = q.mv[0];
        pmv[1] = q.mv[1];
      } else {
        pmv[0] = med3(A.mv[0], Bm.mv[0], Cm.mv[0]);
        pmv[1] = med3(A.mv[1], Bm.mv[1], Cm.mv[1]);
      }
      if (!zero) { smv[0] = pmv[0]; smv[1] = pmv[1]; }
      if (a.pslice && cbp == 0 && h.mv[0][0][0] == smv[0] && h.mv[0][0][1] == smv[1]) {
        m.coded = 0;
        m.has_delta = 0;
      }
      m.mvd[0] = static_cast<int16_t>(h.mv[0][0][0] - pmv[0]);
      m.mvd[1] = static_cast<int16_t>(h.mv[0][0][1] - pmv[1]);
    }
  }
  if (kind0 == h264::MBK_I4x4 && sub < 16) {
    const int blk = sub, bx = h264::kBlkX[blk], by = h264::kBlkY[blk];
    int ma, mbm;
    bool dcpred = false;
    if (bx > 0) ma = h.i4_modes[h264::kRasterToBlk[(bx - 1) + 4 * by]];
    else if (mx > 0) {
      const MbHeader& L = a.hdr[o - 1];
      ma = L.kind == h264::MBK_I4x4 ? L.i4_modes[h264::kRasterToBlk[3 + 4 * by]] : 2;
    } else { dcpred = true; ma = 2; }
    if (by > 0) mbm = h.i4_modes[h264::kRasterToBlk[bx + 4 * (by - 1)]];
    else if (my > 0) {
      const MbHeader& T = a.hdr[o - g.wmb];
      mbm = T.kind == h264::MBK_I4x4 ? T.i4_modes[h264::kRasterToBlk[bx + 12]] : 2;
    } else { dcpred = true; mbm = 2; }
    int pm = dcpred ? 2 : min(ma, mbm);
    int mode = h.i4_modes[blk];
    m.i4code[blk] = static_cast<uint8_t>(mode == pm ? 0x80 : (mode < pm ? mode : mode - 1));
  }
}

// ---------------------------------------------------------------- K2: scans (skip runs, QP_pred)
__global__ __launch_bounds__(1024) void cavlc_scan(CavlcArgs a) {
  const Geom& g = a.g;
  const int slot = blockIdx.x, n = g.nmb();
  const size_t base = static_cast<size_t>(slot) * n;
  __shared__ int s_last_coded[1024], s_last_delta[1024];
  const int per = (n + blockDim.x - 1) / blockDim.x;
  const int i0 = threadIdx.x * per, i1 = min(n, i0 + per);
  int lc = -1, ld = -1;
  for (int i = i0; i < i1; ++i) {
    if (a.mbs[base + i].coded) lc = i;
    if (a.mbs[base + i].has_delta) ld = i;
  }
  s_last_coded[threadIdx.x] = lc;
  s_last_delta[threadIdx.x] = ld;
  __syncthreads();
  // inclusive max-scan (Hillis-Steele)
  for (int off = 1; off < blockDim.x; off <<= 1) {
    int vc = threadIdx.x >= off ? s_last_coded[threadIdx.x - off] : -1;
    int vd = threadIdx.x >= off ? s_last_delta[threadIdx.x - off] : -1;
    __syncthreads();
    s_last_coded[threadIdx.x] = max(s_last_coded[threadIdx.x], vc);
    s_last_delta[threadIdx.x] = max(s_last_delta[threadIdx.x], vd);
    __syncthreads();
  }
  lc = threadIdx.x > 0 ? s_last_coded[threadIdx.x - 1] : -1;
  ld = threadIdx.x > 0 ? s_last_delta[threadIdx.x - 1] : -1;
  for (int i = i0; i < i1; ++i) {
    CavlcMb& m = a.mbs[base + i];
    if (m.coded) {
      m.run = static_cast<int16_t>(i - lc - 1);
      lc = i;
    }
    if (m.has_delta) {
      int prev = ld >= 0 ? a.hdr[base + ld].qp : (a.slot_qp ? a.slot_qp[slot] : a.slice_qp);
      int d = a.hdr[base + i].qp - prev;
      if (d < -26) d += 52;
      if (d > 25) d -= 52;
      m.qp_delta = static_cast<int8_t>(d);
      ld = i;
    }
  }
  if (threadIdx.x == blockDim.x - 1) a.trail[slot] = n - 1 - s_last_coded[blockDim.x - 1];
}

// ---------------------------------------------------------------- per-MB syntax
// lane 0: macroblock header; lanes 1..: residual blocks in coding order.
// Block slots: 1 = I16 DC, 2..17 = luma blkIdx 0..15, 18..19 = chroma DC, 20..27 = chroma AC.
template <class S>
__device__ __forceinline__ void mb_header_bits(S& s, const CavlcMb& m, const MbHeader& h, bool pslice) {
  if (pslice) put_ue(s, static_cast<uint32_t>(m.run));
  const int cbp = m.cbp, cl = cbp & 15, cc = cbp >> 4;
  const int ioff = pslice ? 5 : 0;
  switch (m.kind) {
    case h264::MBK_P16x16: put_ue(s, 0); break;
    case h264::MBK_I4x4: put_ue(s, ioff); break;
    default: put_ue(s, ioff + 1 + h.i16_mode + 4 * cc + (cl ? 12 : 0)); break;
  }
  if (m.kind == h264::MBK_I4x4) {
    for (int b = 0; b < 16; ++b) {
      int code = m.i4code[b];
      if (code & 0x80) s.put(1, 1); else s.put(static_cast<uint32_t>(code), 4);  // '0' + 3-bit rem
    }
  }
  if (m.kind != h264::MBK_P16x16) put_ue(s, h.chroma_mode);
  else {
    put_se(s, m.mvd[0]);
    put_se(s, m.mvd[1]);
  }
  if (m.kind != h264::MBK_I16x16) put_ue(s, m.kind == h264::MBK_P16x16 ? h264::kInterCbpToCode[cbp] : h264::kIntraCbpToCode[cbp]);
  if (m.has_delta) put_se(s, m.qp_delta);
}

template <class S>
__device__ __forceinline__ void mb_block_bits(S& s, int slotid, const CavlcMb* mbs, size_t base, int wmb, int mx, int my,
                                              const CavlcMb& m, const int16_t* c) {
  const int cbp = m.cbp, cl = cbp & 15, cc = cbp >> 4;
  int v[16];
  if (slotid == 1) {
    if (m.kind != h264::MBK_I16x16) return;
    load16(c + h264::COEF_LUMA_DC, v);
    cavlc_block(s, v, 0, 15, 16, nc_luma(mbs, base, wmb, mx, my, m.tc, 0, 0));
  } else if (slotid < 18) {
    int blk = slotid - 2;
    if (!(cl & (1 << (blk >> 2)))) return;
    if (m.tc[blk]) load16(c + h264::COEF_LUMA + blk * 16, v);  // TotalCoeff 0: no load
    else {
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = 0;
    }
    int nc = nc_luma(mbs, base, wmb, mx, my, m.tc, h264::kBlkX[blk], h264::kBlkY[blk]);
    if (m.kind == h264::MBK_I16x16) cavlc_block(s, v, 1, 15, 15, nc);
    else cavlc_block(s, v, 0, 15, 16, nc);
  } else if (slotid < 20) {
    if (!cc) return;
    int comp = slotid - 18;
    const uint2 q = *reinterpret_cast<const uint2*>(c + h264::COEF_CHROMA_DC + comp * 4);
    v[0] = static_cast<int16_t>(q.x & 0xFFFFu);
    v[1] = static_cast<int16_t>(q.x >> 16);
    v[2] = static_cast<int16_t>(q.y & 0xFFFFu);
    v[3] = static_cast<int16_t>(q.y >> 16);
#pragma unroll
    for (int i = 4; i < 16; ++i) v[i] = 0;
    cavlc_block(s, v, 0, 3, 4, -1);
  } else if (slotid < 28) {
    if (!(cc & 2)) return;
    int k = slotid - 20, comp = k >> 2, b = k & 3;
    if (m.tc[16 + k]) load16(c + h264::COEF_CHROMA_AC + k * 16, v);
    else {
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = 0;
    }
    cavlc_block(s, v, 1, 15, 15, nc_chroma(mbs, base, wmb, mx, my, m.tc, comp, b & 1, b >> 1));
  }
}

// exclusive prefix sum over lanes 0..31 of a wave
__device__ __forceinline__ int lane_exscan32(int v, int lane) {
  int x = v;
#pragma unroll
  for (int off = 1; off < 32; off <<= 1) {
    int y = __shfl_up(x, off, 64);
    if ((lane & 31) >= off) x += y;
  }
  return x - v;
}

// ---------------------------------------------------------------- K3: lengths
// Two MBs per wave (lanes 0-31 and 32-63; 28 syntax slots each).  The bit length of
// every slot is kept (blen) so the writer knows its lane offsets without re-running
// the coder.
__global__ __launch_bounds__(64) void cavlc_length(CavlcArgs a) {
  const Geom& g = a.g;
  const int lane = threadIdx.x, sub = lane & 31;
  const int mb = blockIdx.x * 2 + (lane >> 5), slot = blockIdx.y;
  if (mb >= g.nmb()) return;
  const int mx = mb % g.wmb, my = mb / g.wmb;
  const size_t base = static_cast<size_t>(slot) * g.nmb();
  const CavlcMb& m = a.mbs[base + mb];
  LenSink s;
  if (m.coded) {
    if (sub == 0) mb_header_bits(s, m, a.hdr[base + mb], a.pslice);
    else if (sub < 28) mb_block_bits(s, sub, a.mbs, base, g.wmb, mx, my, m, a.coef + (base + mb) * h264::kCoefPerMb);
  }
  if (sub < 28) a.blen[(base + mb) * 28 + sub] = static_cast<uint16_t>(s.n);
  int n = s.n;
#pragma unroll
  for (int off = 16; off >= 1; off >>= 1) n += __shfl_xor(n, off, 64);
  if (sub == 0) a.len[base + mb] = n;
}

// ---------------------------------------------------------------- K4: offsets + header/trailer
__global__ __launch_bounds__(1024) void cavlc_offsets(CavlcArgs a) {
  const Geom& g = a.g;
  const int slot = blockIdx.x, n = g.nmb();
  const size_t base = static_cast<size_t>(slot) * n;
  __shared__ long long s_sum[1024];
  const int per = (n + blockDim.x - 1) / blockDim.x;
  const int i0 = threadIdx.x * per, i1 = min(n, i0 + per);
  long long loc = 0;
  for (int i = i0; i < i1; ++i) loc += a.len[base + i];
  s_sum[threadIdx.x] = loc;
  __syncthreads();
  for (int off = 1; off < blockDim.x; off <<= 1) {
    long long v = threadIdx.x >= off ? s_sum[threadIdx.x - off] : 0;
    __syncthreads();
    s_sum[threadIdx.x] += v;
    __syncthreads();
  }
  const long long hbits = a.hdr_nbits[slot];
  long long p = hbits + (threadIdx.x > 0 ? s_sum[threadIdx.x - 1] : 0);
  for (int i = i0; i < i1; ++i) {
    a.off[base + i] = p;
    p += a.len[base + i];
  }
  if (threadIdx.x == blockDim.x - 1) {
    uint32_t* words = a.words + slot * a.cap_words;
    long long pos = hbits + s_sum[blockDim.x - 1];
    // trailing mb_skip_run, rbsp_stop_one_bit, alignment
    WordSink s(words, pos);
    if (a.pslice && a.trail[slot] > 0) put_ue(s, static_cast<uint32_t>(a.trail[slot]));
    s.put(1, 1);
    long long endpos = pos + (a.pslice && a.trail[slot] > 0 ? 2 * (31 - __clz(a.trail[slot] + 1)) + 1 : 0) + 1;
    s.flush();
    long long total = (endpos + 7) & ~7ll;
    a.total_bits[slot] = total;
    a.slot_bytes[slot] = static_cast<int>(total >> 3);
    // slice header bits at position 0
    WordSink hs(words, 0);
    const uint32_t* hb = a.hdr_bits + slot * 16;
    for (int k = 0; k * 32 < hbits; ++k) hs.put(hb[k] >> (hbits - k * 32 >= 32 ? 0 : 32 - (hbits - k * 32)),
                                                   hbits - k * 32 >= 32 ? 32 : static_cast<int>(hbits - k * 32));
    hs.flush();
  }
}

// ---------------------------------------------------------------- K5: write
__global__ __launch_bounds__(64) void cavlc_write(CavlcArgs a) {
  const Geom& g = a.g;
  const int lane = threadIdx.x, sub = lane & 31;
  const int mb = blockIdx.x * 2 + (lane >> 5), slot = blockIdx.y;
  if (mb >= g.nmb()) return;
  const int mx = mb % g.wmb, my = mb / g.wmb;
  const size_t base = static_cast<size_t>(slot) * g.nmb();
  const CavlcMb& m = a.mbs[base + mb];
  const int n = sub < 28 ? a.blen[(base + mb) * 28 + sub] : 0;
  const int pre = lane_exscan32(n, lane);
  if (!m.coded || n == 0) return;
  const int16_t* c = a.coef + (base + mb) * h264::kCoefPerMb;
  WordSink ws(a.words + slot * a.cap_words, a.off[base + mb] + pre);
  if (sub == 0) mb_header_bits(ws, m, a.hdr[base + mb], a.pslice);
  else mb_block_bits(ws, sub, a.mbs, base, g.wmb, mx, my, m, c);
  ws.flush();
}

// ---------------------------------------------------------------- K6: compact to bytes
__global__ __launch_bounds__(256) void cavlc_compact(CavlcArgs a) {
  const int slot = blockIdx.x;
  long long off = 0;
  for (int s = 0; s < slot; ++s) off += a.slot_bytes[s];
  if (threadIdx.x == 0) a.out_off[slot] = off;
  const int nbytes = a.slot_bytes[slot];
  const uint32_t* words = a.words + slot * a.cap_words;
  uint8_t* dst = a.out + off;
  for (int i = threadIdx.x; i < nbytes; i += blockDim.x) {
    uint32_t w = words[i >> 2];
    dst[i] = static_cast<uint8_t>(w >> (24 - 8 * (i & 3)));
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

// per-MB scratch the caller allocates: the analysis record + 28 slot lengths
extern "C" size_t mivc_cavlc_mb_bytes() { return sizeof(CavlcMb) + 28 * sizeof(uint16_t); }

extern "C" void mivc_launch_cavlc(int B, int wmb, int hmb, const void* hdr, const int16_t* coef, void* mbs, int* len,
                                  long long* off, int* trail, long long* total_bits, int* slot_bytes, uint32_t* words,
                                  long long cap_words, const uint32_t* hdr_bits, const int* hdr_nbits, int pslice,
                                  int slice_qp, const int* slot_qp, uint8_t* out, long long* out_off,
                                  const uint8_t* nz, void* stream) {
  CavlcArgs a;
  a.nz = nz;
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.hdr = static_cast<const mivc::h264::MbHeader*>(hdr);
  a.coef = coef;
  const int nmb = wmb * hmb;
  a.mbs = static_cast<CavlcMb*>(mbs);
  a.blen = reinterpret_cast<uint16_t*>(static_cast<CavlcMb*>(mbs) + static_cast<size_t>(nmb) * B);
  a.len = len;
  a.off = off;
  a.trail = trail;
  a.total_bits = total_bits;
  a.slot_bytes = slot_bytes;
  a.words = words;
  a.cap_words = cap_words;
  a.hdr_bits = hdr_bits;
  a.hdr_nbits = hdr_nbits;
  a.pslice = pslice;
  a.slice_qp = slice_qp;
  a.slot_qp = slot_qp;
  a.out = out;
  a.out_off = out_off;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipMemsetAsync(words, 0, sizeof(uint32_t) * cap_words * B, s);
  hipLaunchKernelGGL(cavlc_analyze, dim3((nmb + 1) / 2, B), dim3(64), 0, s, a);
  hipLaunchKernelGGL(cavlc_scan, dim3(B), dim3(1024), 0, s, a);
  hipLaunchKernelGGL(cavlc_length, dim3((nmb + 1) / 2, B), dim3(64), 0, s, a);
  hipLaunchKernelGGL(cavlc_offsets, dim3(B), dim3(1024), 0, s, a);
  hipLaunchKernelGGL(cavlc_write, dim3((nmb + 1) / 2, B), dim3(64), 0, s, a);
  hipLaunchKernelGGL(cavlc_compact, dim3(B), dim3(256), 0, s, a);
}
