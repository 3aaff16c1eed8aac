// H.264 picture reconstruction on gfx950 from entropy-decoded records (SURVEY.md
// K-C1: the decode half of the transcode path, BASELINE config 3).
//
// The host parses CAVLC or CABAC (csrc/host/h264_decoder.cc, parse-only mode) into the
// same per-MB decision records the encoder produces (MbHeader) plus the quantised levels,
// packed: only non-zero 16-level chunks are stored, located through a per-MB bit mask (bits
// 0-15 luma blkIdx -- or, with the 8x8 transform, 8x8 block b8's levels 16k..16k+15 at
// bit b8 * 4 + k --, 16 Intra16x16 DC, 17 chroma DC Cb|Cr, 18-25 chroma AC comp*4+b) and
// the MB's first block index, plus every 4x4 block's vectors / reference indices, the
// reference lists, the weighted-prediction table and the deblocking boundary strengths.
// Pictures live in a per-slot decoded picture buffer ([B][dpb_n] planes):
//
//  * decode_inter_dpb: every P / B macroblock in parallel (grid = MBs x slots, one wave64
//    per MB): 6-tap luma MC per 4x4 block from LDS windows of its reference pictures,
//    eighth-sample chroma MC, default / explicit / implicit weighted bi-prediction, and
//    the 4x4 (DPP quad exchanges, grp_inv4x4) or 8x8 inverse transform;
//  * decode_intra_wavefront: intra MBs in MB wavefront order (one workgroup per slot, LDS
//    row-progress counters, as the intra encoder) -- Intra4x4, Intra8x8 (reference sample
//    filtering, 9 modes) and Intra16x16; all MBs of an I picture, only the intra MBs of a
//    P / B picture (their inter neighbours are final);
//  * the in-loop filter is the encoder's deblock kernel (deblock.hip) reading the parser's
//    boundary strengths.
//
// Reference parity: the reference decodes with ffmpeg inside the worker
// (client.go:115-118); the CPU decoder (h264_decoder.cc) is the bit-exact oracle.
#include "h264_t8.h"
#include "../common/h264_cabac_tables.h"

namespace mivc {
namespace gpu {

using h264::MbHeader;

struct DecodeArgs {
  Geom g;
  uint8_t *rec_y, *rec_u, *rec_v;        // decoded picture buffers (see dpb_n)
  const MbHeader* hdr;                   // [B, nmb]
  const uint32_t* mask;                  // [B, nmb] present blocks
  const uint32_t* off;                   // [B, nmb] first block (units of 16 levels, into coef)
  const int16_t* coef;                   // packed levels
  const int8_t* run;                     // [B] 0 idle, 1 I picture, 2 P picture
  int chroma_qp_offset;
  uint8_t* nz;                           // [B, nmb, 16] luma non-zero flags (raster), for deblocking
  int* err;
  // rec_* point at the per-slot decoded picture buffers, [B][dpb_n] pictures
  int dpb_n;
  const int16_t* cur_idx;  // [B] DPB index of the picture being decoded
  const int16_t* reftab;   // [B][2][32] DPB index of RefPicListX[i] (-1: none)
  const int16_t* wp;       // [B][kWpEntries] weighted-prediction tables (h264_decoder.h)
  // motion: per 8x8 quadrant in the MbHeader; MBF_SUB4 macroblocks (partitions below 8x8)
  // read their per-4x4 vectors / ref_idx from side-pool entry i4_modes[0..3] of `sub`
  // (h264::kSubEntry int16 per entry, indices already global to the batch step)
  const int16_t* sub;
};

// weighted-prediction table layout (mirrors mivc::h264::kWp* in h264_decoder.h)
enum : int { kWpLw = 4, kWpLo = 68, kWpCw = 132, kWpCo = 260, kWpImp = 388, kWpScale = 516, kWpFlags = 740,
             kWpEntries = 742 };

// Scaling lists of a picture (8.5.6, raster weights; 16 everywhere when the stream sends
// none): 4x4 list li = Intra Y / Cb / Cr, Inter Y / Cb / Cr (0..5), 8x8 list Intra / Inter Y.
// A DPB launch without tables (wp null) dequantises with flat weights.
struct Scaling {
  const int16_t* t;  // [kWpScale ..] of the slot's table, or null
  __device__ __forceinline__ int w4(int li, int x, int y) const { return t ? t[li * 16 + y * 4 + x] : 16; }
  __device__ __forceinline__ int w8(int li, int x, int y) const { return t ? t[96 + li * 64 + y * 8 + x] : 16; }
};
__device__ __forceinline__ Scaling scaling_of(const DecodeArgs& a, int slot) {
  return Scaling{a.wp ? a.wp + static_cast<size_t>(slot) * kWpEntries + kWpScale : nullptr};
}

// the picture being reconstructed (luma / chroma plane) of a slot
__device__ __forceinline__ uint8_t* rec_plane(const DecodeArgs& a, uint8_t* base, int slot, size_t psize) {
  if (a.dpb_n == 0) return base + static_cast<size_t>(slot) * psize;
  return base + (static_cast<size_t>(slot) * a.dpb_n + a.cur_idx[slot]) * psize;
}

// blkIdx -> 4x4 block column / row (no table: lane-varying lookups would be memory loads)
__device__ __forceinline__ int blk_x(int b) { return ((b >> 2) & 1) * 2 + (b & 1); }
__device__ __forceinline__ int blk_y(int b) { return ((b >> 3) & 1) * 2 + ((b >> 1) & 1); }

// level at scan position sp of block `bit` (0 if the block is absent)
__device__ __forceinline__ int level_at(const int16_t* coef, uint32_t mask, uint32_t off, int bit, int sp) {
  if (!((mask >> bit) & 1u)) return 0;
  const uint32_t idx = off + __builtin_popcount(mask & ((1u << bit) - 1u));
  return coef[static_cast<size_t>(idx) * 16 + sp];
}

// dequantised AC/4x4 residual row gy of a block (8.5.12.1): LevelScale4x4 = weight *
// normAdjust4x4; with the flat weight 16 this is level * normAdjust << qp/6.  skip_dc leaves
// (0, 0) at 0; li = the block's 4x4 scaling list
__device__ __forceinline__ void dequant_row(const int16_t* coef, uint32_t mask, uint32_t off, int bit, int gy, int qp,
                                            bool skip_dc, int* v, const Scaling& sc, int li) {
  const int qm = qp % 6, qs = qp / 6;
  const int d0 = h264::kDequantV[qm][0], d1 = h264::kDequantV[qm][1], d2 = h264::kDequantV[qm][2];
  const bool have = (mask >> bit) & 1u;
  const int16_t* c = coef + static_cast<size_t>(off + __builtin_popcount(mask & ((1u << bit) - 1u))) * 16;
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    const int cls = pos_class(x, gy);
    const int ls = sc.w4(li, x, gy) * (cls == 0 ? d0 : (cls == 1 ? d1 : d2));
    const int lv = (have && !(skip_dc && x == 0 && gy == 0)) ? c[zzinv(x, gy)] : 0;
    v[x] = qs >= 4 ? (lv * ls) << (qs - 4) : (lv * ls + (1 << (3 - qs))) >> (4 - qs);
  }
}

// chroma DC of block cb after the 2x2 inverse transform and scaling (8.5.11)
__device__ __forceinline__ int chroma_dc_value(const int16_t* coef, uint32_t mask, uint32_t off, int comp, int cb,
                                               int qpc, int w00) {
  if (!((mask >> 17) & 1u)) return 0;
  const int16_t* c = coef + static_cast<size_t>(off + __builtin_popcount(mask & ((1u << 17) - 1u))) * 16 + comp * 4;
  const int c0 = c[0], c1 = c[1], c2 = c[2], c3 = c[3];
  const int f = cb == 0 ? c0 + c1 + c2 + c3 : (cb == 1 ? c0 - c1 + c2 - c3 : (cb == 2 ? c0 + c1 - c2 - c3 : c0 - c1 - c2 + c3));
  const int ls = w00 * h264::kDequantV[qpc % 6][0];
  return ((f * ls) << (qpc / 6)) >> 5;
}

__device__ __forceinline__ uint32_t pack4(const int* p) {
  return static_cast<uint32_t>(p[0]) | static_cast<uint32_t>(p[1]) << 8 | static_cast<uint32_t>(p[2]) << 16 |
         static_cast<uint32_t>(p[3]) << 24;
}

// ============================================================== inter macroblocks, DPB layout
// Every P / B macroblock of every slot in parallel (one wave64 per MB): per raster 4x4
// block and list its own vector and reference picture (sub-8x8 partitions, B_8x8, direct
// modes and several references all arrive resolved by the host parser), 6-tap luma MC
// from a 9x9 LDS window per block, eighth-sample chroma MC, default / explicit / implicit
// weighted sample prediction (8.4.2.3), and the 4x4 or 8x8 (8.5.13) inverse transform.

// LevelScale8x8 = weight * normAdjust8x8 (8.5.9)
__device__ __forceinline__ int level_scale8(int m, int x, int y, int w) {
  int k;
  if ((x & 3) == 0 && (y & 3) == 0) k = 0;
  else if ((x & 1) && (y & 1)) k = 1;
  else if ((x & 3) == 2 && (y & 3) == 2) k = 2;
  else if (((x & 3) == 0 && (y & 1)) || ((x & 1) && (y & 3) == 0)) k = 3;
  else if (((x & 3) == 0 && (y & 3) == 2) || ((x & 3) == 2 && (y & 3) == 0)) k = 4;
  else k = 5;
  constexpr int t[6][6] = {{20, 18, 32, 19, 25, 24}, {22, 19, 35, 21, 28, 26}, {26, 23, 42, 24, 33, 31},
                           {28, 25, 45, 26, 35, 33}, {32, 28, 51, 30, 40, 38}, {36, 32, 58, 34, 46, 43}};
  return w * t[m][k];
}

// one 8-point pass of the 8x8 inverse transform (8.5.13.2), in place, stride s

// weighted sample prediction of one sample (8.4.2.3); r0 / r1 = ref_idx (-1: list unused)
__device__ __forceinline__ int weigh(const int16_t* w, bool chroma, int comp, int r0, int r1, int p0, int p1) {
  const int mode = w[0];
  const bool b0 = r0 >= 0, b1 = r1 >= 0;
  if (mode == 1) {
    const int logwd = chroma ? w[2] : w[1];
    int w0 = 0, o0 = 0, w1 = 0, o1 = 0;
    if (b0) {
      w0 = chroma ? w[kWpCw + r0 * 2 + comp] : w[kWpLw + r0];
      o0 = chroma ? w[kWpCo + r0 * 2 + comp] : w[kWpLo + r0];
    }
    if (b1) {
      w1 = chroma ? w[kWpCw + (32 + r1) * 2 + comp] : w[kWpLw + 32 + r1];
      o1 = chroma ? w[kWpCo + (32 + r1) * 2 + comp] : w[kWpLo + 32 + r1];
    }
    if (b0 && b1) return h264::clip1(((p0 * w0 + p1 * w1 + (1 << logwd)) >> (logwd + 1)) + ((o0 + o1 + 1) >> 1));
    const int p = b0 ? p0 : p1, ww = b0 ? w0 : w1, o = b0 ? o0 : o1;
    return h264::clip1(logwd >= 1 ? ((p * ww + (1 << (logwd - 1))) >> logwd) + o : p * ww + o);
  }
  if (b0 && b1) {
    if (mode == 2) {
      const int w0 = w[kWpImp + ((r0 & 7) * 8 + (r1 & 7)) * 2], w1 = w[kWpImp + ((r0 & 7) * 8 + (r1 & 7)) * 2 + 1];
      return h264::clip1((p0 * w0 + p1 * w1 + 32) >> 6);
    }
    return (p0 + p1 + 1) >> 1;
  }
  return b0 ? p0 : p1;
}

constexpr int kBW = 9;  // 4x4 block + 6-tap support (-2 .. +6)

__global__ __launch_bounds__(64) void decode_inter_dpb(DecodeArgs a) {
  const Geom& g = a.g;
  int mb, slot;
  xcd_unit_slot(mb, slot);
  if (a.run[slot] != 2) return;
  const size_t o = static_cast<size_t>(slot) * g.nmb() + mb;
  const MbHeader* H = a.hdr + o;
  if (h264::mbk_is_intra(H->kind)) return;
  // reference windows: per (list, 4x4 block) 9x9 when the MB carries sub-8x8 motion, else per
  // (list, 8x8 quadrant) 13x13 (one vector per quadrant: the four blocks' windows overlap)
  // in rows of kQP bytes, staged a row per lane with dword loads
  constexpr int kQP = 16, kQW = 13;
  __shared__ __attribute__((aligned(16))) uint8_t win[2][16][kBW * kBW];
  __shared__ int d8[4][64];
  const int lane = threadIdx.x;
  const int mx = mb % g.wmb, my = mb / g.wmb;
  const int W = g.W, Hh = g.H, cw = g.cw(), ch = g.ch();
  const int X0 = mx * 16, Y0 = my * 16;
  const int qp = H->qp;
  const int qpc = h264::chroma_qp(qp, a.chroma_qp_offset);
  const uint32_t mask = a.mask[o], off = a.off[o];
  const bool t8 = (H->flags & h264::MBF_T8x8) != 0;
  const int D = a.dpb_n;
  const int nmb = g.nmb();
  const int16_t* rt = a.reftab + slot * 64;
  const bool sub4 = (H->flags & h264::MBF_SUB4) != 0;
  const int16_t* se = nullptr;
  if (sub4) {
    uint32_t si;
    __builtin_memcpy(&si, H->i4_modes, 4);
    se = a.sub + static_cast<size_t>(si) * h264::kSubEntry;
  }
  const int16_t* wt = a.wp + static_cast<size_t>(slot) * kWpEntries;
  const Scaling sc = scaling_of(a, slot);
  auto quad = [](int rb) { return ((rb & 3) >> 1) + 2 * (rb >> 3); };
  auto mv_of = [&](int l, int rb, int c) {
    return static_cast<int>(sub4 ? se[(l * 16 + rb) * 2 + c] : H->mv[l][quad(rb)][c]);
  };
  auto ref_of = [&](int l, int rb) {
    return static_cast<int>(sub4 ? reinterpret_cast<const int8_t*>(se + 64)[l * 16 + rb] : H->ref[l][quad(rb)]);
  };
  auto pic_of = [&](int l, int r) {  // DPB index of RefPicListl[r], validated
    const int di = (r >= 0 && r < 32) ? rt[l * 32 + r] : -1;
    if (di < 0 || di >= D) {
      atomicOr(a.err, 16);
      return 0;
    }
    return di;
  };

  // ---- stage the reference windows (clamped: unrestricted vectors)
  uint8_t* qwin = &win[0][0][0];  // quadrant mode: [l][q][kQW rows][kQP] inside the same storage
  static_assert(2 * 4 * kQW * kQP <= 2 * 16 * kBW * kBW, "quadrant windows fit the block windows' storage");
  if (sub4) {
    for (int i = lane; i < 2 * 16 * kBW * kBW; i += 64) {
      const int l = i / (16 * kBW * kBW), j0 = i - l * 16 * kBW * kBW;
      const int rb = j0 / (kBW * kBW), j = j0 - rb * kBW * kBW;
      const int r = ref_of(l, rb);
      if (r < 0) continue;
      const int di = pic_of(l, r);
      const int rr = j / kBW, cc = j - rr * kBW;
      const int x = clampi(X0 + (rb & 3) * 4 + (mv_of(l, rb, 0) >> 2) - 2 + cc, 0, W - 1);
      const int y = clampi(Y0 + (rb >> 2) * 4 + (mv_of(l, rb, 1) >> 2) - 2 + rr, 0, Hh - 1);
      win[l][rb][j] = a.rec_y[(static_cast<size_t>(slot) * D + di) * g.ysize() + static_cast<size_t>(y) * W + x];
    }
  } else {
    for (int i = lane; i < 2 * 4 * kQW; i += 64) {  // one window row per lane
      const int l = i / (4 * kQW), j = i - l * 4 * kQW;
      const int q = j / kQW, rr = j - q * kQW;
      const int r = H->ref[l][q];
      if (r < 0) continue;
      const int di = pic_of(l, r);
      const int x0 = X0 + (q & 1) * 8 + (H->mv[l][q][0] >> 2) - 2;
      const int y = clampi(Y0 + (q >> 1) * 8 + (H->mv[l][q][1] >> 2) - 2 + rr, 0, Hh - 1);
      const uint8_t* row = a.rec_y + (static_cast<size_t>(slot) * D + di) * g.ysize() + static_cast<size_t>(y) * W;
      uint32_t* dst = reinterpret_cast<uint32_t*>(qwin + ((l * 4 + q) * kQW + rr) * kQP);
      if (x0 >= 0 && x0 + 16 <= W) {  // inside the row: four aligned dwords cover the 13 bytes
        const int xa = x0 & ~3, sh = x0 & 3;
        const uint32_t* s4 = reinterpret_cast<const uint32_t*>(row + xa);
        const uint32_t e0 = s4[0], e1 = s4[1], e2 = s4[2], e3 = s4[3];
        dst[0] = __builtin_amdgcn_alignbyte(e1, e0, sh);
        dst[1] = __builtin_amdgcn_alignbyte(e2, e1, sh);
        dst[2] = __builtin_amdgcn_alignbyte(e3, e2, sh);
        dst[3] = __builtin_amdgcn_alignbyte(0u, e3, sh);  // byte 12 (the last one used) lies in e3
      } else {
        uint32_t w4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          uint32_t v = 0;
#pragma unroll
          for (int b = 0; b < 4; ++b) v |= static_cast<uint32_t>(row[clampi(x0 + 4 * k + b, 0, W - 1)]) << (8 * b);
          w4[k] = v;
        }
        dst[0] = w4[0];
        dst[1] = w4[1];
        dst[2] = w4[2];
        dst[3] = w4[3];
      }
    }
  }
  // ---- 8x8 transform: dequantise (lane = b8 * 16 + t, four levels each), then row and
  // column passes in LDS
  if (t8) {
    const int b8 = lane >> 4, t = lane & 15;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = t * 4 + k;  // scan index
      const int pos = h264::kZigzag8x8[i];
      const int x = pos & 7, y = pos >> 3;
      const int lv = level_at(a.coef, mask, off, b8 * 4 + (i >> 4), i & 15);
      const int ls = level_scale8(qp % 6, x, y, sc.w8(1, x, y));
      d8[b8][pos] = qp >= 36 ? (lv * ls) << (qp / 6 - 6) : (lv * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
    }
  }
  __syncthreads();
  if (t8) {
    const int b8 = lane >> 4, t = lane & 15;
    if (t < 8) idct8_pass(&d8[b8][t * 8], 1);
    __syncthreads();
    if (t < 8) idct8_pass(&d8[b8][t], 8);
    __syncthreads();
  }

  // ---- luma: lane = blkIdx * 4 + row
  {
    const int blk = lane >> 2, gy = lane & 3;
    const int bx = blk_x(blk), by = blk_y(blk), rb = bx + 4 * by;
    const int r0 = ref_of(0, rb), r1 = ref_of(1, rb);
    int pl[2][4];
#pragma unroll
    for (int l = 0; l < 2; ++l) {
      const int r = l ? r1 : r0;
      const int fx = mv_of(l, rb, 0) & 3, fy = mv_of(l, rb, 1) & 3;
      // this block's 9x9 window: its own (sub-8x8 motion) or inside its quadrant's 13x13
      const uint8_t* w = sub4 ? win[l][rb] : qwin + (l * 4 + quad(rb)) * kQW * kQP + (by & 1) * 4 * kQP + (bx & 1) * 4;
      const int pitch = sub4 ? kBW : kQP;
      auto ref = [&](int x, int y) { return static_cast<int>(w[(y + 2) * pitch + x + 2]); };
#pragma unroll
      for (int x = 0; x < 4; ++x) pl[l][x] = r >= 0 ? h264::mc_luma_sample(ref, x, gy, fx, fy) : 0;
    }
    int v[4], pr[4];
    if (t8) {
      const int Y = by * 4 + gy;
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const int X = bx * 4 + x;
        v[x] = (d8[(Y >> 3) * 2 + (X >> 3)][(Y & 7) * 8 + (X & 7)] + 32) >> 6;
      }
    } else {
      dequant_row(a.coef, mask, off, blk, gy, qp, false, v, sc, 3);
      grp_inv4x4(v, lane & ~3, gy);
    }
#pragma unroll
    for (int x = 0; x < 4; ++x) pr[x] = h264::clip1(weigh(wt, false, 0, r0, r1, pl[0][x], pl[1][x]) + v[x]);
    uint8_t* recy = rec_plane(a, a.rec_y, slot, g.ysize());
    *reinterpret_cast<uint32_t*>(recy + static_cast<size_t>(Y0 + by * 4 + gy) * W + X0 + bx * 4) = pack4(pr);
    if (lane < 16) a.nz[o * 16 + blk_x(lane) + 4 * blk_y(lane)] = (mask >> lane) & 1u;
  }
  // ---- chroma: (lane & 31) = comp * 16 + block * 4 + row; every chroma sample takes the
  // vector of the luma 4x4 block it lies under; lanes 32-63 mirror 0-31 (transform partners)
  {
    const int cl = lane & 31, comp = cl >> 4, cb = (cl >> 2) & 3, gy = cl & 3;
    const int cbx = (cb & 1) * 4, cby = (cb >> 1) * 4;
    const int Yc = cby + gy;
    int pr[4], v[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int Xc = cbx + x;
      const int rb = (Xc >> 1) + 4 * (Yc >> 1);
      const int r0 = ref_of(0, rb), r1 = ref_of(1, rb);
      int pc[2];
#pragma unroll
      for (int l = 0; l < 2; ++l) {
        const int r = l ? r1 : r0;
        pc[l] = 0;
        if (r >= 0) {
          const int di = pic_of(l, r);
          const uint8_t* refc = (comp == 0 ? a.rec_u : a.rec_v) + (static_cast<size_t>(slot) * D + di) * g.csize();
          const int cmx = mv_of(l, rb, 0), cmy = mv_of(l, rb, 1);
          const int xf = cmx & 7, yf = cmy & 7;
          const int xi = mx * 8 + Xc + (cmx >> 3), yi = my * 8 + Yc + (cmy >> 3);
          const int x0 = clampi(xi, 0, cw - 1), x1 = clampi(xi + 1, 0, cw - 1);
          const int y0 = clampi(yi, 0, ch - 1), y1 = clampi(yi + 1, 0, ch - 1);
          const int A = refc[static_cast<size_t>(y0) * cw + x0], Bv = refc[static_cast<size_t>(y0) * cw + x1];
          const int C = refc[static_cast<size_t>(y1) * cw + x0], Dv = refc[static_cast<size_t>(y1) * cw + x1];
          pc[l] = ((8 - xf) * (8 - yf) * A + xf * (8 - yf) * Bv + (8 - xf) * yf * C + xf * yf * Dv + 32) >> 6;
        }
      }
      pr[x] = weigh(wt, true, comp, r0, r1, pc[0], pc[1]);
    }
    dequant_row(a.coef, mask, off, 18 + comp * 4 + cb, gy, qpc, true, v, sc, 4 + comp);
    if (gy == 0) v[0] = chroma_dc_value(a.coef, mask, off, comp, cb, qpc, sc.w4(4 + comp, 0, 0));
    grp_inv4x4(v, lane & ~3, gy);
#pragma unroll
    for (int x = 0; x < 4; ++x) pr[x] = h264::clip1(pr[x] + v[x]);
    if (lane < 32) {
      uint8_t* recc = rec_plane(a, comp == 0 ? a.rec_u : a.rec_v, slot, g.csize());
      *reinterpret_cast<uint32_t*>(recc + static_cast<size_t>(my * 8 + Yc) * cw + mx * 8 + cbx) = pack4(pr);
    }
  }
}

// ============================================================== intra macroblocks
// Intra4x4 neighbour availability of block b (top-right per 6.4.11.4 / the blkIdx order)
__device__ __forceinline__ int i4_avail(int b, int mbav) {
  const int bx = blk_x(b), by = blk_y(b);
  const bool left = bx > 0 || (mbav & h264::AV_LEFT), top = by > 0 || (mbav & h264::AV_TOP);
  int av = 0;
  if (left) av |= h264::AV_LEFT;
  if (top) av |= h264::AV_TOP;
  if (left && top) av |= h264::AV_TOPLEFT;
  bool tr;
  if (b == 3 || b == 7 || b == 11 || b == 13 || b == 15) tr = false;
  else if (b == 5) tr = (mbav & h264::AV_TOPRIGHT) != 0;
  else if (b == 0 || b == 1 || b == 4) tr = (mbav & h264::AV_TOP) != 0;
  else tr = true;
  if (tr) av |= h264::AV_TOPRIGHT;
  return av;
}

constexpr int kDecIntraWaves = 8;
constexpr int TS = kTileStride;

struct DecIntraShared {
  uint8_t tile[17 * TS];            // luma: row 0 / col 0 = reconstructed neighbours
  int16_t res[16][16];              // Intra4x4 residual per blkIdx (raster)
  int e4[16];                       // Intra4x4 neighbour vector of the current block
  int lv16dc[16];                   // Intra16x16 DC after the inverse Hadamard + scaling (raster)
  uint8_t ctop[2][9], cleft[2][8];  // chroma neighbours [comp][-1..7]
  int cdcp[2][4];                   // chroma DC predictions per (comp, block)
  int saved_x;
  uint8_t saved_y[16];
  uint8_t saved_c[2][8];
  // Intra8x8: residual (16x16 raster, before the final rounding), the row above the MB at
  // x = 16..23 (top-right of 8x8 block 1), and the filtered references of the current block
  int r8[256];
  uint8_t tr8[8];
  int e8t[16], e8l[8], e8tl;
  int f8t[16], f8l[8], f8tl;
};

// Intra_8x8 sample (8.3.2.2.2 .. 8.3.2.2.10) from the filtered references ft / fl / ftl

__device__ __forceinline__ void decode_intra_mb(const DecodeArgs& a, DecIntraShared& S, int slot, int mx, int my) {
  const Geom& g = a.g;
  const int lane = lane_id();
  const int gy = lane & 3;
  const int W = g.W, cw = g.cw();
  const int X0 = mx * 16, Y0 = my * 16;
  const size_t o = static_cast<size_t>(slot) * g.nmb() + my * g.wmb + mx;
  const MbHeader* H = a.hdr + o;
  const int kind = __builtin_amdgcn_readfirstlane(H->kind);
  const int qp = __builtin_amdgcn_readfirstlane(H->qp);
  const int qpc = h264::chroma_qp(qp, a.chroma_qp_offset);
  const int mode16 = __builtin_amdgcn_readfirstlane(H->i16_mode);
  const int cmode = __builtin_amdgcn_readfirstlane(H->chroma_mode);
  const uint32_t mask = __builtin_amdgcn_readfirstlane(a.mask[o]);
  const uint32_t off = __builtin_amdgcn_readfirstlane(a.off[o]);
  uint8_t* recy = rec_plane(a, a.rec_y, slot, g.ysize());
  // neighbour MBs are available when inside the picture and in this MB's slice (the
  // parser's records carry the slice index in pad0; 6.4.8)
  const int sl = __builtin_amdgcn_readfirstlane(H->pad0);
  const Scaling sc = scaling_of(a, slot);
  // constrained_intra_pred_flag: inter neighbours are not available for intra prediction
  const bool cip = a.wp && (a.wp[static_cast<size_t>(slot) * kWpEntries + kWpFlags] & 1);
  auto same = [&](int dx, int dy) {
    const MbHeader& n = H[dy * g.wmb + dx];
    return static_cast<int>(n.pad0) == sl && (!cip || h264::mbk_is_intra(n.kind));
  };
  int mbav = 0;
  if (mx > 0 && same(-1, 0)) mbav |= h264::AV_LEFT;
  if (my > 0 && same(0, -1)) mbav |= h264::AV_TOP;
  if (mx > 0 && my > 0 && same(-1, -1)) mbav |= h264::AV_TOPLEFT;
  if (my > 0 && mx < g.wmb - 1 && same(1, -1)) mbav |= h264::AV_TOPRIGHT;

  if (kind == h264::MBK_IPCM) {
    // I_PCM: the samples ride in the level pool (24 chunks: luma raster, Cb, Cr)
    const int16_t* pcm = a.coef + static_cast<size_t>(off) * 16;
    {
      const int y = lane >> 2, x4 = (lane & 3) * 4;
      uint32_t word = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) word |= static_cast<uint32_t>(pcm[y * 16 + x4 + k] & 0xFF) << (8 * k);
      *reinterpret_cast<uint32_t*>(recy + static_cast<size_t>(Y0 + y) * W + X0 + x4) = word;
      if ((lane & 3) == 3) S.saved_y[y] = static_cast<uint8_t>(word >> 24);
    }
    if (lane < 32) {
      const int comp = lane >> 4, y = (lane >> 1) & 7, x4 = (lane & 1) * 4;
      uint32_t word = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) word |= static_cast<uint32_t>(pcm[256 + comp * 64 + y * 8 + x4 + k] & 0xFF) << (8 * k);
      uint8_t* recc = rec_plane(a, comp == 0 ? a.rec_u : a.rec_v, slot, g.csize());
      *reinterpret_cast<uint32_t*>(recc + static_cast<size_t>(my * 8 + y) * cw + mx * 8 + x4) = word;
      if (lane & 1) S.saved_c[comp][y] = static_cast<uint8_t>(word >> 24);
    }
    if (lane < 16) a.nz[o * 16 + blk_x(lane) + 4 * blk_y(lane)] = 1;
    if (lane == 0) S.saved_x = my * g.wmb + mx;  // raster index: rows differ
    wave_sync();
    return;
  }

  // ---- stage the reconstructed neighbourhood
  if (lane < 21) {  // tile row 0: x = X0-1 .. X0+19
    const int x = X0 - 1 + lane;
    const bool ok = x < W && (lane == 0 ? (mbav & h264::AV_TOPLEFT) : lane < 17 ? (mbav & h264::AV_TOP)
                                                                         : (mbav & h264::AV_TOPRIGHT));
    S.tile[lane] = ok ? recy[static_cast<size_t>(Y0 - 1) * W + x] : 0;
  } else if (lane >= 24 && lane < 32) {  // x = X0+16 .. X0+23 (Intra8x8 block 1's top-right)
    const int x = X0 + 16 + (lane - 24);
    const bool ok = (mbav & h264::AV_TOPRIGHT) && x < W;
    S.tr8[lane - 24] = ok ? recy[static_cast<size_t>(Y0 - 1) * W + x] : 0;
  } else if (lane >= 32 && lane < 48) {  // tile col 0, rows 1..16
    const int r = lane - 32;
    uint8_t v = 0;
    if (mbav & h264::AV_LEFT) v = S.saved_x == my * g.wmb + mx - 1 ? S.saved_y[r] : recy[static_cast<size_t>(Y0 + r) * W + X0 - 1];
    S.tile[(r + 1) * TS] = v;
  }
  if (lane < 18) {
    const int c = lane / 9, i = lane % 9;
    const uint8_t* rc = rec_plane(a, c == 0 ? a.rec_u : a.rec_v, slot, g.csize());
    const int x = mx * 8 - 1 + i;
    S.ctop[c][i] = (i == 0 ? (mbav & h264::AV_TOPLEFT) : (mbav & h264::AV_TOP)) ? rc[static_cast<size_t>(my * 8 - 1) * cw + x] : 0;
  } else if (lane >= 48) {
    const int c = (lane - 48) >> 3, i = (lane - 48) & 7;
    const uint8_t* rc = rec_plane(a, c == 0 ? a.rec_u : a.rec_v, slot, g.csize());
    uint8_t v = 0;
    if (mbav & h264::AV_LEFT) v = S.saved_x == my * g.wmb + mx - 1 ? S.saved_c[c][i] : rc[static_cast<size_t>(my * 8 + i) * cw + mx * 8 - 1];
    S.cleft[c][i] = v;
  }
  wave_sync();
  if (lane >= 16 && lane < 24) {
    const int c = (lane - 16) >> 2, b = (lane - 16) & 3;
    S.cdcp[c][b] = h264::chroma_dc(S.ctop[c] + 1, S.cleft[c], mbav, b & 1, b >> 1);
  }

  // ---- luma
  const int blk = lane >> 2;
  const int bx = blk_x(blk), by = blk_y(blk);
  if (kind == h264::MBK_I16x16) {
    if (lane == 0) {
      int d[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) d[h264::kZigzag4x4[i]] = level_at(a.coef, mask, off, 16, i);
      h264::hadamard4x4(d);
      const int ls = sc.w4(0, 0, 0) * h264::kDequantV[qp % 6][0];
#pragma unroll
      for (int r = 0; r < 16; ++r)
        S.lv16dc[r] = qp >= 36 ? (d[r] * ls) << (qp / 6 - 6) : (d[r] * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
    }
    uint8_t top[16], left[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      top[i] = S.tile[1 + i];
      left[i] = S.tile[(i + 1) * TS];
    }
    int pa = 0, pb = 0, pc = 0;
    if (mode16 == 3) h264::i16_plane_params(top, left, static_cast<int>(S.tile[0]), &pa, &pb, &pc);
    const int dc = mode16 == 2 ? h264::i16_dc(top, left, mbav) : 0;
    int v[4], pr[4];
    dequant_row(a.coef, mask, off, blk, gy, qp, true, v, sc, 0);
    wave_sync();
    if (gy == 0) v[0] = S.lv16dc[bx + 4 * by];
    grp_inv4x4(v, lane & ~3, gy);
    const int Yr = by * 4 + gy;
    const int lft = S.tile[(Yr + 1) * TS];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int X = bx * 4 + x;
      const int p = mode16 == 0 ? static_cast<int>(S.tile[1 + X])
                  : (mode16 == 1 ? lft : (mode16 == 2 ? dc : h264::clip1((pa + pb * (X - 7) + pc * (Yr - 7) + 16) >> 5)));
      pr[x] = h264::clip1(p + v[x]);
    }
    wave_sync();
    uint8_t* row = S.tile + (Yr + 1) * TS + bx * 4 + 1;
#pragma unroll
    for (int x = 0; x < 4; ++x) row[x] = static_cast<uint8_t>(pr[x]);
  } else if (kind == h264::MBK_I8x8) {
    // Intra8x8: the four residual blocks at once (dequantise, 8x8 inverse transform), then
    // the four predictions in order from reference-filtered neighbours (8.3.2.2.1)
    {
      const int b8 = lane >> 4, t = lane & 15, ox = (b8 & 1) * 8, oy = (b8 >> 1) * 8;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int i = t * 4 + k;
        const int pos = h264::kZigzag8x8[i];
        const int x = pos & 7, y = pos >> 3;
        const int lv = level_at(a.coef, mask, off, b8 * 4 + (i >> 4), i & 15);
        const int ls = level_scale8(qp % 6, x, y, sc.w8(0, x, y));
        S.r8[(oy + y) * 16 + ox + x] = qp >= 36 ? (lv * ls) << (qp / 6 - 6) : (lv * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
      }
      wave_sync();
      if (t < 8) idct8_pass(&S.r8[(oy + t) * 16 + ox], 1);
      wave_sync();
      if (t < 8) idct8_pass(&S.r8[oy * 16 + ox + t], 16);
      wave_sync();
    }
    for (int b8 = 0; b8 < 4; ++b8) {
      const int bx = (b8 & 1) * 8, by = (b8 >> 1) * 8;
      const bool has_top = by > 0 || (mbav & h264::AV_TOP);
      const bool has_left = bx > 0 || (mbav & h264::AV_LEFT);
      const bool has_tl = b8 == 3 || (b8 == 0 ? (mbav & h264::AV_TOPLEFT) != 0
                                              : (b8 == 1 ? (mbav & h264::AV_TOP) != 0 : (mbav & h264::AV_LEFT) != 0));
      const bool has_tr = b8 == 2 || (b8 == 0 ? (mbav & h264::AV_TOP) != 0 : (b8 == 1 && (mbav & h264::AV_TOPRIGHT)));
      const uint8_t* above = S.tile + by * TS + bx + 1;  // row above the block, x = 0
      if (lane < 16) {
        int v = lane < 8 ? above[lane] : (has_tr ? (b8 == 1 ? S.tr8[lane - 8] : above[lane]) : above[7]);
        S.e8t[lane] = v;
      } else if (lane < 24) {
        S.e8l[lane - 16] = S.tile[(by + 1 + lane - 16) * TS + bx];
      } else if (lane == 24) {
        S.e8tl = S.tile[by * TS + bx];
      }
      wave_sync();
      const int tl = S.e8tl;
      if (lane < 16 && has_top) {
        const int* t = S.e8t;
        int f;
        if (lane == 0) f = has_tl ? (tl + 2 * t[0] + t[1] + 2) >> 2 : (3 * t[0] + t[1] + 2) >> 2;
        else if (lane == 15) f = (t[14] + 3 * t[15] + 2) >> 2;
        else f = (t[lane - 1] + 2 * t[lane] + t[lane + 1] + 2) >> 2;
        S.f8t[lane] = f;
      } else if (lane >= 16 && lane < 24 && has_left) {
        const int* l = S.e8l;
        const int y = lane - 16;
        int f;
        if (y == 0) f = has_tl ? (tl + 2 * l[0] + l[1] + 2) >> 2 : (3 * l[0] + l[1] + 2) >> 2;
        else if (y == 7) f = (l[6] + 3 * l[7] + 2) >> 2;
        else f = (l[y - 1] + 2 * l[y] + l[y + 1] + 2) >> 2;
        S.f8l[y] = f;
      } else if (lane == 24) {
        int f = 0;
        if (has_tl) {
          if (has_top && has_left) f = (S.e8t[0] + 2 * tl + S.e8l[0] + 2) >> 2;
          else if (has_top) f = (3 * tl + S.e8t[0] + 2) >> 2;
          else if (has_left) f = (3 * tl + S.e8l[0] + 2) >> 2;
          else f = tl;
        }
        S.f8tl = f;
      }
      wave_sync();
      const int mode = __builtin_amdgcn_readfirstlane(H->i4_modes[b8 * 4]);
      int dc = 128;
      if (mode == 2) {
        int st = 0, sl = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          st += has_top ? S.f8t[i] : 0;
          sl += has_left ? S.f8l[i] : 0;
        }
        dc = (has_top && has_left) ? (st + sl + 8) >> 4 : (has_left ? (sl + 4) >> 3 : (has_top ? (st + 4) >> 3 : 128));
      }
      const int x = lane & 7, y = lane >> 3;
      const int pr = i8_pred_sample(mode, x, y, S.f8t, S.f8l, S.f8tl, dc);
      const int rv = (S.r8[(by + y) * 16 + bx + x] + 32) >> 6;
      S.tile[(by + 1 + y) * TS + bx + 1 + x] = static_cast<uint8_t>(h264::clip1(pr + rv));
      wave_sync();
    }
  } else {
    // Intra4x4: all 16 residual blocks at once, then the 16 predictions in order
    {
      int v[4];
      dequant_row(a.coef, mask, off, blk, gy, qp, false, v, sc, 0);
      grp_inv4x4(v, lane & ~3, gy);
#pragma unroll
      for (int x = 0; x < 4; ++x) S.res[blk][gy * 4 + x] = static_cast<int16_t>(v[x]);
    }
    wave_sync();
    for (int b = 0; b < 16; ++b) {
      const int cbx = blk_x(b), cby = blk_y(b);
      const int av = i4_avail(b, mbav);
      if (lane < 13) {  // neighbour vector e[] of h264::i4_pred_sample, one entry per lane
        const uint8_t* rowp = S.tile + (cby * 4) * TS + cbx * 4;
        int v;
        if (lane == 0) v = rowp[0];
        else if (lane < 5) v = rowp[lane];
        else if (lane < 9) v = (av & h264::AV_TOPRIGHT) ? rowp[lane] : rowp[4];
        else v = S.tile[(cby * 4 + 1 + lane - 9) * TS + cbx * 4];
        S.e4[lane] = v;
      }
      wave_sync();
      const int mode = __builtin_amdgcn_readfirstlane(H->i4_modes[b]);
      if (lane < 4) {
        int pr[4];
#pragma unroll
        for (int x = 0; x < 4; ++x) pr[x] = h264::i4_pred_sample(mode, av, S.e4, x, gy);
        uint8_t* row = S.tile + (cby * 4 + gy + 1) * TS + cbx * 4 + 1;
#pragma unroll
        for (int x = 0; x < 4; ++x) row[x] = static_cast<uint8_t>(h264::clip1(pr[x] + S.res[b][gy * 4 + x]));
      }
      wave_sync();
    }
  }
  wave_sync();
  {  // write the luma reconstruction
    const int y = lane >> 2, x4 = (lane & 3) * 4;
    uint32_t word = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) word |= static_cast<uint32_t>(S.tile[(y + 1) * TS + x4 + k + 1]) << (8 * k);
    *reinterpret_cast<uint32_t*>(recy + static_cast<size_t>(Y0 + y) * W + X0 + x4) = word;
  }
  if (lane < 16) a.nz[o * 16 + blk_x(lane) + 4 * blk_y(lane)] = (mask >> lane) & 1u;

  // ---- chroma: (lane & 31) = comp * 16 + block * 4 + row
  {
    const int cl = lane & 31, comp = cl >> 4, cb = (cl >> 2) & 3;
    const int cbx = (cb & 1) * 4, cby = (cb >> 1) * 4;
    int pa = 0, pb = 0, pc = 0;
    if (cmode == 3) h264::chroma_plane_params(S.ctop[comp] + 1, S.cleft[comp], static_cast<int>(S.ctop[comp][0]), &pa, &pb, &pc);
    int v[4], pr[4];
    dequant_row(a.coef, mask, off, 18 + comp * 4 + cb, gy, qpc, true, v, sc, 1 + comp);
    if (gy == 0) v[0] = chroma_dc_value(a.coef, mask, off, comp, cb, qpc, sc.w4(1 + comp, 0, 0));
    grp_inv4x4(v, lane & ~3, gy);
    const int Yc = cby + gy;
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int X = cbx + x;
      const int p = cmode == 0 ? S.cdcp[comp][cb]
                  : (cmode == 1 ? S.cleft[comp][Yc]
                  : (cmode == 2 ? S.ctop[comp][1 + X] : h264::clip1((pa + pb * (X - 3) + pc * (Yc - 3) + 16) >> 5)));
      pr[x] = h264::clip1(p + v[x]);
    }
    const uint32_t word = pack4(pr);
    if (lane < 32) {
      uint8_t* recc = rec_plane(a, comp == 0 ? a.rec_u : a.rec_v, slot, g.csize());
      *reinterpret_cast<uint32_t*>(recc + static_cast<size_t>(my * 8 + Yc) * cw + mx * 8 + cbx) = word;
      if (cb & 1) S.saved_c[comp][(cb >> 1) * 4 + gy] = static_cast<uint8_t>(word >> 24);
    }
  }
  if (lane < 16) S.saved_y[lane] = S.tile[(lane + 1) * TS + 16];
  if (lane == 0) S.saved_x = my * g.wmb + mx;  // raster index: rows differ
  wave_sync();
}

__global__ __launch_bounds__(64 * kDecIntraWaves) void decode_intra_wavefront(DecodeArgs a) {
  __shared__ DecIntraShared SS[kDecIntraWaves];
  __shared__ int prog[kMaxRows];
  const Geom& g = a.g;
  const int slot = blockIdx.x;
  const int run = a.run[slot];
  if (run == 0) return;  // uniform per workgroup
  for (int i = threadIdx.x; i < g.hmb; i += blockDim.x) prog[i] = 0;
  const int w = wave_id();
  const int lane = lane_id();
  if (lane == 0) SS[w].saved_x = -2;
  __syncthreads();
  DecIntraShared& S = SS[w];
  for (int y = w; y < g.hmb; y += kDecIntraWaves) {
    if (run == 1) {  // I picture: every MB
      for (int x = 0; x < g.wmb; ++x) {
        if (y > 0) row_wait(prog, y - 1, min(x + 2, g.wmb), a.err);
        decode_intra_mb(a, S, slot, x, y);
        row_publish(prog, y, x + 1);
      }
      continue;
    }
    // P picture: visit only the intra MBs of the row (64 flags per ballot)
    const size_t rowo = static_cast<size_t>(slot) * g.nmb() + static_cast<size_t>(y) * g.wmb;
    for (int x0 = 0; x0 < g.wmb; x0 += 64) {
      const int xl = x0 + lane;
      unsigned long long m = __ballot(xl < g.wmb && h264::mbk_is_intra(a.hdr[rowo + xl].kind));
      while (m) {
        const int x = x0 + __builtin_ctzll(m);
        m &= m - 1;
        if (x > 0) row_publish(prog, y, x);
        if (y > 0) row_wait(prog, y - 1, min(x + 2, g.wmb), a.err);
        decode_intra_mb(a, S, slot, x, y);
        row_publish(prog, y, x + 1);
      }
    }
    row_publish(prog, y, g.wmb);
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

static DecodeArgs make_decode_args(int B, int wmb, int hmb, uint8_t* rec_y, uint8_t* rec_u, uint8_t* rec_v,
                                   const void* hdr, const uint32_t* mask, const uint32_t* off, const int16_t* coef,
                                   const int8_t* run, int chroma_qp_offset, uint8_t* nz, int* err) {
  DecodeArgs a;
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.rec_y = rec_y;
  a.rec_u = rec_u;
  a.rec_v = rec_v;
  a.hdr = static_cast<const MbHeader*>(hdr);
  a.mask = mask;
  a.off = off;
  a.coef = coef;
  a.run = run;
  a.chroma_qp_offset = chroma_qp_offset;
  a.nz = nz;
  a.err = err;
  a.dpb_n = 0;
  a.cur_idx = nullptr;
  a.reftab = nullptr;
  a.wp = nullptr;
  a.sub = nullptr;
  return a;
}

// One picture of every slot in the DPB layout: rec_* = [B][dpb_n] picture buffers; the
// decoded picture goes to buffer cur_idx[slot]; P and B macroblocks from reftab + the headers'
// motion (and the side pool `sub` for MBF_SUB4 macroblocks).
extern "C" void mivc_launch_decode_picture_dpb(int B, int wmb, int hmb, int dpb_n, uint8_t* dpb_y, uint8_t* dpb_u,
                                               uint8_t* dpb_v, const int16_t* cur_idx, const int16_t* reftab,
                                               const int16_t* wp, const int16_t* sub,
                                               const void* hdr, const uint32_t* mask, const uint32_t* off,
                                               const int16_t* coef, const int8_t* run, int any_inter,
                                               int chroma_qp_offset, uint8_t* nz, int* err, void* stream) {
  DecodeArgs a = make_decode_args(B, wmb, hmb, dpb_y, dpb_u, dpb_v, hdr, mask, off, coef, run,
                                  chroma_qp_offset, nz, err);
  a.dpb_n = dpb_n;
  a.cur_idx = cur_idx;
  a.reftab = reftab;
  a.wp = wp;
  a.sub = sub;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (any_inter) hipLaunchKernelGGL(decode_inter_dpb, dim3(wmb * hmb, B), dim3(64), 0, s, a);
  hipLaunchKernelGGL(decode_intra_wavefront, dim3(B), dim3(64 * kDecIntraWaves), 0, s, a);
}
