// Lookahead with the SATD Hadamard on the matrix cores (K-C6).
//
// The reference gets its frame-level rate control from libx264's lookahead inside
// the worker's ffmpeg (client.go:115, `-vcodec libx264` = CRF 23 by default,
// server.go:70).  Here every frame of every segment slot is analysed in ONE pass,
// before the encode: the lookahead has no reconstruction dependency, so B x F
// frames (15360 at the headline config) are independent work.
//
//   la_downscale  half-resolution luma ("lowres", 2x2 box) with a replicated border,
//                 so the search and the intra neighbours never clamp.
//   la_cost       per 8x8 lowres block (one per 16x16 macroblock):
//                   * inter: integer full search (2R+1)^2 against the previous lowres
//                     frame of the same segment, SAD (v_sad_u8) + 2 * |mv|;
//                   * intra: DC / horizontal / vertical predictions from the lowres
//                     neighbours;
//                   * cost of each of the 4 candidates = 8x8 Hadamard SATD of the
//                     residual, computed as ONE int8 GEMM on MFMA:
//                       D[64 x 16 blocks] = (H8 (x) H8)[64 x 64] . vec(S - P)[64 x 16]
//                     H8 (x) H8 is the Sylvester H64 (entries (-1)^popcount(i & k)),
//                     and S - P in [-255, 255] does not fit int8, so
//                       H.(S - P) = H.(S - 128) + (-H).(P - 128)
//                     (u8 ^ 0x80 is u8 - 128 as int8): the source half is computed
//                     once per block and is the accumulator input of every candidate.
//                     4 x mfma_i32_16x16x64_i8 per candidate per 16 blocks; the int32
//                     accumulation is exact.
//                 frame sums (intra, min(intra, inter)) -> [N, 2] u64, optional
//                 per-block costs for the numerics tests.
//
// Layout: one wave64 = a strip of 16 horizontally adjacent blocks.  Lane l owns block
// column c = l & 15 and rows 2g, 2g+1 (g = l >> 4) of it: exactly the B-operand
// fragment of mfma_i32_16x16x64_i8 (16 int8 of k = 16g + j, k = 8 * row + col), so
// the source and the predictions are loaded straight into MFMA operands.  The A
// operand (H64, 4 row tiles of 16) is generated in registers.  SADs of the search
// are summed over the four row groups of a column with two v_permlane{16,32}_swap.
#include "kcommon.h"

namespace mivc {
namespace gpu {

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int kLaPad = 16;  // replicated border of the lowres planes (bytes / rows)

struct LaGeom {
  int w, h;          // full-resolution display size of the input (even)
  long long fstride; // bytes between consecutive input luma frames
  int N, F;          // frames in total (slot-major), frames per segment
  int lbw, lbh;      // lowres 8x8 blocks per row / column
  int ls, lrows;     // lowres plane pitch and rows (with the border)
  long long lsize;   // bytes per lowres plane
};

__global__ void la_downscale(const uint8_t* __restrict__ y, LaGeom g, uint8_t* __restrict__ low) {
  const int qw = g.ls >> 2;  // dwords per lowres row
  const long long total = static_cast<long long>(g.N) * g.lrows * qw;
  const long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int n = static_cast<int>(i / (static_cast<long long>(g.lrows) * qw));
  const int rem = static_cast<int>(i - static_cast<long long>(n) * g.lrows * qw);
  const int py = rem / qw, px4 = (rem - py * qw) * 4;
  const int lw = g.w >> 1, lh = g.h >> 1;
  const int ly = clampi(py - kLaPad, 0, lh - 1);
  const uint8_t* r0 = y + n * g.fstride + static_cast<long long>(2 * ly) * g.w;
  const uint8_t* r1 = r0 + g.w;
  const int lx0 = px4 - kLaPad;
  uint32_t out = 0;
  if (lx0 >= 0 && lx0 + 4 <= lw && (g.w & 3) == 0 && (g.fstride & 3) == 0) {
    // interior: 8 source bytes per row, dword aligned (lx0 is a multiple of 4)
    const uint2 a = *reinterpret_cast<const uint2*>(r0 + 2 * lx0);
    const uint2 b = *reinterpret_cast<const uint2*>(r1 + 2 * lx0);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t wa = k < 2 ? a.x : a.y, wb = k < 2 ? b.x : b.y;
      const int sh = (k & 1) * 16;
      const uint32_t s = ((wa >> sh) & 255u) + ((wa >> (sh + 8)) & 255u) + ((wb >> sh) & 255u) +
                         ((wb >> (sh + 8)) & 255u);
      out |= ((s + 2u) >> 2) << (8 * k);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int lx = clampi(lx0 + k, 0, lw - 1);
      const uint32_t s = r0[2 * lx] + r0[2 * lx + 1] + r1[2 * lx] + r1[2 * lx + 1];
      out |= ((s + 2u) >> 2) << (8 * k);
    }
  }
  *reinterpret_cast<uint32_t*>(low + n * g.lsize + static_cast<long long>(py) * g.ls + px4) = out;
}

// v(l) + v(l ^ 16) + v(l ^ 32) + v(l ^ 48): the sum over the four row groups of a block column
__device__ __forceinline__ int sum_col_groups(int v) {
  auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  v = static_cast<int>(p[0]) + static_cast<int>(p[1]);
  auto q = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return static_cast<int>(q[0]) + static_cast<int>(q[1]);
}

// sum |D| of one candidate: D = accS + (-H) . (P - 128), 4 row tiles of 16
__device__ __forceinline__ int satd_mfma(const v4i (&negH)[4], const v4i (&accS)[4], v4i pf) {
  int s = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const v4i d = __builtin_amdgcn_mfma_i32_16x16x64_i8(negH[t], pf, accS[t], 0, 0, 0);
    s += abs(d[0]) + abs(d[1]) + abs(d[2]) + abs(d[3]);
  }
  return (sum_col_groups(s) + 2) >> 2;
}

__device__ __forceinline__ v4i as_s8(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  v4i r;
  r[0] = static_cast<int>(a ^ 0x80808080u);
  r[1] = static_cast<int>(b ^ 0x80808080u);
  r[2] = static_cast<int>(c ^ 0x80808080u);
  r[3] = static_cast<int>(d ^ 0x80808080u);
  return r;
}

struct LaArgs {
  LaGeom g;
  const uint8_t* low;
  unsigned long long* frame_cost;  // [N, 2]: sum intra, sum min(intra, inter)
  int* blk_cost;                   // optional [N, 2, lbh, lbw]: intra, inter (inter = intra on key frames)
  int* blk_mv;                     // optional [N, lbh, lbw]: lowres integer vector (dx & 0xFFFF) | (dy << 16)
  // hierarchical search (optional): [N, cbh, cbw] quarter-resolution vectors (la_cost on the
  // quarter planes); lowres block (bx, by) searches around twice the vector of its quarter
  // block (bx / 2, by / 2) instead of around zero, and keeps the zero vector as a candidate
  const int* center;
  int cbw, cbs;  // quarter blocks per row / per frame
  // lowres weighting (nullable): [N][kLaWtCols] (w, o) per reference distance d (column d);
  // w == 0: not weighted.  A weighted P candidate is priced with the source mapped through
  // the inverse weight, s' = (s - o) / w, and its SATD scaled back by w -- the lowres form of
  // the weighted prediction the encoder will use (x264 analyses weights in its lookahead too:
  // unweighted fades look like new content and break the P / B decisions and the CRF curve)
  const float2* wt;
};
constexpr int kLaWtCols = 8;

// inverse weight of 4 packed samples: clamp(round((s - o) / w), 0, 255)
__device__ __forceinline__ uint32_t la_inv_weight4(uint32_t s, float inv_w, float o) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float v = (static_cast<float>((s >> (8 * k)) & 255u) - o) * inv_w;
    const int q = clampi(static_cast<int>(rintf(v)), 0, 255);
    r |= static_cast<uint32_t>(q) << (8 * k);
  }
  return r;
}

// per-frame sums of the lowres interior (lw x lh): [N][2] = sum, sum of squares.  Grid
// (row groups, N): a block walks rows blockIdx.x, + gridDim.x, ...; a lane takes 4 samples
// per dword load (the interior starts kLaPad = 16 bytes into a row of a multiple of 8), sums
// and squares on the dot-product unit
__global__ __launch_bounds__(256) void la_stats(const uint8_t* __restrict__ low, LaGeom g,
                                                unsigned long long* __restrict__ st) {
  const int n = blockIdx.y;
  const int lw = g.w >> 1, lh = g.h >> 1;
  const int w4 = (lw + 3) >> 2, tail = lw & 3;
  const uint8_t* p = low + n * g.lsize + static_cast<long long>(kLaPad) * g.ls + kLaPad;
  uint32_t s = 0, s2 = 0;
  for (int y = blockIdx.x; y < lh; y += gridDim.x) {
    const uint32_t* row = reinterpret_cast<const uint32_t*>(p + static_cast<long long>(y) * g.ls);
    for (int x = threadIdx.x; x < w4; x += 256) {
      uint32_t v = row[x];
      if (tail && x == w4 - 1) v &= (1u << (8 * tail)) - 1u;  // samples past lw (the border copy)
      s = __builtin_amdgcn_udot4(v, 0x01010101u, s, false);
      s2 = __builtin_amdgcn_udot4(v, v, s2, false);
    }
  }
  unsigned long long s64 = s, q64 = s2;
  for (int off = 32; off > 0; off >>= 1) {
    s64 += __shfl_xor(s64, off, 64);
    q64 += __shfl_xor(q64, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(st + 2 * n, s64);
    atomicAdd(st + 2 * n + 1, q64);
  }
}

// weights of every (frame, distance) pair from the statistics: x264-style weightp rule --
// w = sqrt(var_cur / var_ref), o = mean_cur - w * mean_ref, used when the mean moved by >=
// thr_mean levels or the contrast by >= thr_scale
__global__ __launch_bounds__(256) void la_weights(const unsigned long long* __restrict__ st, LaGeom g, float thr_mean,
                                                  float thr_scale, float2* __restrict__ wt) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= g.N * kLaWtCols) return;
  const int n = i / kLaWtCols, d = i - n * kLaWtCols;
  const int f = n % g.F;
  float2 r = make_float2(0.f, 0.f);
  if (d >= 1 && d <= f) {
    const double cnt = static_cast<double>(g.w >> 1) * static_cast<double>(g.h >> 1);
    const double mc = static_cast<double>(st[2 * n]) / cnt, mr = static_cast<double>(st[2 * (n - d)]) / cnt;
    const double vc = fmax(static_cast<double>(st[2 * n + 1]) / cnt - mc * mc, 0.0);
    const double vr = fmax(static_cast<double>(st[2 * (n - d) + 1]) / cnt - mr * mr, 0.0);
    const double w = vr > 1e-3 ? sqrt(vc / vr) : 1.0;
    if ((fabs(mc - mr) >= thr_mean || fabs(w - 1.0) >= thr_scale) && w > 1.0 / 64)
      r = make_float2(static_cast<float>(w), static_cast<float>(mc - w * mr));
  }
  wt[i] = r;
}

// Quarter-resolution planes from the lowres ones (2x2 box of the lowres interior, replicated
// border): the coarse level of the hierarchical lookahead search.  q: the quarter geometry
// (q.w x q.h = the lowres size).
__global__ void la_downscale_low(const uint8_t* __restrict__ low, LaGeom g, LaGeom q, uint8_t* __restrict__ low4) {
  const long long total = static_cast<long long>(q.N) * q.lsize;
  const long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int n = static_cast<int>(i / q.lsize);
  const int rem = static_cast<int>(i - static_cast<long long>(n) * q.lsize);
  const int py = rem / q.ls, px = rem - py * q.ls;
  const int qw = q.w >> 1, qh = q.h >> 1;
  const int ly = clampi(py - kLaPad, 0, qh - 1), lx = clampi(px - kLaPad, 0, qw - 1);
  const uint8_t* sp = low + n * g.lsize + static_cast<long long>(kLaPad + 2 * ly) * g.ls + kLaPad + 2 * lx;
  low4[i] = static_cast<uint8_t>((sp[0] + sp[1] + sp[g.ls] + sp[g.ls + 1] + 2) >> 2);
}

// 8 lowres bytes of rows (y, y + 1) at column x (any alignment) as MFMA B-operand bytes
__device__ __forceinline__ v4i la_rows8(const uint8_t* plane, long long ls, int x, int y) {
  const int xa = x & ~3, sh = x & 3;
  const uint32_t* q0 = reinterpret_cast<const uint32_t*>(plane + static_cast<long long>(y) * ls + xa);
  const uint32_t* q1 = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(q0) + ls);
  const uint32_t e0 = q0[0], e1 = q0[1], e2 = q0[2], f0 = q1[0], f1 = q1[1], f2 = q1[2];
  return as_s8(__builtin_amdgcn_alignbyte(e1, e0, sh), __builtin_amdgcn_alignbyte(e2, e1, sh),
               __builtin_amdgcn_alignbyte(f1, f0, sh), __builtin_amdgcn_alignbyte(f2, f1, sh));
}

// raw 8 bytes of rows (y, y + 1) at column x (the four dwords of la_rows8 before the bias)
__device__ __forceinline__ uint4 la_raw8(const uint8_t* plane, long long ls, int x, int y) {
  const int xa = x & ~3, sh = x & 3;
  const uint32_t* q0 = reinterpret_cast<const uint32_t*>(plane + static_cast<long long>(y) * ls + xa);
  const uint32_t* q1 = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(q0) + ls);
  const uint32_t e0 = q0[0], e1 = q0[1], e2 = q0[2], f0 = q1[0], f1 = q1[1], f2 = q1[2];
  return make_uint4(__builtin_amdgcn_alignbyte(e1, e0, sh), __builtin_amdgcn_alignbyte(e2, e1, sh),
                    __builtin_amdgcn_alignbyte(f1, f0, sh), __builtin_amdgcn_alignbyte(f2, f1, sh));
}

// (2R+1)^2 integer search around (cx, cy) (clamped so the window stays inside the padded
// plane); returns the best offset (SAD + 2 |offset from the centre|), the lane holding its
// two rows of the block's column
template <int R>
__device__ __forceinline__ void la_small_search(const uint8_t* ref, const LaGeom& g, int X0, int ry, uint2 s0, uint2 s1,
                                                int cx, int cy, int& bx, int& by) {
  constexpr int side = 2 * R + 1;
  // the window's 7 aligned dwords per row (from x0 & ~3) and its rows stay inside the plane
  const int Yb = ry & ~7;  // the block's top row
  cx = clampi(cx, R - X0, g.ls - 28 - X0 + R);
  cy = clampi(cy, R - Yb, g.lrows - 8 - R - Yb);
  const int x0 = X0 + cx - R;
  const int xa = x0 & ~3, s = x0 & 3;
  int best = 0x7FFFFFFF;
  for (int dy = -R; dy <= R; ++dy) {
    const uint32_t* p0 = reinterpret_cast<const uint32_t*>(ref + static_cast<long long>(ry + cy + dy) * g.ls + xa);
    const uint32_t* p1 = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(p0) + g.ls);
    uint32_t w0[6], w1[6];
    {
      uint32_t t0[7], t1[7];
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        t0[k] = p0[k];
        t1[k] = p1[k];
      }
#pragma unroll
      for (int k = 0; k < 6; ++k) {  // realign: w starts at column x0
        w0[k] = __builtin_amdgcn_alignbyte(t0[k + 1], t0[k], s);
        w1[k] = __builtin_amdgcn_alignbyte(t1[k + 1], t1[k], s);
      }
    }
#pragma unroll
    for (int dx = -R; dx <= R; ++dx) {
      const int o = R + dx, wi = o >> 2, sh = o & 3;
      const uint32_t a0 = __builtin_amdgcn_alignbyte(w0[wi + 1], w0[wi], sh);
      const uint32_t a1 = __builtin_amdgcn_alignbyte(w0[wi + 2], w0[wi + 1], sh);
      const uint32_t b0 = __builtin_amdgcn_alignbyte(w1[wi + 1], w1[wi], sh);
      const uint32_t b1 = __builtin_amdgcn_alignbyte(w1[wi + 2], w1[wi + 1], sh);
      uint32_t sad = sad4(s0.x, a0, 0);
      sad = sad4(s0.y, a1, sad);
      sad = sad4(s1.x, b0, sad);
      sad = sad4(s1.y, b1, sad);
      const int cost = sum_col_groups(static_cast<int>(sad)) + 2 * (abs(dx) + abs(dy));
      best = min(best, (cost << 9) | ((dy + R) * side + (dx + R)));
    }
  }
  const int bi = best & 511;
  bx = cx + bi % side - R;
  by = cy + bi / side - R;
}

// WT: the instance with lowres weighting (a.wt non-null): its extra registers stay out of the
// plain instance
template <int R, bool WT = false>
__global__ __launch_bounds__(256) void la_cost(LaArgs a) {
  const LaGeom& g = a.g;
  constexpr int side = 2 * R + 1;
  const int nstrips = (g.lbw + 15) >> 4;
  const int per_frame = nstrips * g.lbh;
  const long long waves = static_cast<long long>(per_frame) * g.N;
  const int nwg = static_cast<int>((waves + 3) >> 2);
  int lin = blockIdx.x;
  if ((nwg & 7) == 0) lin = (lin & 7) * (nwg >> 3) + (lin >> 3);  // each XCD walks a contiguous range
  const long long wv = static_cast<long long>(lin) * 4 + wave_id();
  if (wv >= waves) return;  // wave-uniform
  const int n = static_cast<int>(wv / per_frame);
  const int rem = static_cast<int>(wv - static_cast<long long>(n) * per_frame);
  const int by = rem / nstrips, strip = rem - by * nstrips;
  const int lane = lane_id(), c = lane & 15, grp = lane >> 4;
  const int bx = strip * 16 + c;
  const bool valid = bx < g.lbw;
  const int bxc = valid ? bx : g.lbw - 1;  // idle columns read a valid block
  const int f = n % g.F;
  const bool has_ref = f > 0;

  // H64 row tiles as int8 A operands (and their negation): row i = 16t + (l & 15), k = 16 grp + j
  v4i H[4], negH[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t wp = 0, wn = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int i = 16 * t + c, k = 16 * grp + 4 * q + b;
        const bool neg = __builtin_popcount(i & k) & 1;
        wp |= (neg ? 0xFFu : 0x01u) << (8 * b);
        wn |= (neg ? 0x01u : 0xFFu) << (8 * b);
      }
      H[t][q] = static_cast<int>(wp);
      negH[t][q] = static_cast<int>(wn);
    }
  }

  const uint8_t* cur = a.low + n * g.lsize;
  const int X0 = kLaPad + bxc * 8, Y0 = kLaPad + by * 8;
  const int ry = Y0 + 2 * grp;  // this lane's two rows
  const uint8_t* c0 = cur + static_cast<long long>(ry) * g.ls + X0;
  uint2 s0 = *reinterpret_cast<const uint2*>(c0);
  uint2 s1 = *reinterpret_cast<const uint2*>(c0 + g.ls);
  // intra neighbours: the row above (8 bytes) and this lane's two left samples
  const uint2 top = *reinterpret_cast<const uint2*>(cur + static_cast<long long>(Y0 - 1) * g.ls + X0);
  const uint32_t l0 = c0[-1], l1 = c0[g.ls - 1];

  // source half of every candidate's Hadamard: H . (S - 128)
  const v4i sf = as_s8(s0.x, s0.y, s1.x, s1.y);
  v4i accS[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) accS[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(H[t], sf, v4i{0, 0, 0, 0}, 0, 0, 0);

  // ---- intra: DC, H, V
  auto bsum = [](uint32_t w) { return (w & 255u) + ((w >> 8) & 255u) + ((w >> 16) & 255u) + (w >> 24); };
  const int tsum = static_cast<int>(bsum(top.x) + bsum(top.y));
  const int lsum = sum_col_groups(static_cast<int>(l0 + l1));
  const uint32_t dc = static_cast<uint32_t>((tsum + lsum + 8) >> 4) * 0x01010101u;
  const uint32_t h0 = l0 * 0x01010101u, h1 = l1 * 0x01010101u;
  int intra = satd_mfma(negH, accS, as_s8(dc, dc, dc, dc));
  intra = min(intra, satd_mfma(negH, accS, as_s8(h0, h0, h1, h1)));
  intra = min(intra, satd_mfma(negH, accS, as_s8(top.x, top.y, top.x, top.y)));
  intra += 5;  // mode-cost bias

  // weighted reference (lowres weighting): the source through the inverse weight, its
  // Hadamard half recomputed (intra is done with the plain source)
  float wsc = 0.f;
  if (WT && has_ref && a.wt) {
    const float2 wo = a.wt[static_cast<long long>(n) * kLaWtCols + 1];
    if (wo.x > 0.f) {  // frame-uniform
      const float inv = 1.0f / wo.x;
      s0 = make_uint2(la_inv_weight4(s0.x, inv, wo.y), la_inv_weight4(s0.y, inv, wo.y));
      s1 = make_uint2(la_inv_weight4(s1.x, inv, wo.y), la_inv_weight4(s1.y, inv, wo.y));
      const v4i sw = as_s8(s0.x, s0.y, s1.x, s1.y);
#pragma unroll
      for (int t = 0; t < 4; ++t) accS[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(H[t], sw, v4i{0, 0, 0, 0}, 0, 0, 0);
      wsc = wo.x;
    }
  }
  // SATD of a weighted candidate in the source's units
  auto wsatd = [&](int v) { return WT && wsc > 0.f ? static_cast<int>(rintf(wsc * static_cast<float>(v))) : v; };

  int inter = intra;
  int mvx = 0, mvy = 0;
  if (has_ref && a.center) {  // frame-uniform: hierarchical search around the coarse vector
    const uint8_t* ref = cur - g.lsize;
    const int cv = a.center[static_cast<long long>(n) * a.cbs + (by >> 1) * a.cbw + (bxc >> 1)];
    const int cx = 2 * static_cast<int16_t>(cv & 0xFFFF), cy = 2 * (cv >> 16);
    int mx, my;
    la_small_search<R>(ref, g, X0, ry, s0, s1, cx, cy, mx, my);
    const int cst = wsatd(satd_mfma(negH, accS, la_rows8(ref, g.ls, X0 + mx, ry + my))) + 2 * (abs(mx) + abs(my));
    const int c0 = wsatd(satd_mfma(negH, accS, la_rows8(ref, g.ls, X0, ry)));
    inter = min(cst, c0);
    mvx = cst < c0 ? mx : 0;
    mvy = cst < c0 ? my : 0;
  } else if (has_ref) {  // frame-uniform
    const uint8_t* ref = cur - g.lsize;
    // ---- integer full search: lane accumulates the SAD of its two rows, then the column sum
    int best = 0x7FFFFFFF;
    for (int dy = -R; dy <= R; ++dy) {
      uint32_t w0[7], w1[7];
      const uint32_t* p0 = reinterpret_cast<const uint32_t*>(ref + static_cast<long long>(ry + dy) * g.ls + X0 - 8);
      const uint32_t* p1 = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(p0) + g.ls);
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        w0[k] = p0[k];
        w1[k] = p1[k];
      }
#pragma unroll
      for (int dx = -R; dx <= R; ++dx) {
        const int o = 8 + dx, wi = o >> 2, sh = o & 3;
        const uint32_t a0 = __builtin_amdgcn_alignbyte(w0[wi + 1], w0[wi], sh);
        const uint32_t a1 = __builtin_amdgcn_alignbyte(w0[wi + 2], w0[wi + 1], sh);
        const uint32_t b0 = __builtin_amdgcn_alignbyte(w1[wi + 1], w1[wi], sh);
        const uint32_t b1 = __builtin_amdgcn_alignbyte(w1[wi + 2], w1[wi + 1], sh);
        uint32_t sad = sad4(s0.x, a0, 0);
        sad = sad4(s0.y, a1, sad);
        sad = sad4(s1.x, b0, sad);
        sad = sad4(s1.y, b1, sad);
        const int cost = sum_col_groups(static_cast<int>(sad)) + 2 * (abs(dx) + abs(dy));
        const int key = (cost << 9) | ((dy + R) * side + (dx + R));
        best = min(best, key);
      }
    }
    const int bi = best & 511;
    const int mdy = bi / side - R, mdx = bi % side - R;
    // best prediction rows (unaligned 8 bytes: three aligned dwords + alignbyte)
    const int xo = X0 + mdx;
    const int xa = xo & ~3, shb = xo & 3;
    const uint32_t* q0 = reinterpret_cast<const uint32_t*>(ref + static_cast<long long>(ry + mdy) * g.ls + xa);
    const uint32_t* q1 = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(q0) + g.ls);
    const uint32_t e0 = q0[0], e1 = q0[1], e2 = q0[2], f0 = q1[0], f1 = q1[1], f2 = q1[2];
    const v4i pf = as_s8(__builtin_amdgcn_alignbyte(e1, e0, shb), __builtin_amdgcn_alignbyte(e2, e1, shb),
                         __builtin_amdgcn_alignbyte(f1, f0, shb), __builtin_amdgcn_alignbyte(f2, f1, shb));
    inter = wsatd(satd_mfma(negH, accS, pf)) + 2 * (abs(mdx) + abs(mdy));
    mvx = mdx;
    mvy = mdy;
  }
  const int pcost = min(intra, inter);
  if (a.blk_cost && grp == 0 && valid) {
    const long long base = static_cast<long long>(n) * 2 * g.lbh * g.lbw + static_cast<long long>(by) * g.lbw + bx;
    a.blk_cost[base] = intra;
    a.blk_cost[base + static_cast<long long>(g.lbh) * g.lbw] = inter;
  }
  if (a.blk_mv && grp == 0 && valid)
    a.blk_mv[static_cast<long long>(n) * g.lbh * g.lbw + static_cast<long long>(by) * g.lbw + bx] =
        (mvx & 0xFFFF) | (mvy << 16);
  const bool mine = grp == 0 && valid;
  const int si = sum64(mine ? intra : 0), sp = sum64(mine ? pcost : 0);
  if (lane == 0) {
    atomicAdd(a.frame_cost + 2 * n, static_cast<unsigned long long>(si));
    atomicAdd(a.frame_cost + 2 * n + 1, static_cast<unsigned long long>(sp));
  }
}

// ---------------------------------------------------------------- b-adapt costs (x264 --b-adapt 1)
// x264's fast B-frame placement compares, per run of pictures, the lowres cost of coding a
// picture as P from anchors 2..bframes+1 pictures back and as B between its two neighbours.
// la_multi prices exactly those for every frame of every slot in one launch, reusing
// la_cost's lowres planes, its per-block intra costs and distance-1 vectors:
//   * P at distance d = 2..D: a (2R+1)^2 integer search centred on d times the block's
//     distance-1 vector (constant motion), SATD of the best prediction on MFMA;
//   * B between f - 1 and f + 1: list 0 = the distance-1 prediction, list 1 = a search of
//     f + 1 centred on the reversed vector, bi = their rounded average; the block takes the
//     cheapest of intra, L0, L1, bi.
// Frame sums of min(intra, candidate) go to out[n][d] (d = 2..D) and out[n][0] (B), each
// plus (number of blocks that chose intra) << kLaIntraShift: x264's b-adapt guards force P
// pictures when a P candidate is mostly intra (rc/badapt.py).
constexpr int kLaMultiCols = 8;
constexpr int kLaIntraShift = 40;  // frame cost sums stay far below 2^40

struct LaMultiArgs {
  LaGeom g;
  const uint8_t* low;
  const int* blk_cost;  // [N, 2, lbh, lbw] (la_cost): intra, inter at distance 1
  const int* blk_mv;    // [N, lbh, lbw] (la_cost): distance-1 lowres vectors
  int D;                // largest P distance (bframes + 1), <= kLaMultiCols - 1
  unsigned long long* out;  // [N, kLaMultiCols]
  const float2* wt;         // lowres weighting (LaArgs::wt), nullable
};

template <int R, bool WT = false>
__global__ __launch_bounds__(256) void la_multi(LaMultiArgs a) {
  const LaGeom& g = a.g;
  const int nstrips = (g.lbw + 15) >> 4;
  const int per_frame = nstrips * g.lbh;
  const long long waves = static_cast<long long>(per_frame) * g.N;
  const int nwg = static_cast<int>((waves + 3) >> 2);
  int lin = blockIdx.x;
  if ((nwg & 7) == 0) lin = (lin & 7) * (nwg >> 3) + (lin >> 3);
  const long long wv = static_cast<long long>(lin) * 4 + wave_id();
  if (wv >= waves) return;  // wave-uniform
  const int n = static_cast<int>(wv / per_frame);
  const int rem = static_cast<int>(wv - static_cast<long long>(n) * per_frame);
  const int by = rem / nstrips, strip = rem - by * nstrips;
  const int lane = lane_id(), c = lane & 15, grp = lane >> 4;
  const int bx = strip * 16 + c;
  const bool valid = bx < g.lbw;
  const int bxc = valid ? bx : g.lbw - 1;
  const int f = n % g.F;
  if (f == 0) return;  // the IDR picture: neither P nor B candidates (frame-uniform)
  v4i H[4], negH[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t wp = 0, wn = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int i = 16 * t + c, k = 16 * grp + 4 * q + b;
        const bool neg = __builtin_popcount(i & k) & 1;
        wp |= (neg ? 0xFFu : 0x01u) << (8 * b);
        wn |= (neg ? 0x01u : 0xFFu) << (8 * b);
      }
      H[t][q] = static_cast<int>(wp);
      negH[t][q] = static_cast<int>(wn);
    }
  }
  const uint8_t* cur = a.low + n * g.lsize;
  const int X0 = kLaPad + bxc * 8, Y0 = kLaPad + by * 8;
  const int ry = Y0 + 2 * grp;
  const uint8_t* c0 = cur + static_cast<long long>(ry) * g.ls + X0;
  const uint2 s0 = *reinterpret_cast<const uint2*>(c0);
  const uint2 s1 = *reinterpret_cast<const uint2*>(c0 + g.ls);
  const v4i sf = as_s8(s0.x, s0.y, s1.x, s1.y);
  v4i accS[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) accS[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(H[t], sf, v4i{0, 0, 0, 0}, 0, 0, 0);
  const long long bo = static_cast<long long>(by) * g.lbw + bxc;
  const long long plane_b = static_cast<long long>(g.lbh) * g.lbw;
  const int intra = a.blk_cost[static_cast<long long>(n) * 2 * plane_b + bo];
  const int inter1 = a.blk_cost[static_cast<long long>(n) * 2 * plane_b + plane_b + bo];
  const int mv1 = a.blk_mv[static_cast<long long>(n) * plane_b + bo];
  const int v1x = static_cast<int16_t>(mv1 & 0xFFFF), v1y = mv1 >> 16;
  const bool mine = grp == 0 && valid;
  // P at distances 2..D
  for (int d = 2; d <= a.D && d <= f; ++d) {  // frame-uniform
    const uint8_t* ref = cur - d * g.lsize;
    const float2 wo = WT ? a.wt[static_cast<long long>(n) * kLaWtCols + d] : make_float2(0.f, 0.f);
    uint2 w0 = s0, w1 = s1;
    v4i accW[4] = {accS[0], accS[1], accS[2], accS[3]};
    if (wo.x > 0.f) {  // frame-uniform: weighted reference at this distance
      const float inv = 1.0f / wo.x;
      w0 = make_uint2(la_inv_weight4(s0.x, inv, wo.y), la_inv_weight4(s0.y, inv, wo.y));
      w1 = make_uint2(la_inv_weight4(s1.x, inv, wo.y), la_inv_weight4(s1.y, inv, wo.y));
      const v4i sw = as_s8(w0.x, w0.y, w1.x, w1.y);
#pragma unroll
      for (int t = 0; t < 4; ++t) accW[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(H[t], sw, v4i{0, 0, 0, 0}, 0, 0, 0);
    }
    int mx, my;
    la_small_search<R>(ref, g, X0, ry, w0, w1, d * v1x, d * v1y, mx, my);
    const int sraw = satd_mfma(negH, accW, la_rows8(ref, g.ls, X0 + mx, ry + my));
    const int cst = (wo.x > 0.f ? static_cast<int>(rintf(wo.x * static_cast<float>(sraw))) : sraw) +
                    2 * (abs(mx - d * v1x) + abs(my - d * v1y)) + 2 * (abs(v1x) + abs(v1y));
    const int s = sum64(mine ? min(intra, cst) : 0);
    const int ni = sum64(mine && intra < cst ? 1 : 0);
    if (lane == 0)
      atomicAdd(a.out + static_cast<long long>(n) * kLaMultiCols + d,
                static_cast<unsigned long long>(s) + (static_cast<unsigned long long>(ni) << kLaIntraShift));
  }
  // B between f - 1 and f + 1
  if (f + 1 < g.F) {  // frame-uniform
    const uint8_t* r0 = cur - g.lsize;
    const uint8_t* r1 = cur + g.lsize;
    int mx, my;
    la_small_search<R>(r1, g, X0, ry, s0, s1, -v1x, -v1y, mx, my);
    const int c1 = satd_mfma(negH, accS, la_rows8(r1, g.ls, X0 + mx, ry + my)) + 2 * (abs(mx) + abs(my));
    const int cx0 = clampi(v1x, -8, 8), cy0 = clampi(v1y, -8, 8);  // la_cost's range: |v1| <= 8
    const uint4 p0 = la_raw8(r0, g.ls, X0 + cx0, ry + cy0);
    const uint4 p1 = la_raw8(r1, g.ls, X0 + mx, ry + my);
    auto avg = [](uint32_t x, uint32_t y) { return (x | y) - (((x ^ y) >> 1) & 0x7F7F7F7Fu); };
    const int cbi = satd_mfma(negH, accS, as_s8(avg(p0.x, p1.x), avg(p0.y, p1.y), avg(p0.z, p1.z), avg(p0.w, p1.w))) +
                    2 * (abs(mx) + abs(my) + abs(v1x) + abs(v1y));
    const int bc = min(min(intra, inter1), min(c1, cbi));
    const int s = sum64(mine ? bc : 0);
    const int ni = sum64(mine && intra < min(inter1, min(c1, cbi)) ? 1 : 0);
    if (lane == 0)
      atomicAdd(a.out + static_cast<long long>(n) * kLaMultiCols,
                static_cast<unsigned long long>(s) + (static_cast<unsigned long long>(ni) << kLaIntraShift));
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

// Bytes of the lowres workspace for N frames of w x h.
extern "C" long long mivc_lookahead_low_bytes(int w, int h, int N) {
  const int lbw = ((w >> 1) + 7) >> 3, lbh = ((h >> 1) + 7) >> 3;
  return static_cast<long long>(N) * (lbw * 8 + 2 * kLaPad) * (lbh * 8 + 2 * kLaPad);
}

// y: luma of N = B*F frames (slot-major), frame f of slot b at y + (b*F + f) * fstride.
// low: workspace of mivc_lookahead_low_bytes(); frame_cost: [N, 2] u64 (zeroed here);
// blk_cost: optional [N, 2, lbh, lbw] int32.
// Hierarchical (low4 / mv4 / cost4 non-null): quarter-resolution planes of the lowres ones,
// an integer full search +-8 there (= +-32 full-resolution pixels) into mv4, and the lowres
// search centred on twice those vectors.  low4: mivc_lookahead_quarter_bytes(); mv4:
// [N, cbh, cbw] int32 with cbw x cbh the quarter 8x8 blocks; cost4: [N, 2] u64 scratch.
extern "C" long long mivc_lookahead_quarter_bytes(int w, int h, int N) {
  const int qw = (w >> 1) & ~1, qh = (h >> 1) & ~1;
  const int qbw = ((qw >> 1) + 7) >> 3, qbh = ((qh >> 1) + 7) >> 3;
  return static_cast<long long>(N) * (qbw * 8 + 2 * kLaPad) * (qbh * 8 + 2 * kLaPad);
}

extern "C" int mivc_launch_lookahead(const uint8_t* y, int w, int h, long long fstride, int N, int F, uint8_t* low,
                                     unsigned long long* frame_cost, int* blk_cost, int* blk_mv, int range,
                                     void* stream, uint8_t* low4, int* mv4, unsigned long long* cost4, float* wt,
                                     unsigned long long* wstats, float thr_mean, float thr_scale, int stage) {
  // stage bit 0: lowres planes (+ the weights when wt and wstats are given); bit 1: the costs
  // (the weighted instances when wt is given).  The caller may look at the weights between
  // the two and run the plain instances when no picture is weighted.
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (w < 16 || h < 16 || (w & 1) || (h & 1) || N <= 0 || F <= 0 || N % F) return -1;
  if (range != 4 && range != 6 && range != 8) return -2;
  LaGeom g{};
  g.w = w;
  g.h = h;
  g.fstride = fstride;
  g.N = N;
  g.F = F;
  g.lbw = ((w >> 1) + 7) >> 3;
  g.lbh = ((h >> 1) + 7) >> 3;
  g.ls = g.lbw * 8 + 2 * kLaPad;
  g.lrows = g.lbh * 8 + 2 * kLaPad;
  g.lsize = static_cast<long long>(g.ls) * g.lrows;
  LaArgs a{g, low, frame_cost, blk_cost, blk_mv, nullptr, 0, 0, reinterpret_cast<const float2*>(wt)};
  if (stage & 1) {
    const long long dwords = static_cast<long long>(N) * g.lrows * (g.ls >> 2);
    hipLaunchKernelGGL(la_downscale, dim3(static_cast<unsigned>((dwords + 255) / 256)), dim3(256), 0, s, y, g, low);
    if (wt && wstats) {  // lowres weighting: statistics of the lowres planes, then the weights
      hipMemsetAsync(wstats, 0, sizeof(unsigned long long) * 2 * N, s);
      hipLaunchKernelGGL(la_stats, dim3(8, N), dim3(256), 0, s, low, g, wstats);  // 8 row groups per picture
      hipLaunchKernelGGL(la_weights, dim3((N * kLaWtCols + 255) / 256), dim3(256), 0, s, wstats, g, thr_mean, thr_scale,
                         reinterpret_cast<float2*>(wt));
    }
  }
  if (!(stage & 2)) return 0;
  hipMemsetAsync(frame_cost, 0, sizeof(unsigned long long) * 2 * N, s);
  if (low4 && mv4 && cost4 && w >= 64 && h >= 64) {
    LaGeom q{};
    q.w = (w >> 1) & ~1;
    q.h = (h >> 1) & ~1;
    q.fstride = 0;
    q.N = N;
    q.F = F;
    q.lbw = ((q.w >> 1) + 7) >> 3;
    q.lbh = ((q.h >> 1) + 7) >> 3;
    q.ls = q.lbw * 8 + 2 * kLaPad;
    q.lrows = q.lbh * 8 + 2 * kLaPad;
    q.lsize = static_cast<long long>(q.ls) * q.lrows;
    const long long qbytes = static_cast<long long>(N) * q.lsize;
    hipLaunchKernelGGL(la_downscale_low, dim3(static_cast<unsigned>((qbytes + 255) / 256)), dim3(256), 0, s, low, g, q,
                       low4);
    hipMemsetAsync(cost4, 0, sizeof(unsigned long long) * 2 * N, s);
    LaArgs aq{q, low4, cost4, nullptr, mv4, nullptr, 0, 0, nullptr};
    const long long qwaves = static_cast<long long>((q.lbw + 15) >> 4) * q.lbh * N;
    hipLaunchKernelGGL(la_cost<8>, dim3(static_cast<unsigned>((qwaves + 3) >> 2)), dim3(256), 0, s, aq);
    a.center = mv4;
    a.cbw = q.lbw;
    a.cbs = q.lbw * q.lbh;
  }
  const long long waves = static_cast<long long>((g.lbw + 15) >> 4) * g.lbh * N;
  const dim3 grid(static_cast<unsigned>((waves + 3) >> 2));
  if (a.wt) {
    switch (range) {
      case 4: hipLaunchKernelGGL((la_cost<4, true>), grid, dim3(256), 0, s, a); break;
      case 6: hipLaunchKernelGGL((la_cost<6, true>), grid, dim3(256), 0, s, a); break;
      default: hipLaunchKernelGGL((la_cost<8, true>), grid, dim3(256), 0, s, a); break;
    }
  } else {
    switch (range) {
      case 4: hipLaunchKernelGGL(la_cost<4>, grid, dim3(256), 0, s, a); break;
      case 6: hipLaunchKernelGGL(la_cost<6>, grid, dim3(256), 0, s, a); break;
      default: hipLaunchKernelGGL(la_cost<8>, grid, dim3(256), 0, s, a); break;
    }
  }
  return 0;
}

// b-adapt costs of N = B*F frames (la_multi): needs the lowres planes, block costs and vectors
// of a preceding mivc_launch_lookahead on the same workspace.  out: [N, 8] u64 (zeroed here):
// column d = 2..D the P cost at distance d, column 0 the B cost between the neighbours; bits
// 40.. of each the number of lowres blocks that chose intra.
extern "C" int mivc_launch_lookahead_multi(const uint8_t* low, int w, int h, int N, int F, const int* blk_cost,
                                           const int* blk_mv, int D, int range, unsigned long long* out,
                                           void* stream, const float* wt) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (w < 16 || h < 16 || (w & 1) || (h & 1) || N <= 0 || F <= 0 || N % F) return -1;
  if (D < 2 || D >= kLaMultiCols || !blk_cost || !blk_mv || !low || !out) return -2;
  LaGeom g{};
  g.w = w;
  g.h = h;
  g.N = N;
  g.F = F;
  g.lbw = ((w >> 1) + 7) >> 3;
  g.lbh = ((h >> 1) + 7) >> 3;
  g.ls = g.lbw * 8 + 2 * kLaPad;
  g.lrows = g.lbh * 8 + 2 * kLaPad;
  g.lsize = static_cast<long long>(g.ls) * g.lrows;
  hipMemsetAsync(out, 0, sizeof(unsigned long long) * kLaMultiCols * N, s);
  LaMultiArgs a{g, low, blk_cost, blk_mv, D, out, reinterpret_cast<const float2*>(wt)};
  const long long waves = static_cast<long long>((g.lbw + 15) >> 4) * g.lbh * N;
  const dim3 grid(static_cast<unsigned>((waves + 3) >> 2));
  if (a.wt) {
    if (range <= 1) hipLaunchKernelGGL((la_multi<1, true>), grid, dim3(256), 0, s, a);
    else if (range <= 2) hipLaunchKernelGGL((la_multi<2, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((la_multi<4, true>), grid, dim3(256), 0, s, a);
  } else {
    if (range <= 1) hipLaunchKernelGGL(la_multi<1>, grid, dim3(256), 0, s, a);
    else if (range <= 2) hipLaunchKernelGGL(la_multi<2>, grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL(la_multi<4>, grid, dim3(256), 0, s, a);
  }
  return 0;
}
