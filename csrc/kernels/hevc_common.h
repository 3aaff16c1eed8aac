// Device helpers of the HEVC kernels (gfx950): wave-level integer transforms through
// LDS, intra reference-sample construction (8.4.4.2.2 availability + substitution,
// 8.4.4.2.3 filtering) and intra sample prediction (8.4.4.2.4 - 8.4.4.2.6).
//
// Samples are uint16 for 8- and 10-bit content (one code path; the bit depth is a
// runtime parameter).  A transform of an n x n block (n = 4..32) is two matrix
// products done by one wave64: lane (ti, tj) owns a T x T output tile (T = n / 8,
// 8 x 8 tiles), the DCT matrix lives in LDS as int16.
#pragma once
#include "kcommon.h"
#include "../common/hevc_tables.h"

namespace mivc {
namespace gpu {

// intra analysis candidates per CTB (int32): [0, 21) best cost per CU (32, 4 x 16, 16 x 8 in
// z-order), [21, 42) its mode, [42, 58) per 8x8 CU the chosen PART_NxN PU modes (bit 24 set,
// four 6-bit modes) or 0 (PART_2Nx2N)
constexpr int kCandStride = 58;

// z-order index of 4x4 block (gx, gy) inside a 32x32 CTB (0..63)
__device__ __forceinline__ int zorder4(int gx, int gy) {
  return (gx & 1) | ((gy & 1) << 1) | ((gx & 2) << 1) | ((gy & 2) << 2) | ((gx & 4) << 2) | ((gy & 4) << 3);
}

// CuInfo of an intra PART_NxN 8x8 CU from a packed candidate (bit 24 | four 6-bit modes):
// flags bit 3, PU 0's mode in `mode`, the four PU modes in the bytes of the unused vector
__device__ __forceinline__ void set_nxn(hevc::CuInfo& c, int packed) {
  c.flags |= 8;
  c.mode = static_cast<uint8_t>(packed & 63);
  uint8_t* b = reinterpret_cast<uint8_t*>(c.mv);
  for (int j = 0; j < 4; ++j) b[j] = static_cast<uint8_t>((packed >> (6 * j)) & 63);
}

// batched HEVC picture geometry (coded size, multiple of the 32x32 CTB)
struct HevcGeom {
  int B, W, H, wctb, hctb;
  __host__ __device__ size_t ysize() const { return static_cast<size_t>(W) * H; }
  __host__ __device__ size_t csize() const { return static_cast<size_t>(W / 2) * (H / 2); }
  __host__ __device__ int nctb() const { return wctb * hctb; }
};

namespace hv {

using hevc::dct_coef;

// ---------------------------------------------------------------- DCT matrix in LDS
struct DctLds {
  int16_t m[32][32];
  int16_t dst[4][4];  // DST-VII (8.6.4.2, trType 1: 4x4 intra luma)
};
__device__ __forceinline__ void dct_lds_init(DctLds& D) {
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) D.m[i >> 5][i & 31] = static_cast<int16_t>(dct_coef(i >> 5, i & 31));
  if (threadIdx.x < 16) {
    const int16_t t[16] = {29, 55, 74, 84, 74, 74, 0, -74, 84, -29, -74, 55, 55, -84, 74, -29};
    D.dst[threadIdx.x >> 2][threadIdx.x & 3] = t[threadIdx.x];
  }
}
// entry (k, m) of the n-point matrix
__device__ __forceinline__ int cn(const DctLds& D, int log2n, int k, int m) { return D.m[k << (5 - log2n)][m]; }

// ---------------------------------------------------------------- wave matrix product
// out(i, j) = sum_k A(i, k) * B(k, j), i, j, k < n.  Every lane must call (no lane-
// dependent early exit before): lanes beyond the tile grid idle inside.
template <int T, class FA, class FB, class FO>
__device__ __forceinline__ void wave_matmul_t(int n, FA A, FB B, FO out) {
  const int lane = lane_id();
  const int tiles = n / T;
  if (lane < tiles * tiles) {
    const int i0 = (lane / tiles) * T, j0 = (lane % tiles) * T;
    int acc[T][T];
#pragma unroll
    for (int r = 0; r < T; ++r)
#pragma unroll
      for (int c = 0; c < T; ++c) acc[r][c] = 0;
    for (int k = 0; k < n; ++k) {
      int a[T], b[T];
#pragma unroll
      for (int r = 0; r < T; ++r) a[r] = A(i0 + r, k);
#pragma unroll
      for (int c = 0; c < T; ++c) b[c] = B(k, j0 + c);
#pragma unroll
      for (int r = 0; r < T; ++r)
#pragma unroll
        for (int c = 0; c < T; ++c) acc[r][c] += a[r] * b[c];
    }
#pragma unroll
    for (int r = 0; r < T; ++r)
#pragma unroll
      for (int c = 0; c < T; ++c) out(i0 + r, j0 + c, acc[r][c]);
  }
}
template <class FA, class FB, class FO>
__device__ __forceinline__ void wave_matmul(int n, FA A, FB B, FO out) {
  if (n == 32) wave_matmul_t<4>(n, A, B, out);
  else if (n == 16) wave_matmul_t<2>(n, A, B, out);
  else wave_matmul_t<1>(n, A, B, out);
}

// ---------------------------------------------------------------- transform + quantisation of one block
// R: residual (in) / reconstructed residual (out), int32 [n][n] in LDS, row stride 32.
// S: scratch int32 [32][32].  Levels go to lev (global, row stride lstride).  Returns
// (on every lane) whether any level is non-zero.
struct TqParams {
  int log2n, bd, qp;  // qp: Qp' (QpY + QpBdOffset, or the chroma equivalent)
  bool intra;
  bool dst = false;   // 4x4 intra luma: DST-VII instead of the DCT
  int sdh_scan = -1;  // >= 0: sign data hiding with this scanIdx (0 diagonal, 1 horizontal, 2 vertical)
  // 16 / 32-point TUs on the matrix cores (transform_quant_mfma); false: the LDS wave products
  // (the CTB-wavefront intra kernel keeps them: the MFMA form's registers would spill there)
  bool mfma = true;
};

// scanIdx of a TU (7.4.9.11): intra luma 4x4 / 8x8 and intra chroma 4x4 follow the mode
__device__ __forceinline__ int tu_scan_idx(bool intra, bool luma, int log2n, int mode) {
  if (!intra || !(log2n == 2 || (log2n == 3 && luma))) return 0;
  return (mode >= 6 && mode <= 14) ? 2 : ((mode >= 22 && mode <= 30) ? 1 : 0);
}

// ---------------------------------------------------------------- 16 / 32-point transforms on the matrix cores
// The four 1-D passes of a TU (forward rows, forward columns, inverse columns, inverse rows) as
// v_mfma_f32_32x32x16_f16 products that stay in registers between passes: each pass's result has
// its column on the lane and its rows in the 16 accumulator registers, so the next pass takes it
// as an operand without lane movement (the accumulator-as-operand order: element j of lane half h
// in k-step s is row kperm(s, h, j) of it).  fwd: S = R C^T, coef = C S; inv: Z = Rq^T C (= S'^T),
// R = Z^T C.  Exact integer arithmetic in f16 x f16 -> f32: residuals (<= 10 bits) and DCT entries
// (|c| <= 90) are exact in f16; the 16-bit intermediates enter as hi * 64 + lo (|hi| <= 718,
// lo in 0..63, two products combined in int32); every f32 sum stays below 2^24 (32 x 90 x 1023).
// A 16-point TU fills the top-left quarter of the 32x32 tiles (the other rows / columns are zero).
typedef _Float16 hv_half8 __attribute__((ext_vector_type(8)));
typedef float hv_float16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int kperm(int s, int h, int j) { return 16 * s + 8 * (j >> 2) + 4 * h + (j & 3); }
// row of accumulator register g (32x32 C/D layout: col = lane & 31)
__device__ __forceinline__ int acc_row(int g, int h) { return (g & 3) + 8 * (g >> 2) + 4 * h; }

template <int LG>
__device__ __forceinline__ bool transform_quant_mfma(const DctLds& D, int* R, int16_t* lev, int lstride, const TqParams& p) {
  constexpr int N = 1 << LG, KS = N / 16;
  const int lane = lane_id(), r = lane & 31, h = lane >> 5;
  const bool rv = r < N;
  auto C = [&](int k, int m) { return static_cast<int>(D.m[k << (5 - LG)][m]); };  // N-point entry (k, m)
  // ---- forward rows: S[y][u] = (sum_x R[y][x] C[u][x] + rnd) >> sh1 (A = R, B = C^T)
  hv_float16 acc = {};
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    hv_half8 a, b;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int x = 16 * s + 8 * h + j;
      a[j] = static_cast<_Float16>(rv ? R[r * 32 + x] : 0);
      b[j] = static_cast<_Float16>(rv ? C(r, x) : 0);
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
  }
  const int sh1 = LG + p.bd - 9, r1 = 1 << (sh1 - 1);
  int v[16];
#pragma unroll
  for (int g = 0; g < 16; ++g) v[g] = (static_cast<int>(acc[g]) + r1) >> sh1;
  // ---- forward columns: coef[v][u] = (sum_y C[v][y] S[y][u] + rnd) >> sh2 (A = C, B = S)
  hv_float16 chi = {}, clo = {};
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    hv_half8 a, bh, bl;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a[j] = static_cast<_Float16>(rv ? C(r, kperm(s, h, j)) : 0);
      bh[j] = static_cast<_Float16>(v[8 * s + j] >> 6);
      bl[j] = static_cast<_Float16>(v[8 * s + j] & 63);
    }
    chi = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, bh, chi, 0, 0, 0);
    clo = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, bl, clo, 0, 0, 0);
  }
  const int sh2 = LG + 6, r2 = 1 << (sh2 - 1);
  const int qm = p.qp % 6, qs = p.qp / 6;
  const int qbits = 14 + qs + (15 - p.bd - LG);
  const int qscale = hevc::kQuantScale[qm];
  const int64_t qoff = static_cast<int64_t>(p.intra ? 171 : 85) << (qbits - 9);
  const int dscale = 16 * hevc::kLevelScale[qm];
  const int dsh = p.bd + LG - 5;
  const int64_t drnd = 1ll << (dsh - 1);
  int any = 0;
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const int vr = acc_row(g, h);
    int c = (static_cast<int>(chi[g]) * 64 + static_cast<int>(clo[g]) + r2) >> sh2;
    const int a = c < 0 ? -c : c;
    int l = static_cast<int>((static_cast<int64_t>(a) * qscale + qoff) >> qbits);
    l = l > 32767 ? 32767 : l;
    l = c < 0 ? -l : l;
    const bool in = rv && vr < N;
    if (in) lev[vr * lstride + r] = static_cast<int16_t>(l);
    any |= in && l != 0;
    // dequantise (8.6.3, flat scaling): the inverse's input, kept in the register
    int64_t d = ((static_cast<int64_t>(in ? l : 0) * dscale) << qs) + drnd;
    d >>= dsh;
    v[g] = static_cast<int>(d < -32768 ? -32768 : (d > 32767 ? 32767 : d));
  }
  if (__ballot(any) == 0) {
    for (int i = lane; i < N * N; i += 64) R[(i >> LG) * 32 + (i & (N - 1))] = 0;
    wave_sync();
    return false;
  }
  // ---- inverse columns: Z[x][y] = S'[y][x] = clip16((sum_k C[k][y] Rq[k][x] + 64) >> 7)
  // (A = Rq as the transposed operand, B = C with B[k][y] = C[k][y])
  hv_float16 zhi = {}, zlo = {};
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    hv_half8 ah, al, b;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ah[j] = static_cast<_Float16>(v[8 * s + j] >> 6);
      al[j] = static_cast<_Float16>(v[8 * s + j] & 63);
      b[j] = static_cast<_Float16>(rv ? C(kperm(s, h, j), r) : 0);
    }
    zhi = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, b, zhi, 0, 0, 0);
    zlo = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, b, zlo, 0, 0, 0);
  }
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const int z = (static_cast<int>(zhi[g]) * 64 + static_cast<int>(zlo[g]) + 64) >> 7;
    v[g] = z < -32768 ? -32768 : (z > 32767 ? 32767 : z);
  }
  // ---- inverse rows: R[y][x] = (sum_k S'[y][k] C[k][x] + rnd) >> (20 - bd) (A = Z transposed)
  hv_float16 rhi = {}, rlo = {};
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    hv_half8 ah, al, b;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ah[j] = static_cast<_Float16>(v[8 * s + j] >> 6);
      al[j] = static_cast<_Float16>(v[8 * s + j] & 63);
      b[j] = static_cast<_Float16>(rv ? C(kperm(s, h, j), r) : 0);
    }
    rhi = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, b, rhi, 0, 0, 0);
    rlo = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, b, rlo, 0, 0, 0);
  }
  const int sh4 = 20 - p.bd, r4 = 1 << (sh4 - 1);
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const int y = acc_row(g, h);
    if (rv && y < N) R[y * 32 + r] = (static_cast<int>(rhi[g]) * 64 + static_cast<int>(rlo[g]) + r4) >> sh4;
  }
  wave_sync();
  return true;
}

__device__ __forceinline__ bool transform_quant_block(const DctLds& D, int* R, int* S, int16_t* lev, int lstride,
                                                      const TqParams& p) {
  const int n = 1 << p.log2n, lg = p.log2n;
  if (p.mfma && !p.dst && p.sdh_scan < 0 && (lg == 4 || lg == 5)) {
    wave_sync();  // R was written by other lanes
    return lg == 5 ? transform_quant_mfma<5>(D, R, lev, lstride, p) : transform_quant_mfma<4>(D, R, lev, lstride, p);
  }
  const bool dst = p.dst;
  auto cn = [&](const DctLds& M, int l2, int k, int m) { return dst ? static_cast<int>(M.dst[k][m]) : hv::cn(M, l2, k, m); };
  // forward, stage 1 (rows): S[y][k] = (sum_x R[y][x] * C[k][x] + rnd) >> sh1
  const int sh1 = lg + p.bd - 9, r1 = 1 << (sh1 - 1);
  wave_matmul(n, [&](int y, int x) { return R[y * 32 + x]; }, [&](int x, int k) { return cn(D, lg, k, x); },
              [&](int y, int k, int v) { S[y * 32 + k] = (v + r1) >> sh1; });
  wave_sync();
  // stage 2 (columns): coefficient (v, u) = (sum_y C[v][y] * S[y][u] + rnd) >> sh2
  const int sh2 = lg + 6, r2 = 1 << (sh2 - 1);
  const int qm = p.qp % 6, qs = p.qp / 6;
  const int qbits = 14 + qs + (15 - p.bd - lg);
  const int qscale = hevc::kQuantScale[qm];
  const int64_t qoff = static_cast<int64_t>(p.intra ? 171 : 85) << (qbits - 9);
  const int dscale = 16 * hevc::kLevelScale[qm];
  const int dsh = p.bd + lg - 5;
  const int64_t drnd = 1ll << (dsh - 1);
  int any = 0;
  wave_matmul(n, [&](int v, int y) { return cn(D, lg, v, y); }, [&](int y, int u) { return S[y * 32 + u]; },
              [&](int v, int u, int c) {
                c = (c + r2) >> sh2;
                const int a = c < 0 ? -c : c;
                int l = static_cast<int>((static_cast<int64_t>(a) * qscale + qoff) >> qbits);
                l = l > 32767 ? 32767 : l;
                if (p.sdh_scan >= 0) {
                  // level, quantisation remainder (HM deltaU) and coefficient sign, packed for
                  // the parity pass below; dequantisation follows it
                  const int dl = static_cast<int>(((static_cast<int64_t>(a) * qscale) - (static_cast<int64_t>(l) << qbits)) >>
                                                  (qbits - 8));
                  const int sl = c < 0 ? -l : l;
                  R[v * 32 + u] = static_cast<int>((static_cast<uint32_t>(sl) & 0xFFFFu) |
                                                   ((static_cast<uint32_t>(dl) & 0x7FFFu) << 16) | (c < 0 ? 0x80000000u : 0u));
                  return;
                }
                l = c < 0 ? -l : l;
                lev[v * lstride + u] = static_cast<int16_t>(l);
                any |= l != 0;
                // dequantise (8.6.3, flat scaling) into R for the inverse transform
                int64_t d = ((static_cast<int64_t>(l) * dscale) << qs) + drnd;
                d >>= dsh;
                R[v * 32 + u] = static_cast<int>(d < -32768 ? -32768 : (d > 32767 ? 32767 : d));
              });
  wave_sync();
  if (p.sdh_scan >= 0) {
    // sign data hiding (7.4.9.11; HM's parity fix): in every 4x4 group whose significant
    // span exceeds 3 scan positions the sum of absolute levels must be odd exactly when the
    // first significant coefficient is negative; otherwise the cheapest +-1 change by the
    // quantisation remainder fixes it.  One lane per group.
    const int nsb = n >> 2, lsb = lg - 2, ngr = nsb * nsb;
    const int lane = lane_id();
    auto lvl_at = [&](int x, int y) { return static_cast<int>(static_cast<int16_t>(R[y * 32 + x] & 0xFFFF)); };
    int gi = -1, gnz = 0;
    if (lane < ngr) {
      const int gx = lane % nsb, gy = lane / nsb;
      for (int i = 0; i < ngr; ++i)
        if (hevc::scan_pos(p.sdh_scan, lsb, i) == (gx | (gy << 8))) gi = i;
      for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) gnz |= lvl_at(gx * 4 + x, gy * 4 + y);
    }
    const int lastgi = -min64(-(gnz ? gi : -1));
    if (lane < ngr && gnz) {
      const int gx = lane % nsb, gy = lane / nsb;
      int px[16], py[16], lv[16], first = -1, last = -1, sum = 0;
      for (int q = 0; q < 16; ++q) {
        const int sp = hevc::scan_pos(p.sdh_scan, 2, q);
        px[q] = gx * 4 + (sp & 255);
        py[q] = gy * 4 + (sp >> 8);
        lv[q] = lvl_at(px[q], py[q]);
        if (lv[q]) {
          if (first < 0) first = q;
          last = q;
          sum += lv[q] < 0 ? -lv[q] : lv[q];
        }
      }
      const int signbit = lv[first] < 0 ? 1 : 0;
      if (last - first > 3 && (sum & 1) != signbit) {
        int best = 0x7FFFFFFF, bq = first, bch = 1;
        for (int q = (gi == lastgi ? last : 15); q >= 0; --q) {
          const int w = R[py[q] * 32 + px[q]];
          const int dl = (w << 1) >> 17;  // 15-bit signed remainder
          int cost, ch = 1;
          if (lv[q] != 0) {
            if (dl > 0) {
              cost = -dl;
            } else if (q == first && (lv[q] == 1 || lv[q] == -1)) {
              cost = 0x7FFFFFFF;
            } else {
              cost = dl;
              ch = -1;
            }
          } else if (q < first && ((static_cast<uint32_t>(w) >> 31) != static_cast<uint32_t>(signbit))) {
            cost = 0x7FFFFFFF;
          } else {
            cost = -dl;
          }
          if (cost < best) {
            best = cost;
            bq = q;
            bch = ch;
          }
        }
        const int w = R[py[bq] * 32 + px[bq]];
        const bool neg = (static_cast<uint32_t>(w) >> 31) != 0;
        int l = lv[bq];
        if (l == 32767 || l == -32767) bch = -1;
        l += neg ? -bch : bch;
        R[py[bq] * 32 + px[bq]] = static_cast<int>((static_cast<uint32_t>(w) & 0xFFFF0000u) | (static_cast<uint32_t>(l) & 0xFFFFu));
      }
    }
    wave_sync();
    for (int i = lane; i < n * n; i += 64) {  // levels out + dequantisation (8.6.3, flat scaling)
      const int y = i >> lg, x = i & (n - 1);
      const int l = lvl_at(x, y);
      lev[y * lstride + x] = static_cast<int16_t>(l);
      any |= l != 0;
      int64_t d = ((static_cast<int64_t>(l) * dscale) << qs) + drnd;
      d >>= dsh;
      R[y * 32 + x] = static_cast<int>(d < -32768 ? -32768 : (d > 32767 ? 32767 : d));
    }
    wave_sync();
  }
  const bool nz = __ballot(any) != 0;
  if (!nz) return false;  // residual is zero: R is all zero too
  // inverse, stage 1 (columns): S[y][x] = clip16((sum_k C[k][y] * R[k][x] + 64) >> 7)
  wave_matmul(n, [&](int y, int k) { return cn(D, lg, k, y); }, [&](int k, int x) { return R[k * 32 + x]; },
              [&](int y, int x, int v) {
                v = (v + 64) >> 7;
                S[y * 32 + x] = v < -32768 ? -32768 : (v > 32767 ? 32767 : v);
              });
  wave_sync();
  // stage 2 (rows): R[y][x] = (sum_k S[y][k] * C[k][x] + rnd) >> (20 - bd)
  const int sh4 = 20 - p.bd, r4 = 1 << (sh4 - 1);
  wave_matmul(n, [&](int y, int k) { return S[y * 32 + k]; }, [&](int k, int x) { return cn(D, lg, k, x); },
              [&](int y, int x, int v) { R[y * 32 + x] = (v + r4) >> sh4; });
  wave_sync();
  return true;
}

// ---------------------------------------------------------------- intra reference samples
// p[0 .. 4n]: p[2n - 1 - y] = p(-1, y) for y = -1 .. 2n-1 (index 2n = corner),
// p[2n + 1 + x] = p(x, -1).  `avail(i)` / `fetch(i)` give availability and value of
// entry i; substitution per 8.4.4.2.2 (nearest available entry before i in this
// order, or the first available one), done wave-parallel with ballots.
template <class FAV, class FGET>
__device__ __forceinline__ void build_refs(int* p, int n, int bd, FAV avail, FGET fetch) {
  const int lane = lane_id();
  const int E = 4 * n + 1;
  const int i0 = lane, i1 = lane + 64;
  const bool a0 = i0 < E && avail(i0);
  const bool a1 = i1 < E && avail(i1);
  const unsigned long long b0 = __ballot(a0), b1 = __ballot(a1);
  const bool a2 = E > 128 && avail(128);  // uniform
  if (a0) p[i0] = fetch(i0);
  if (a1) p[i1] = fetch(i1);
  if (lane == 0 && a2) p[128] = fetch(128);
  wave_sync();
  const bool none = b0 == 0 && b1 == 0 && !a2;
  int first = 0;
  if (b0) first = __builtin_ctzll(b0);
  else if (b1) first = 64 + __builtin_ctzll(b1);
  else first = 128;
  auto src_of = [&](int i) {
    // highest available index < i
    if (i < 64) {
      const unsigned long long m = i ? (b0 & ((1ull << i) - 1ull)) : 0ull;
      if (m) return 63 - __builtin_clzll(m);
      return -1;
    }
    if (i < 128) {
      const unsigned long long m = (i - 64) ? (b1 & ((1ull << (i - 64)) - 1ull)) : 0ull;
      if (m) return 64 + 63 - __builtin_clzll(m);
      if (b0) return 63 - __builtin_clzll(b0);
      return -1;
    }
    if (b1) return 64 + 63 - __builtin_clzll(b1);
    if (b0) return 63 - __builtin_clzll(b0);
    return -1;
  };
  int v0 = 0, v1 = 0, v2 = 0;
  const int mid = 1 << (bd - 1);
  if (i0 < E && !a0) {
    const int s = src_of(i0);
    v0 = none ? mid : p[s >= 0 ? s : first];
  }
  if (i1 < E && !a1) {
    const int s = src_of(i1);
    v1 = none ? mid : p[s >= 0 ? s : first];
  }
  if (lane == 0 && E > 128 && !a2) {
    const int s = src_of(128);
    v2 = none ? mid : p[s >= 0 ? s : first];
  }
  wave_sync();
  if (i0 < E && !a0) p[i0] = v0;
  if (i1 < E && !a1) p[i1] = v1;
  if (lane == 0 && E > 128 && !a2) p[128] = v2;
  wave_sync();
}

// 8.4.4.2.3 filtering of luma references (q: output array, same layout)
__device__ __forceinline__ bool intra_filter_flag(int mode, int n) {
  if (mode == 1 || n == 4) return false;
  const int d0 = mode - 26 < 0 ? 26 - mode : mode - 26, d1 = mode - 10 < 0 ? 10 - mode : mode - 10;
  const int md = d0 < d1 ? d0 : d1;
  const int thr = n == 8 ? 7 : (n == 16 ? 1 : 0);
  return md > thr;
}
__device__ __forceinline__ void filter_refs(const int* p, int* q, int n, int bd, bool strong_enabled) {
  const int lane = lane_id();
  const int E = 4 * n + 1, c = 2 * n;
  const int tl = p[c], bl = p[0], tr = p[E - 1];
  const bool bi = strong_enabled && n == 32 &&
                  abs(tl + tr - 2 * p[c + 1 + (n - 1)]) < (1 << (bd - 5)) &&
                  abs(tl + bl - 2 * p[c - 1 - (n - 1)]) < (1 << (bd - 5));
  for (int i = lane; i < E; i += 64) {
    int v;
    if (i == 0 || i == E - 1 || (bi && i == c)) {
      v = p[i];
    } else if (bi) {
      if (i < c) {
        const int y = c - 1 - i;  // 0..62
        v = ((63 - y) * tl + (y + 1) * bl + 32) >> 6;
      } else {
        const int x = i - c - 1;
        v = ((63 - x) * tl + (x + 1) * tr + 32) >> 6;
      }
    } else {
      v = (p[i - 1] + 2 * p[i] + p[i + 1] + 2) >> 2;
    }
    q[i] = v;
  }
  wave_sync();
}

// one predicted sample (8.4.4.2.4 - 8.4.4.2.6); dc: precomputed DC value (mode 1);
// edge: luma block smaller than 32 (DC / pure horizontal / pure vertical boundary filters)
template <typename RT>
__device__ __forceinline__ int intra_pred_sample(const RT* p, int n, int log2n, int mode, int x, int y, int dc,
                                                 bool edge, int maxv) {
  const int c = 2 * n;
  auto L = [&](int yy) { return p[c - 1 - yy]; };
  auto T = [&](int xx) { return p[c + 1 + xx]; };
  if (mode == 0) return ((n - 1 - x) * L(y) + (x + 1) * T(n) + (n - 1 - y) * T(x) + (y + 1) * L(n) + n) >> (log2n + 1);
  if (mode == 1) {
    if (!edge) return dc;
    if (x == 0 && y == 0) return (L(0) + 2 * dc + T(0) + 2) >> 2;
    if (y == 0) return (T(x) + 3 * dc + 2) >> 2;
    if (x == 0) return (L(y) + 3 * dc + 2) >> 2;
    return dc;
  }
  const int ang = hevc::kIntraPredAngle[mode];
  const int inv = (mode >= 11 && mode <= 25) ? hevc::kInvAngle[mode - 11] : 0;
  if (mode >= 18) {
    const int idx = ((y + 1) * ang) >> 5, fact = ((y + 1) * ang) & 31;
    const int k0 = x + idx + 1;
    auto R = [&](int k) { return k >= 0 ? T(k - 1) : L(-1 + ((k * inv + 128) >> 8)); };
    int v = fact ? ((32 - fact) * R(k0) + fact * R(k0 + 1) + 16) >> 5 : R(k0);
    if (mode == 26 && edge && x == 0) {
      v = T(0) + ((L(y) - L(-1)) >> 1);
      v = v < 0 ? 0 : (v > maxv ? maxv : v);
    }
    return v;
  }
  const int idx = ((x + 1) * ang) >> 5, fact = ((x + 1) * ang) & 31;
  const int k0 = y + idx + 1;
  auto R = [&](int k) { return k >= 0 ? L(k - 1) : T(-1 + ((k * inv + 128) >> 8)); };
  int v = fact ? ((32 - fact) * R(k0) + fact * R(k0 + 1) + 16) >> 5 : R(k0);
  if (mode == 10 && edge && y == 0) {
    v = L(0) + ((T(x) - T(-1)) >> 1);
    v = v < 0 ? 0 : (v > maxv ? maxv : v);
  }
  return v;
}

// Four predicted samples of an n x n block for the MFMA SATD layout (hevc_intra.hip): the 4x4
// block at (bx, by), lane group g.  Vertical-family, planar and DC modes give row g (samples
// (bx + j, by + g)); horizontal-family modes give column g (samples (bx + g, by + j)), so the
// angular interpolation position is the same for all four samples and 5 reference loads
// serve them (the Hadamard SATD of a block equals that of its transpose).  *transposed tells
// the caller which layout was produced.
template <typename RT>
__device__ __forceinline__ void intra_pred4(const RT* p, int n, int log2n, int mode, int bx, int by, int g, int dc,
                                            bool edge, int maxv, int (&o)[4], bool* transposed) {
  const int c = 2 * n;
  auto L = [&](int yy) { return p[c - 1 - yy]; };
  auto T = [&](int xx) { return p[c + 1 + xx]; };
  *transposed = mode >= 2 && mode < 18;
  if (mode < 2) {
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = intra_pred_sample(p, n, log2n, mode, bx + j, by + g, dc, edge, maxv);
    return;
  }
  const int ang = hevc::kIntraPredAngle[mode];
  const int inv = (mode >= 11 && mode <= 25) ? hevc::kInvAngle[mode - 11] : 0;
  const bool vert = mode >= 18;
  const int along = vert ? by + g : bx + g;    // the coordinate the projection depends on
  const int across = vert ? bx : by;           // first of the 4 samples' other coordinate
  const int idx = ((along + 1) * ang) >> 5, f = ((along + 1) * ang) & 31;
  const int k0 = across + idx + 1;
  int r[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int k = k0 + j;
    const int proj = -1 + ((k * inv + 128) >> 8);
    r[j] = k >= 0 ? (vert ? T(k - 1) : L(k - 1)) : (vert ? L(proj) : T(proj));
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = f ? ((32 - f) * r[j] + f * r[j + 1] + 16) >> 5 : r[j];
  if (edge && mode == 26 && bx == 0) {  // column x = 0 of the pure vertical mode (row layout: sample j = 0)
    const int v = T(0) + ((L(by + g) - L(-1)) >> 1);
    o[0] = v < 0 ? 0 : (v > maxv ? maxv : v);
  }
  if (edge && mode == 10 && by == 0) {  // row y = 0 of the pure horizontal mode (column layout: sample j = 0)
    const int v = L(0) + ((T(bx + g) - T(-1)) >> 1);
    o[0] = v < 0 ? 0 : (v > maxv ? maxv : v);
  }
}

// 8x8 block of the prediction of an n x n block (n >= 8) at offset (ox, oy): angular
// modes load 9 reference samples per row (vertical family) or column (horizontal
// family) and interpolate 8 outputs from registers.
__device__ __forceinline__ void intra_pred8(const int* p, int n, int log2n, int mode, int ox, int oy, int dc, bool edge,
                                            int maxv, int (&o)[64]) {
  const int c = 2 * n;
  auto L = [&](int yy) { return p[c - 1 - yy]; };
  auto T = [&](int xx) { return p[c + 1 + xx]; };
  if (mode == 0) {
    const int tn = T(n), ln = L(n);
    int lv[8], tv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      lv[k] = L(oy + k);
      tv[k] = T(ox + k);
    }
#pragma unroll
    for (int y = 0; y < 8; ++y)
#pragma unroll
      for (int x = 0; x < 8; ++x) {
        const int X = ox + x, Y = oy + y;
        o[y * 8 + x] = ((n - 1 - X) * lv[y] + (X + 1) * tn + (n - 1 - Y) * tv[x] + (Y + 1) * ln + n) >> (log2n + 1);
      }
    return;
  }
  if (mode == 1) {
#pragma unroll
    for (int i = 0; i < 64; ++i) o[i] = dc;
    if (edge) {
      if (oy == 0)
#pragma unroll
        for (int x = 0; x < 8; ++x) o[x] = (T(ox + x) + 3 * dc + 2) >> 2;
      if (ox == 0)
#pragma unroll
        for (int y = 0; y < 8; ++y) o[y * 8] = (L(oy + y) + 3 * dc + 2) >> 2;
      if (ox == 0 && oy == 0) o[0] = (L(0) + 2 * dc + T(0) + 2) >> 2;
    }
    return;
  }
  const int ang = hevc::kIntraPredAngle[mode];
  const int inv = (mode >= 11 && mode <= 25) ? hevc::kInvAngle[mode - 11] : 0;
  if (mode >= 18) {
#pragma unroll
    for (int y = 0; y < 8; ++y) {
      const int Y = oy + y;
      const int idx = ((Y + 1) * ang) >> 5, f = ((Y + 1) * ang) & 31;
      const int base = ox + idx + 1;
      int r[9];
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const int k = base + j;
        r[j] = k >= 0 ? T(k - 1) : L(-1 + ((k * inv + 128) >> 8));
      }
#pragma unroll
      for (int x = 0; x < 8; ++x) o[y * 8 + x] = f ? ((32 - f) * r[x] + f * r[x + 1] + 16) >> 5 : r[x];
      if (mode == 26 && edge && ox == 0) {
        const int v = T(0) + ((L(Y) - L(-1)) >> 1);
        o[y * 8] = v < 0 ? 0 : (v > maxv ? maxv : v);
      }
    }
    return;
  }
#pragma unroll
  for (int x = 0; x < 8; ++x) {
    const int X = ox + x;
    const int idx = ((X + 1) * ang) >> 5, f = ((X + 1) * ang) & 31;
    const int base = oy + idx + 1;
    int r[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int k = base + j;
      r[j] = k >= 0 ? L(k - 1) : T(-1 + ((k * inv + 128) >> 8));
    }
#pragma unroll
    for (int y = 0; y < 8; ++y) o[y * 8 + x] = f ? ((32 - f) * r[y] + f * r[y + 1] + 16) >> 5 : r[y];
    if (mode == 10 && edge && oy == 0) {
      const int v = L(0) + ((T(X) - T(-1)) >> 1);
      o[x] = v < 0 ? 0 : (v > maxv ? maxv : v);
    }
  }
}

// DC value of the reference array (wave reduction)
__device__ __forceinline__ int intra_dc(const int* p, int n, int log2n) {
  const int lane = lane_id();
  const int c = 2 * n;
  int s = 0;
  if (lane < n) s = p[c + 1 + lane] + p[c - 1 - lane];
  s = sum64(s);
  return (s + n) >> (log2n + 1);
}

}  // namespace hv
}  // namespace gpu
}  // namespace mivc
