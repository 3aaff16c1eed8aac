// HEVC intra coding on gfx950: open-loop analysis + closed-loop
// reconstruction.
//
// * hevc_intra_analyze (grid = CTBs x slots, 256 threads): every CU of the 32/16/8
//   quadtree x all 35 modes is predicted from *source* neighbours (normative
//   availability, substitution and filtering) and costed with 4x4 Hadamard SATDs on the
//   matrix cores (v_mfma_f32_16x16x16_f16: 16 blocks per instruction); the
//   CTB then picks the best mode per CU and the split that minimises SATD + lambda *
//   bits.  No dependency between CTBs: the whole picture is analysed in parallel.
// * hevc_intra_recon (grid = slots x 3 components, 8 waves per workgroup): CTBs in wavefront order
//   (MB-row progress counters in LDS, 2-CTB lag as the H.264 kernels), CUs in z-order
//   inside a CTB: reference samples from the reconstruction, prediction, forward
//   transform, quantisation, dequantisation and the normative inverse transform
//   (wave-level matrix products in LDS, hevc_common.h).  In P pictures only intra
//   CUs are visited (inter CUs were reconstructed by hevc_inter).
#include "hevc_common.h"

namespace mivc {
namespace gpu {

using hevc::CtuInfo;
using hevc::CuInfo;
using hevc::zorder8;

struct HevcIntraArgs {
  HevcGeom g;
  const uint16_t *src_y, *src_u, *src_v;  // [B] padded source planes
  uint16_t *rec_y, *rec_u, *rec_v;        // [B] reconstruction (unfiltered)
  CtuInfo* ctu;                           // [B, nctb]
  CuInfo* cu;                             // [B, nctb * 16]
  int16_t *coef_y, *coef_u, *coef_v;      // [B] level planes
  const int* qp;                          // [B, nctb] QpY per CTB (AQ, hevc_aq_ctb)
  const int8_t* run;                      // [B] 0 idle, 1 all CUs (I picture), 2 intra CUs only (P picture)
  int* cand;                              // [B, nctb, 2, 21] best cost / mode per CU of the analysis (may be null)
  int bd;
  int* err;
  int sdh;                                // sign data hiding in the quantiser
  int nxn_in_p;                           // evaluate PART_NxN in P pictures too
  const uint8_t* ctb_mask;                // [B, nctb] analyse only where nonzero (P pictures: the CTBs
                                          // where intra may beat the motion search); null = every CTB
  int ctu64;                              // 64x64 CTUs: the 32x32 blocks are coded in z-order inside them
};

constexpr int kNoIntra = 1 << 26;  // candidate cost of a CTB the analysis skipped (inter decisive)

// luma neighbour (xr, yr) of a position relative to the 32x32 block (rx, ry): z-scan
// availability (6.4.1) at the 4x4 minimum-TB granularity; zcur = z-order index (zorder4) of
// the current block's first 4x4 block.  32x32 CTBs: blocks in raster order; 64x64 CTUs
// (ctu64): CTUs in raster order, their four blocks in z-order.
__device__ __forceinline__ bool nb_avail(int xr, int yr, int zcur, int rx, int ry, int wctb, int hctb, int ctu64) {
  const int tx = rx + (xr >> 5), ty = ry + (yr >> 5);
  if (tx < 0 || ty < 0 || tx >= wctb || ty >= hctb) return false;
  if (tx == rx && ty == ry) return zorder4((xr & 31) >> 2, (yr & 31) >> 2) < zcur;
  if (!ctu64) return ty < ry || (ty == ry && tx < rx);
  const int ux = tx >> 1, uy = ty >> 1, cx = rx >> 1, cy = ry >> 1;
  if (ux != cx || uy != cy) return uy < cy || (uy == cy && ux < cx);
  return ((tx & 1) | ((ty & 1) << 1)) < ((rx & 1) | ((ry & 1) << 1));
}

__device__ __forceinline__ void ref_pos(int i, int n, int cx, int cy, int* x, int* y) {
  if (i < 2 * n) {
    *x = cx - 1;
    *y = cy + 2 * n - 1 - i;
  } else if (i == 2 * n) {
    *x = cx - 1;
    *y = cy - 1;
  } else {
    *x = cx + i - 2 * n - 1;
    *y = cy - 1;
  }
}

__device__ __forceinline__ int lambda_satd(int qp, int bd) {
  return static_cast<int>(0.755f * exp2f((qp - 12) / 6.0f) * static_cast<float>(1 << (bd - 8)) + 0.5f);
}

// ============================================================== analysis
constexpr int kCuCount = 21;  // 1 x 32, 4 x 16, 16 x 8
constexpr int kPuCount = 64;  // PART_NxN: four 4x4 PUs of each 8x8 CU (z-order)
struct AnalyzeShared {
  int16_t ext[65 * 65];        // source samples, x, y in [-1, 63] relative to the CTB
  int16_t refs[2][917];        // per CU: unfiltered / filtered reference arrays (samples: 16 bits)
  int cost[kCuCount][36];
  uint8_t done[kCuCount][36];  // (CU, mode) evaluated
  int dc[kCuCount];
  int best_mode[kCuCount], best_cost[kCuCount];
  int16_t refs4[kPuCount][17]; // 4x4 PUs: reference arrays (no filtering at 4x4)
  int cost4[kPuCount][36];
  uint8_t done4[kPuCount][36];
  int dc4[kPuCount];
  int best4_mode[kPuCount], best4_cost[kPuCount];
  int nxn[16];                 // per 8x8 CU: packed PU modes (bit 24) or 0
  int rmode[128];              // refinement rounds: the mode each item evaluates (-1: none)
};

// SATD on the matrix cores.  One v_mfma_f32_16x16x16_f16 transforms 16 4x4 residual blocks:
// B column n = block n as a 16-vector (k = 4 * row + column; lane (n = lane & 15, g = lane >> 4)
// supplies row g), A = the Sylvester H16 = H4 (x) H4 (entries (-1)^popcount(m & k)), so column n
// of the product holds the 2-D Hadamard coefficients of block n.  Residuals of 8- and 10-bit
// samples are integers below 2^11 in magnitude (exact in f16) and every product sum is below
// 2^24 (exact in the f32 accumulator).  Returns, at every lane of column n, the block's
// sum |coefficients| (the VALU formulation's butterflies and registers are gone: a lane holds
// 4 residuals instead of 64).
typedef float v4f_t __attribute__((ext_vector_type(4)));
typedef _Float16 v4h_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4h_t h16_rows() {
  const int lane = threadIdx.x & 63, m = lane & 15, kg = lane >> 4;
  v4h_t h;
#pragma unroll
  for (int j = 0; j < 4; ++j) h[j] = (__builtin_popcount(m & (4 * kg + j)) & 1) ? _Float16(-1.0f) : _Float16(1.0f);
  return h;
}

__device__ __forceinline__ int hadamard_col_sum(v4h_t H, const int (&r)[4]) {
  v4h_t b;
#pragma unroll
  for (int j = 0; j < 4; ++j) b[j] = static_cast<_Float16>(static_cast<float>(r[j]));
  const v4f_t d = __builtin_amdgcn_mfma_f32_16x16x16f16(H, b, v4f_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  int s = static_cast<int>(__builtin_fabsf(d[0]) + __builtin_fabsf(d[1]) + __builtin_fabsf(d[2]) + __builtin_fabsf(d[3]));
  s += __shfl_xor(s, 16, 64);
  s += __shfl_xor(s, 32, 64);
  return s;
}

// CTB-relative position of 4x4 PU `pu` (8x8 CU pu >> 2 in z-order, PU pu & 3 in raster)
__device__ __forceinline__ void pu_of(int pu, int* px, int* py) {
  const int k8 = pu >> 2, k = pu & 3;
  *px = ((k8 & 1) | ((k8 >> 1) & 2)) * 8 + (k & 1) * 4;
  *py = (((k8 >> 1) & 1) | ((k8 >> 2) & 2)) * 8 + (k >> 1) * 4;
}

__device__ __forceinline__ void cu_of(int c, int* cx, int* cy, int* n, int* off) {
  if (c == 0) {
    *cx = 0;
    *cy = 0;
    *n = 32;
    *off = 0;
  } else if (c < 5) {
    const int q = c - 1;
    *cx = (q & 1) * 16;
    *cy = (q >> 1) * 16;
    *n = 16;
    *off = 129 + q * 65;
  } else {
    const int k = c - 5;  // z-order of the 8x8 CU inside the CTB
    *cx = ((k & 1) | ((k >> 1) & 2)) * 8;
    *cy = (((k >> 1) & 1) | ((k >> 2) & 2)) * 8;
    *n = 8;
    *off = 129 + 4 * 65 + k * 33;
  }
}

__global__ __launch_bounds__(256, 4) void hevc_intra_analyze(HevcIntraArgs a) {
  __shared__ AnalyzeShared S;
  const HevcGeom& g = a.g;
  const int ci = blockIdx.x, slot = blockIdx.y;
  if (a.run[slot] == 0) return;
  // PART_NxN candidates in I pictures (and P pictures when asked): intra CUs are rare in P
  // pictures and 8x8 ones rarer, the 4x4 search is a third of this kernel
  const bool nxn_on = a.run[slot] == 1 || a.nxn_in_p;
  if (a.ctb_mask && !a.ctb_mask[static_cast<size_t>(slot) * g.nctb() + ci]) {
    // inter is decisive in this CTB: no intra candidates (a cost no inter cost reaches, DC)
    if (a.cand && threadIdx.x < kCandStride) {
      int* cd = a.cand + (static_cast<size_t>(slot) * g.nctb() + ci) * kCandStride;
      const int t = threadIdx.x;
      cd[t] = t < kCuCount ? kNoIntra : (t < 2 * kCuCount ? 1 : 0);
    }
    return;
  }
  const int rx = ci % g.wctb, ry = ci / g.wctb;
  const int X0 = rx * 32, Y0 = ry * 32;
  const int tid = threadIdx.x;
  const int bd = a.bd, maxv = (1 << bd) - 1;
  const uint16_t* src = a.src_y + slot * g.ysize();
  for (int i = tid; i < 65 * 65; i += 256) {
    const int y = i / 65 - 1, x = i % 65 - 1;
    const int xx = clampi(X0 + x, 0, g.W - 1), yy = clampi(Y0 + y, 0, g.H - 1);
    S.ext[i] = static_cast<int16_t>(src[static_cast<size_t>(yy) * g.W + xx]);
  }
  for (int i = tid; i < kCuCount * 36; i += 256) {
    (&S.cost[0][0])[i] = 0;
    (&S.done[0][0])[i] = 0;
  }
  __syncthreads();
  // reference arrays of the 21 CUs: availability + serial substitution, one thread per CU
  if (tid < kCuCount) {
    int cx, cy, n, off;
    cu_of(tid, &cx, &cy, &n, &off);
    const int zc = 4 * zorder8(cx >> 3, cy >> 3);
    const int E = 4 * n + 1;
    int16_t* p = S.refs[0] + off;
    int first = -1;
    for (int i = 0; i < E; ++i) {
      int x, y;
      ref_pos(i, n, cx, cy, &x, &y);
      if (nb_avail(x, y, zc, rx, ry, g.wctb, g.hctb, a.ctu64)) {
        p[i] = S.ext[(y + 1) * 65 + x + 1];
        if (first < 0) first = i;
      } else {
        p[i] = -1;
      }
    }
    if (first < 0) {
      for (int i = 0; i < E; ++i) p[i] = 1 << (bd - 1);
    } else {
      if (p[0] < 0) p[0] = p[first];
      for (int i = 1; i < E; ++i)
        if (p[i] < 0) p[i] = p[i - 1];
    }
    // filtered copy (8.4.4.2.3; strong smoothing for 32x32)
    int16_t* q = S.refs[1] + off;
    const int c = 2 * n, tl = p[c], bl = p[0], tr = p[E - 1];
    const bool bi = n == 32 && abs(tl + tr - 2 * p[c + n]) < (1 << (bd - 5)) && abs(tl + bl - 2 * p[c - n]) < (1 << (bd - 5));
    for (int i = 0; i < E; ++i) {
      if (i == 0 || i == E - 1) q[i] = p[i];
      else if (bi) q[i] = i == c ? tl : (i < c ? ((63 - (c - 1 - i)) * tl + (c - i) * bl + 32) >> 6
                                              : ((63 - (i - c - 1)) * tl + (i - c) * tr + 32) >> 6);
      else q[i] = (p[i - 1] + 2 * p[i] + p[i + 1] + 2) >> 2;
    }
    int s = n;
    for (int k = 0; k < n; ++k) s += p[c + 1 + k] + p[c - 1 - k];
    const int lg = n == 32 ? 5 : (n == 16 ? 4 : 3);
    S.dc[tid] = s >> (lg + 1);
  } else if (nxn_on && tid >= 64 && tid < 64 + kPuCount) {  // 4x4 PU reference arrays (z4 = PU index)
    const int pu = tid - 64;
    int px, py;
    pu_of(pu, &px, &py);
    int16_t* p = S.refs4[pu];
    int first = -1;
    for (int i = 0; i < 17; ++i) {
      int x, y;
      ref_pos(i, 4, px, py, &x, &y);
      if (nb_avail(x, y, pu, rx, ry, g.wctb, g.hctb, a.ctu64)) {
        p[i] = S.ext[(y + 1) * 65 + x + 1];
        if (first < 0) first = i;
      } else {
        p[i] = -1;
      }
    }
    if (first < 0) {
      for (int i = 0; i < 17; ++i) p[i] = 1 << (bd - 1);
    } else {
      if (p[0] < 0) p[0] = p[first];
      for (int i = 1; i < 17; ++i)
        if (p[i] < 0) p[i] = p[i - 1];
    }
    int s = 4;
    for (int k = 0; k < 4; ++k) s += p[9 + k] + p[7 - k];
    S.dc4[pu] = s >> 3;
  }
  for (int i = tid; i < kPuCount * 36; i += 256) {
    (&S.cost4[0][0])[i] = 0;
    (&S.done4[0][0])[i] = 0;
  }
  __syncthreads();
  // SATD of (CU, mode, 8x8 region) items, coarse to fine: 11 seed modes (planar, DC and
  // every 4th angular direction) for every CU, then best-angular +-2, then +-1.  An item
  // index i < 48 names the (CU, region): 0-15 the regions of the 32x32 CU, 16-31 the 4 x 4
  // regions of the 16x16 CUs, 32-47 the 16 8x8 CUs.  A wave evaluates 4 items per MFMA:
  // item (lane & 15) >> 2, 4x4 block lane & 3 of its 8x8 region, row lane >> 4; the region
  // cost is the sum of its four 4x4 Hadamard SATDs ((sum + 1) >> 1 each, HM's 4x4 form; the
  // same scale as the 8x8 transform's (sum + 2) >> 2).
  const int wave = tid >> 6, lane = tid & 63;
  const v4h_t H16 = h16_rows();
  auto eval_q = [&](int slot48, int mode, bool active) {
    const int level = slot48 >> 4, k = slot48 & 15;
    int c, bx, by;
    if (level == 0) {
      c = 0;
      bx = k & 3;
      by = k >> 2;
    } else if (level == 1) {
      c = 1 + (k >> 2);
      bx = k & 1;
      by = (k >> 1) & 1;
    } else {
      c = 5 + k;
      bx = 0;
      by = 0;
    }
    int cx, cy, n, off;
    cu_of(c, &cx, &cy, &n, &off);
    const int lg = n == 32 ? 5 : (n == 16 ? 4 : 3);
    const int16_t* p = S.refs[hv::intra_filter_flag(mode, n) ? 1 : 0] + off;
    const int b4 = lane & 3, row = lane >> 4;
    const int X = bx * 8 + (b4 & 1) * 4, Y = by * 8 + (b4 >> 1) * 4;  // the 4x4 block in the CU
    int pr[4], r[4];
    bool tr;
    hv::intra_pred4(p, n, lg, mode, X, Y, row, S.dc[c], n < 32, maxv, pr, &tr);
    // source samples in the same layout (row `row`, or column `row` when transposed)
    const int s0 = tr ? (cy + Y + 1) * 65 + cx + X + row + 1 : (cy + Y + row + 1) * 65 + cx + X + 1;
    const int sd = tr ? 65 : 1;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = active ? S.ext[s0 + j * sd] - pr[j] : 0;
    int blk = (hadamard_col_sum(H16, r) + 1) >> 1;
    blk += __shfl_xor(blk, 1, 64);
    blk += __shfl_xor(blk, 2, 64);
    if (active && lane < 16 && b4 == 0) {
      atomicAdd(&S.cost[c][mode], blk);
      S.done[c][mode] = 1;
    }
  };
  // 16 items (4x4 PU, mode) per MFMA: item lane & 15, row lane >> 4; prediction from the
  // source references, 4x4 Hadamard SATD
  auto eval4_q = [&](int pu, int mode, bool active) {
    int px, py;
    pu_of(pu, &px, &py);
    const int16_t* p = S.refs4[pu];
    const int row = lane >> 4;
    int pr[4], r[4];
    bool tr;
    hv::intra_pred4(p, 4, 2, mode, 0, 0, row, S.dc4[pu], true, maxv, pr, &tr);
    const int s0 = tr ? (py + 1) * 65 + px + row + 1 : (py + row + 1) * 65 + px + 1;
    const int sd = tr ? 65 : 1;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = active ? S.ext[s0 + j * sd] - pr[j] : 0;
    const int sv = (hadamard_col_sum(H16, r) + 1) >> 1;
    if (active && lane < 16) {
      S.cost4[pu][mode] = sv;
      S.done4[pu][mode] = 1;
    }
  };
  for (int q = wave; q < 11 * 12; q += 4) {  // wave-uniform mode and CU level
    const int si = q / 12;
    eval_q(4 * (q % 12) + ((lane & 15) >> 2), si < 2 ? si : 2 + 4 * (si - 2), true);
  }
  __syncthreads();
  for (int step = 2; step >= 1; step >>= 1) {
    if (tid < kCuCount) {  // best angular so far -> its two neighbours at distance step
      int bm = 2, bc = 0x7FFFFFFF;
      for (int m = 2; m < 35; ++m) {
        const int cst = S.cost[tid][m];
        if (S.done[tid][m] && cst < bc) {
          bc = cst;
          bm = m;
        }
      }
      S.best_mode[tid] = bm;
    }
    __syncthreads();
    // the items of this round, decided before any of them marks its (CU, mode) done
    if (tid < 96) {
      const int slot48 = tid % 48;
      const int level = slot48 >> 4, k = slot48 & 15;
      const int c = level == 0 ? 0 : (level == 1 ? 1 + (k >> 2) : 5 + k);
      const int m = S.best_mode[c] + (tid < 48 ? -step : step);
      S.rmode[tid] = (m >= 2 && m <= 34 && !S.done[c][m]) ? m : -1;
    }
    __syncthreads();
    for (int q = wave; q < 24; q += 4) {
      const int it = 4 * q + ((lane & 15) >> 2);
      const int m = S.rmode[it];
      eval_q(it % 48, m < 0 ? 0 : m, m >= 0);
    }
    __syncthreads();
  }
  __syncthreads();
  const int qp = a.qp[static_cast<size_t>(slot) * g.nctb() + ci];
  const int lam = lambda_satd(qp, bd);
  if (tid < kCuCount) {
    int bm = 0, bc = 0x7FFFFFFF;
    for (int m = 0; m < 35; ++m) {
      if (!S.done[tid][m]) continue;
      const int cst = S.cost[tid][m] + lam * (m < 2 ? 3 : 5);
      if (cst < bc) {
        bc = cst;
        bm = m;
      }
    }
    S.best_mode[tid] = bm;
    S.best_cost[tid] = bc + lam * 4;  // CU overhead: split flag, chroma mode, cbfs
  }
  __syncthreads();
  // 4x4 PUs (PART_NxN candidates): seeds planar, DC and the parent 8x8 CU's best mode
  // +-2 (or the pure directions when it is planar / DC), then +-1 around the best angular
  // (clamped duplicates of one PU write the same value)
  for (int q = wave; nxn_on && q < 5 * kPuCount / 16; q += 4) {
    const int it = 16 * q + (lane & 15);
    const int pu = it % kPuCount, si = it / kPuCount;
    const int m8 = S.best_mode[5 + (pu >> 2)];
    int m;
    if (si < 2) m = si;
    else if (m8 >= 2) m = clampi(m8 + (si - 3) * 2, 2, 34);
    else m = si == 2 ? 10 : (si == 3 ? 26 : 18);
    eval4_q(pu, m, true);
  }
  __syncthreads();
  if (nxn_on && tid < kPuCount) {
    int bm = 2, bc = 0x7FFFFFFF;
    for (int m = 2; m < 35; ++m) {
      const int cst = S.cost4[tid][m];
      if (S.done4[tid][m] && cst < bc) {
        bc = cst;
        bm = m;
      }
    }
    S.best4_mode[tid] = bm;
  }
  __syncthreads();
  if (nxn_on && tid < 2 * kPuCount) {
    const int pu = tid & 63;
    const int m = S.best4_mode[pu] + (tid < 64 ? -1 : 1);
    S.rmode[tid] = (m >= 2 && m <= 34 && !S.done4[pu][m]) ? m : -1;
  }
  __syncthreads();
  for (int q = wave; nxn_on && q < 2 * kPuCount / 16; q += 4) {
    const int it = 16 * q + (lane & 15);
    const int m = S.rmode[it];
    eval4_q(it & 63, m < 0 ? 0 : m, m >= 0);
  }
  __syncthreads();
  if (nxn_on && tid < kPuCount) {
    const int pu = tid;
    int bm = 0, bc = 0x7FFFFFFF;
    for (int m = 0; m < 35; ++m) {
      if (!S.done4[pu][m]) continue;
      const int cst = S.cost4[pu][m] + lam * (m < 2 ? 3 : 5);
      if (cst < bc) {
        bc = cst;
        bm = m;
      }
    }
    S.best4_mode[pu] = bm;
    S.best4_cost[pu] = bc;
  }
  __syncthreads();
  if (tid < 16 && !nxn_on) S.nxn[tid] = 0;
  if (nxn_on && tid < 16) {  // PART_NxN vs PART_2Nx2N per 8x8 CU (NxN: three more PU mode codes, four luma cbfs)
    const int c8 = tid;
    const int cn = S.best4_cost[4 * c8] + S.best4_cost[4 * c8 + 1] + S.best4_cost[4 * c8 + 2] + S.best4_cost[4 * c8 + 3] +
                   lam * 6;
    if (cn < S.best_cost[5 + c8]) {
      S.best_cost[5 + c8] = cn;
      S.nxn[c8] = (1 << 24) | S.best4_mode[4 * c8] | (S.best4_mode[4 * c8 + 1] << 6) | (S.best4_mode[4 * c8 + 2] << 12) |
                  (S.best4_mode[4 * c8 + 3] << 18);
    } else {
      S.nxn[c8] = 0;
    }
  }
  __syncthreads();
  if (a.cand && tid < kCuCount + 16) {
    int* cd = a.cand + (static_cast<size_t>(slot) * g.nctb() + ci) * kCandStride;
    if (tid < kCuCount) {
      cd[tid] = S.best_cost[tid];
      cd[21 + tid] = S.best_mode[tid];
    } else {
      cd[42 + tid - kCuCount] = S.nxn[tid - kCuCount];
    }
  }
  if (tid == 0) {
    int split = 0, c16sum = 0;
    for (int q = 0; q < 4; ++q) {
      int s8 = 0;
      for (int r = 0; r < 4; ++r) s8 += S.best_cost[5 + q * 4 + r];
      const int c16 = S.best_cost[1 + q];
      if (s8 < c16) {
        split |= 1 << (1 + q);
        c16sum += s8;
      } else {
        c16sum += c16;
      }
    }
    if (c16sum < S.best_cost[0]) split |= 1;
    else split = 0;
    CtuInfo* t = a.ctu + static_cast<size_t>(slot) * g.nctb() + ci;
    t->split = static_cast<uint8_t>(split);
    t->qp = static_cast<int8_t>(qp);
    S.best_cost[0] = split;  // broadcast
  }
  __syncthreads();
  if (tid < 16) {
    const int split = S.best_cost[0];
    // granule z-index tid -> the chosen CU covering it
    const int gx = (tid & 1) | ((tid >> 1) & 2), gy = ((tid >> 1) & 1) | ((tid >> 2) & 2);
    const int q = (gx >> 1) + 2 * (gy >> 1);
    int m, lg;
    if (!(split & 1)) {
      m = S.best_mode[0];
      lg = 5;
    } else if (!((split >> (1 + q)) & 1)) {
      m = S.best_mode[1 + q];
      lg = 4;
    } else {
      m = S.best_mode[5 + tid];
      lg = 3;
    }
    CuInfo c{};
    c.pred = hevc::CU_INTRA;
    c.mode = static_cast<uint8_t>(m);
    c.flags = static_cast<uint8_t>((lg - 3) << 1);
    if (lg == 3 && S.nxn[tid]) set_nxn(c, S.nxn[tid]);
    a.cu[(static_cast<size_t>(slot) * g.nctb() + ci) * 16 + tid] = c;
  }
}

// ============================================================== closed-loop reconstruction
constexpr int kHevcIntraWaves = 8;
constexpr int RT = 65;  // recon tile stride (x = -1 .. 63)
constexpr int CT2 = 33; // chroma recon tile stride (x = -1 .. 31)

struct ReconShared {
  uint16_t rt[33 * RT];          // luma: row 0 = y -1 (x -1..63), rows 1..32 = y 0..31, col 0 = x -1
  uint16_t rc[2][17 * CT2];      // chroma tiles, same layout (x -1..31, y -1..15)
  int p[129], q[129];            // reference arrays (unfiltered, filtered)
  int R[32 * 32], S[32 * 32];    // residual / transform scratch
  uint16_t pred[32 * 32];
  int saved_x, saved_ry;            // block whose right column saved_y / saved_c hold
  uint16_t saved_y[32];
  uint16_t saved_c[2][16];
};

// reconstruct one CU component: refs from the LDS tile, predict, transform/quantise, store
template <bool LUMA>
__device__ __forceinline__ bool recon_block(const HevcIntraArgs& a, ReconShared& S, const hv::DctLds& D, int slot,
                                            int comp, int rx, int ry, int cx, int cy, int log2n, int mode, int zc, int qpp,
                                            bool dst = false) {
  const HevcGeom& g = a.g;
  const int lane = lane_id();
  const int n = 1 << log2n;
  const int bd = a.bd, maxv = (1 << bd) - 1;
  const int sc = LUMA ? 0 : 1;  // component -> luma coordinate shift
  const int stride = LUMA ? RT : CT2;
  uint16_t* tile = LUMA ? S.rt : S.rc[comp - 1];
  // 1. reference samples (availability from the luma granule of each sample)
  hv::build_refs(S.p, n, bd,
                 [&](int i) {
                   int x, y;
                   ref_pos(i, n, cx, cy, &x, &y);
                   return nb_avail(x << sc, y << sc, zc, rx, ry, g.wctb, g.hctb, a.ctu64);
                 },
                 [&](int i) {
                   int x, y;
                   ref_pos(i, n, cx, cy, &x, &y);
                   // ctu64: the column below-left (x -1, y >= the block height) is kept in the
                   // tile's last column, which the block itself never uses
                   const int lim = LUMA ? 32 : 16;
                   const bool below = y >= lim;
                   return static_cast<int>(tile[((below ? y - lim : y) + 1) * stride + (below ? stride - 1 : x + 1)]);
                 });
  const int* p = S.p;
  if (LUMA && hv::intra_filter_flag(mode, n)) {
    hv::filter_refs(S.p, S.q, n, bd, true);
    p = S.q;
  }
  const int dc = hv::intra_dc(p, n, log2n);
  // 2. prediction and residual
  const uint16_t* src = (LUMA ? a.src_y : (comp == 1 ? a.src_u : a.src_v)) + slot * (LUMA ? g.ysize() : g.csize());
  const int pw = LUMA ? g.W : g.W / 2;
  const int X0 = (rx * 32 >> sc) + cx, Y0 = (ry * 32 >> sc) + cy;
  for (int i = lane; i < n * n; i += 64) {
    const int x = i & (n - 1), y = i >> log2n;
    const int pv = hv::intra_pred_sample(p, n, log2n, mode, x, y, dc, LUMA && n < 32, maxv);
    S.pred[i] = static_cast<uint16_t>(pv);
    S.R[y * 32 + x] = static_cast<int>(src[static_cast<size_t>(Y0 + y) * pw + X0 + x]) - pv;
  }
  wave_sync();
  // 3. transform / quantisation / reconstruction
  int16_t* lev = (LUMA ? a.coef_y : (comp == 1 ? a.coef_u : a.coef_v)) + slot * (LUMA ? g.ysize() : g.csize()) +
                 static_cast<size_t>(Y0) * pw + X0;
  hv::TqParams tp{log2n, bd, qpp, true, dst, a.sdh ? hv::tu_scan_idx(true, LUMA, log2n, mode) : -1};
  tp.mfma = false;
  const bool nz = hv::transform_quant_block(D, S.R, S.S, lev, pw, tp);
  uint16_t* rec = (LUMA ? a.rec_y : (comp == 1 ? a.rec_u : a.rec_v)) + slot * (LUMA ? g.ysize() : g.csize());
  for (int i = lane; i < n * n; i += 64) {
    const int x = i & (n - 1), y = i >> log2n;
    int v = S.pred[i] + (nz ? S.R[y * 32 + x] : 0);
    v = v < 0 ? 0 : (v > maxv ? maxv : v);
    tile[(cy + y + 1) * stride + cx + x + 1] = static_cast<uint16_t>(v);
    rec[static_cast<size_t>(Y0 + y) * pw + X0 + x] = static_cast<uint16_t>(v);
  }
  wave_sync();
  return nz;
}

// (inlined at its single call site: its LDS structures stay ds_ addressed, no call frame)
// One colour component per workgroup (comp = blockIdx.y): the three planes of a picture are
// independent intra wavefronts (no cross-component prediction in Main / Main 10), so a slot's
// luma, Cb and Cr run side by side on three CUs instead of one after another in one wave.
__device__ __forceinline__ void hevc_recon_ctb(const HevcIntraArgs& a, ReconShared& S, const hv::DctLds& D, int slot,
                                               int rx, int ry, int run, int comp) {
  const HevcGeom& g = a.g;
  const int lane = lane_id();
  const int X0 = rx * 32, Y0 = ry * 32;
  const size_t cb = static_cast<size_t>(slot) * g.nctb() + ry * g.wctb + rx;
  const bool luma = comp == 0;
  const int c1 = comp - 1;
  // the component's plane, its width and the CTB's extent in it
  const uint16_t* rp = luma ? a.rec_y + slot * g.ysize() : (comp == 1 ? a.rec_u : a.rec_v) + slot * g.csize();
  const int pw = luma ? g.W : g.W / 2;
  const int n = luma ? 32 : 16, st = luma ? RT : CT2;
  const int x0 = luma ? X0 : X0 / 2, y0 = luma ? Y0 : Y0 / 2;
  uint16_t* tile = luma ? S.rt : S.rc[c1];
  const bool same_left = S.saved_x == rx - 1 && S.saved_ry == ry;
  // ---- stage the neighbourhood: row above (x -1 .. 2n - 1), left column, and (P) the CTB interior
  for (int i = lane; i < 2 * n + 1; i += 64) {
    const int x = x0 - 1 + i;
    tile[i] = (ry > 0 && x >= 0 && x < pw) ? rp[static_cast<size_t>(y0 - 1) * pw + x] : 0;
  }
  if (lane < n) {
    uint16_t v = 0;
    if (rx > 0) v = same_left ? (luma ? S.saved_y[lane] : S.saved_c[c1][lane]) : rp[static_cast<size_t>(y0 + lane) * pw + x0 - 1];
    tile[(lane + 1) * st] = v;
  }
  if (a.ctu64 && !((rx | ry) & 1) && rx > 0 && ry + 1 < g.hctb && lane < n) {
    // the top-left block of a CTU: the left column below it (x -1, y n .. 2n - 1, in the previous
    // CTU's bottom-right block) into the tile's last column (x 2n - 1 of rows 0 .. n - 1: right of
    // the block, never referenced by it)
    tile[(lane + 1) * st + st - 1] = rp[static_cast<size_t>(y0 + n + lane) * pw + x0 - 1];
  }
  if (run == 2) {  // P picture: inter CUs of this CTB are already reconstructed
    for (int i = lane; i < n * n; i += 64) {
      const int y = i / n, x = i - y * n;
      tile[(y + 1) * st + x + 1] = rp[static_cast<size_t>(y0 + y) * pw + x0 + x];
    }
  }
  wave_sync();
  const int split = __builtin_amdgcn_readfirstlane(a.ctu[cb].split);
  const int qpy = a.qp[cb];
  const int off = 6 * (a.bd - 8);
  const int qpl = qpy + off;
  const int qpc = hevc::chroma_qp_map(clampi(qpy, -off, 57)) + off;
  // ---- CUs in z-order
  for (int k = 0; k < 16;) {
    const int q = k >> 2;
    int log2n;
    if (!(split & 1)) log2n = 5;
    else if (!((split >> (1 + q)) & 1)) log2n = 4;
    else log2n = 3;
    const int step = 1 << (2 * (log2n - 3));  // granules covered
    CuInfo* cu = a.cu + cb * 16 + k;
    const int pred = __builtin_amdgcn_readfirstlane(cu->pred);
    if (run == 1 || pred == hevc::CU_INTRA) {
      const int mode = __builtin_amdgcn_readfirstlane(cu->mode);
      const int gx = (k & 1) | ((k >> 1) & 2), gy = ((k >> 1) & 1) | ((k >> 2) & 2);
      const int cx = gx * 8, cy = gy * 8;
      bool nz = false;
      if (!luma) {
        nz = recon_block<false>(a, S, D, slot, comp, rx, ry, cx / 2, cy / 2, log2n - 1, mode, 4 * k, qpc);
      } else if (log2n == 3 && (__builtin_amdgcn_readfirstlane(cu->flags) & 8)) {
        // PART_NxN: four 4x4 luma PUs in z-order, DST, each predicted from the previous ones
        const uint32_t pm = __builtin_amdgcn_readfirstlane(*reinterpret_cast<const uint32_t*>(cu->mv));
        for (int j = 0; j < 4; ++j)
          nz |= recon_block<true>(a, S, D, slot, 0, rx, ry, cx + (j & 1) * 4, cy + (j >> 1) * 4, 2,
                                  static_cast<int>((pm >> (8 * j)) & 255u), 4 * k + j, qpl, true);
      } else {
        nz = recon_block<true>(a, S, D, slot, 0, rx, ry, cx, cy, log2n, mode, 4 * k, qpl);
      }
      if (lane < step) {
        // cbf bit `comp` of the granule's record (byte 2 of its first word): the three
        // component workgroups set their own bits of the same byte, so one atomic each
        CuInfo* c = a.cu + cb * 16 + k + lane;
        unsigned int* w0 = reinterpret_cast<unsigned int*>(c);
        const unsigned int bit = 1u << (16 + comp);
        if (nz) atomicOr(w0, bit);
        else atomicAnd(w0, ~bit);
        if (luma) c->pred = hevc::CU_INTRA;
      }
    }
    k += step;
  }
  // ---- keep this CTB's right column for the next CTB of the row
  if (lane < n) {
    const uint16_t v = tile[(lane + 1) * st + n];
    if (luma) S.saved_y[lane] = v;
    else S.saved_c[c1][lane] = v;
  }
  if (lane == 0) {
    S.saved_x = rx;
    S.saved_ry = ry;
  }
  // the next blocks of a CTU read this one's samples back from memory (ctu64: the row above
  // of the lower blocks, a left column across CTUs): this wave's stores before its loads
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  wave_sync();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__global__ __launch_bounds__(64 * kHevcIntraWaves) void hevc_intra_recon(HevcIntraArgs a) {
  __shared__ ReconShared SS[kHevcIntraWaves];
  __shared__ hv::DctLds D;
  __shared__ int prog[kMaxRows];
  const HevcGeom& g = a.g;
  const int slot = blockIdx.x, comp = blockIdx.y;
  const int run = a.run[slot];
  if (run == 0) return;
  hv::dct_lds_init(D);
  for (int i = threadIdx.x; i < g.hctb; i += blockDim.x) prog[i] = 0;
  const int w = wave_id();
  if (lane_id() == 0) {
    SS[w].saved_x = -2;
    SS[w].saved_ry = -1;
  }
  __syncthreads();
  ReconShared& S = SS[w];
  // units in wavefront order (one unit row per wave, the unit above-right done first): 32x32
  // CTBs, or (ctu64) 64x64 CTUs whose four 32x32 blocks follow in z-order
  const int c64 = a.ctu64 ? 1 : 0;
  const int wu = (g.wctb + c64) >> c64, hu = (g.hctb + c64) >> c64, nq = c64 ? 4 : 1;
  // a block's "has intra CUs" flag (P pictures): any of its 16 granule records is intra
  auto block_work = [&](int bx, int by) {
    const size_t cb = (static_cast<size_t>(slot) * g.nctb() + by * g.wctb + bx) * 16;
    return __ballot(lane_id() < 16 && a.cu[cb + lane_id()].pred == hevc::CU_INTRA) != 0;
  };
  for (int y = w; y < hu; y += kHevcIntraWaves) {
    if (run == 1) {  // I picture: every unit
      for (int x = 0; x < wu; ++x) {
        if (y > 0) row_wait(prog, y - 1, min(x + 2, wu), a.err);
        for (int q = 0; q < nq; ++q) {
          const int bx = (x << c64) + (q & 1), by = (y << c64) + (q >> 1);
          if (bx >= g.wctb || by >= g.hctb) continue;
          hevc_recon_ctb(a, S, D, slot, bx, by, run, comp);
        }
        row_publish(prog, y, x + 1);
      }
      continue;
    }
    // P / B picture: the units of the row with intra CUs, 64 at a time (one lane per unit, its
    // blocks' 16 records each); the others were fully reconstructed by hevc_inter and need
    // neither a wait nor staging (the next block then reads its left column from memory)
    for (int x0 = 0; x0 < wu; x0 += 64) {
      const int xl = x0 + lane_id();
      bool any = false;
      if (xl < wu)
        for (int q = 0; q < nq && !any; ++q) {
          const int bx = (xl << c64) + (q & 1), by = (y << c64) + (q >> 1);
          if (bx >= g.wctb || by >= g.hctb) continue;
          const CuInfo* c = a.cu + (static_cast<size_t>(slot) * g.nctb() + by * g.wctb + bx) * 16;
          for (int k = 0; k < 16 && !any; ++k) any = c[k].pred == hevc::CU_INTRA;
        }
      unsigned long long mask = __ballot(any);
      while (mask) {
        const int x = x0 + __builtin_ctzll(mask);
        mask &= mask - 1;
        if (x > 0) row_publish(prog, y, x);  // the units before x in this row are final
        if (y > 0) row_wait(prog, y - 1, min(x + 2, wu), a.err);
        for (int q = 0; q < nq; ++q) {
          const int bx = (x << c64) + (q & 1), by = (y << c64) + (q >> 1);
          if (bx >= g.wctb || by >= g.hctb) continue;
          if (block_work(bx, by)) {
            hevc_recon_ctb(a, S, D, slot, bx, by, run, comp);
          } else {
            if (lane_id() == 0) S.saved_x = -2;
            wave_sync();
          }
        }
        row_publish(prog, y, x + 1);
      }
    }
    row_publish(prog, y, wu);
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

static HevcIntraArgs make_intra_args(int B, int W, int H, const uint16_t* sy, const uint16_t* su, const uint16_t* sv,
                                     uint16_t* ry, uint16_t* ru, uint16_t* rv, void* ctu, void* cu, int16_t* cy,
                                     int16_t* cu_, int16_t* cv, const int* qp, const int8_t* run, int* cand, int bd,
                                     int* err, int sdh) {
  HevcIntraArgs a;
  a.g = HevcGeom{B, W, H, W / 32, H / 32};
  a.src_y = sy;
  a.src_u = su;
  a.src_v = sv;
  a.rec_y = ry;
  a.rec_u = ru;
  a.rec_v = rv;
  a.ctu = static_cast<CtuInfo*>(ctu);
  a.cu = static_cast<CuInfo*>(cu);
  a.coef_y = cy;
  a.coef_u = cu_;
  a.coef_v = cv;
  a.qp = qp;
  a.run = run;
  a.cand = cand;
  a.bd = bd;
  a.err = err;
  a.sdh = sdh;
  a.nxn_in_p = 0;
  a.ctb_mask = nullptr;
  a.ctu64 = 0;
  return a;
}

extern "C" void mivc_launch_hevc_intra(int B, int W, int H, const uint16_t* sy, const uint16_t* su, const uint16_t* sv,
                                       uint16_t* ry, uint16_t* ru, uint16_t* rv, void* ctu, void* cu, int16_t* cy,
                                       int16_t* cu_, int16_t* cv, const int* qp, const int8_t* run, int* cand, int bd,
                                       int analyze, int recon, int* err, int sdh, const uint8_t* ctb_mask,
                                       void* stream, int ctu64) {
  HevcIntraArgs a = make_intra_args(B, W, H, sy, su, sv, ry, ru, rv, ctu, cu, cy, cu_, cv, qp, run, cand, bd, err, sdh);
  a.ctb_mask = ctb_mask;
  a.ctu64 = ctu64;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (analyze) hipLaunchKernelGGL(hevc_intra_analyze, dim3(a.g.nctb(), B), dim3(256), 0, s, a);
  if (recon) hipLaunchKernelGGL(hevc_intra_recon, dim3(B, 3), dim3(64 * kHevcIntraWaves), 0, s, a);
}
