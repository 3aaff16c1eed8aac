// HEVC P pictures on gfx950.
//
// Motion comes from the batched motion-estimation kernel (me.hip) run on 8-bit
// proxies of the source and the reference reconstruction (one vector per 16x16
// block).  Here:
//
// * hevc_p_decide (grid = CTBs x slots, one wave): per 16x16 quadrant, inter (ME
//   cost) versus the best intra choice of the open-loop analysis (16x16 or four
//   8x8); four inter quadrants with one vector become a 32x32 inter CU.  Writes the
//   CTB split and the CU records (the CABAC writer turns zero-residual CUs whose
//   vector equals a merge candidate into skip CUs).
// * hevc_inter_cu (grid = CTBs*4 x slots, one wave per 16x16 quadrant or 32x32
//   CU): normative HEVC motion compensation (8-tap luma, 4-tap chroma, separable
//   through LDS, default weighted prediction), transform / quantisation with the
//   inter rounding offset, reconstruction.  No dependency between CUs: fully
//   parallel; the intra CUs of the picture are then coded by hevc_intra_recon.
#include "hevc_common.h"

namespace mivc {
namespace gpu {

using hevc::CtuInfo;
using hevc::CuInfo;

struct HevcInterArgs {
  HevcGeom g;
  const uint16_t *src_y, *src_u, *src_v;
  const uint16_t *ref_y, *ref_u, *ref_v;
  uint16_t *rec_y, *rec_u, *rec_v;
  CtuInfo* ctu;
  CuInfo* cu;
  int16_t *coef_y, *coef_u, *coef_v;
  const int* qp;          // [B, nctb] QpY per CTB
  const int8_t* run;
  const int* cand;       // [B, nctb, kCandStride] intra analysis: best cost / mode per CU, NxN PUs
  const int16_t* mv;     // [B, nmb16, 2] quarter-sample vectors per 16x16 block (P pictures)
  const int16_t* mvb;    // [B, nmb16, 4] B pictures: (L0 x, y, L1 x, y) per 16x16 block, or null
  const uint8_t* dirb;   // [B, nmb16] B pictures: CuDir per 16x16 block
  const uint16_t *ref1_y, *ref1_u, *ref1_v;  // RefPicList1[0] (B pictures)
  const int* me_cost;    // [B, nmb16] (8-bit proxy units)
  int bd;
  int tu_split;          // inter CUs may code their residual as four quarter TUs (RD choice)
  int sdh;               // sign data hiding in the quantiser
  int intra_bias;        // lambda multiples added to the open-loop intra costs of P pictures
  // explicit weighted prediction of P pictures (x265 --weightp; pred_weight_table with
  // log2 denominators kWpLog2 for luma and chroma): [B][6] = weight, offset (8-bit units) of
  // Y, Cb, Cr; weight 0 = the slot's picture is not weighted.  Null: default weighting.
  const int16_t* wp;
  // x265 --ref: RefPicList0[1 ..] reconstructions of a P picture (a motion's direction byte in
  // dirb carries its list-0 refIdx in bits 2-3; the CU records take it in pad[0]); explicit
  // weights apply to RefPicList0[0] only
  const uint16_t *xref_y[3], *xref_u[3], *xref_v[3];
  // 8x8 inter CUs (P pictures, x265's minimum CU): [B, nmb16, 4, 2] per-quadrant vectors of
  // each 16x16 block (p_part8x8 in its HEVC form; all equal = no split); null: 16x16 / 32x32 only
  const int16_t* mv8;
};

// plane c of RefPicList0[r] (constant indices only: no scratch)
__device__ __forceinline__ const uint16_t* l0_plane(const HevcInterArgs& a, int c, int r) {
  const uint16_t* const* x = c == 0 ? a.xref_y : (c == 1 ? a.xref_u : a.xref_v);
  return r == 0 ? (c == 0 ? a.ref_y : (c == 1 ? a.ref_u : a.ref_v)) : (r == 1 ? x[0] : (r == 2 ? x[1] : x[2]));
}

constexpr int kWpLog2 = 6;

__device__ __forceinline__ int lambda_satd_i(int qp, int bd) {
  return static_cast<int>(0.755f * exp2f((qp - 12) / 6.0f) * static_cast<float>(1 << (bd - 8)) + 0.5f);
}

// ============================================================== decision
__global__ __launch_bounds__(64) void hevc_p_decide(HevcInterArgs a) {
  const HevcGeom& g = a.g;
  const int ci = blockIdx.x, slot = blockIdx.y;
  if (a.run[slot] != 2) return;
  const int lane = threadIdx.x;
  const int rx = ci % g.wctb, ry = ci / g.wctb;
  const size_t cb = static_cast<size_t>(slot) * g.nctb() + ci;
  const int* cd = a.cand + cb * kCandStride;
  const int wmb = g.W / 16, nmb = wmb * (g.H / 16);
  const int qp = a.qp[cb];
  const int lam = lambda_satd_i(qp, a.bd);
  __shared__ int s_inter[4], s_mvx[4], s_mvy[4], s_mv1x[4], s_mv1y[4], s_dir[4], s_split8[4], s_intra[4], s_isplit[4];
  __shared__ uint32_t s_mv8[4][4];
  __shared__ int s_split;
  if (lane < 4) {
    const int q = lane;
    const int mb = (ry * 2 + (q >> 1)) * wmb + rx * 2 + (q & 1);
    const size_t o = static_cast<size_t>(slot) * nmb + mb;
    const int inter = (a.me_cost[o] << (a.bd - 8)) + lam * 3;
    int s8 = 0;
    for (int r = 0; r < 4; ++r) s8 += cd[5 + q * 4 + r];
    const int c16 = cd[1 + q];
    s_split8[q] = s8 < c16;
    s_intra[q] = (s8 < c16 ? s8 : c16) + lam * a.intra_bias;
    s_inter[q] = inter;
    if (a.dirb) {
      const int16_t* m = a.mvb + o * 4;
      s_mvx[q] = m[0];
      s_mvy[q] = m[1];
      s_mv1x[q] = m[2];
      s_mv1y[q] = m[3];
      s_dir[q] = a.dirb[o];
    } else {
      s_mvx[q] = a.mv[o * 2];
      s_mvy[q] = a.mv[o * 2 + 1];
      s_mv1x[q] = s_mv1y[q] = 0;
      s_dir[q] = hevc::DIR_L0;
    }
    // an inter quadrant split into four 8x8 inter CUs: RefPicList0[0] list-0 motion whose four
    // quadrant vectors differ
    s_isplit[q] = 0;
    if (a.mv8 && s_dir[q] == hevc::DIR_L0) {
      const uint32_t* m8 = reinterpret_cast<const uint32_t*>(a.mv8 + o * 8);
      for (int k = 0; k < 4; ++k) s_mv8[q][k] = m8[k];
      s_isplit[q] = m8[0] != m8[1] || m8[0] != m8[2] || m8[0] != m8[3];
    }
  }
  __syncthreads();
  if (lane == 0) {
    int n_inter = 0, icost = 0, tcost = 0;
    for (int q = 0; q < 4; ++q) {
      const bool inter = s_inter[q] < s_intra[q];
      n_inter += inter;
      icost += s_intra[q];
      tcost += inter ? s_inter[q] : s_intra[q];
    }
    int split;
    if (n_inter == 0) {
      // the analysis' own 32-vs-16 choice
      split = icost < cd[0] ? 1 : 0;
      for (int q = 0; q < 4; ++q) split |= (split & 1) && s_split8[q] ? 1 << (1 + q) : 0;
      for (int q = 0; q < 4; ++q) s_inter[q] = 0x7FFFFFFF;  // mark intra
    } else {
      bool same = n_inter == 4 && !s_isplit[0];
      for (int q = 1; q < 4; ++q)
        same = same && s_dir[q] == s_dir[0] && s_mvx[q] == s_mvx[0] && s_mvy[q] == s_mvy[0] && s_mv1x[q] == s_mv1x[0] &&
               s_mv1y[q] == s_mv1y[0] && !s_isplit[q];
      split = same ? 0 : 1;
      for (int q = 0; q < 4; ++q) {
        const bool inter = s_inter[q] < s_intra[q];
        if (!inter && s_split8[q]) split |= 1 << (1 + q);
        if (inter && s_isplit[q]) split |= 1 << (1 + q);
        if (!inter) s_inter[q] = 0x7FFFFFFF;
      }
    }
    s_split = split;
    a.ctu[cb].split = static_cast<uint8_t>(split);
    a.ctu[cb].qp = static_cast<int8_t>(qp);
  }
  __syncthreads();
  if (lane < 16) {
    const int k = lane;
    const int gx = (k & 1) | ((k >> 1) & 2), gy = ((k >> 1) & 1) | ((k >> 2) & 2);
    const int q = (gx >> 1) + 2 * (gy >> 1);
    const int split = s_split;
    CuInfo c{};
    int lg;
    if (!(split & 1)) lg = 5;
    else if (!((split >> (1 + q)) & 1)) lg = 4;
    else lg = 3;
    c.flags = static_cast<uint8_t>((lg - 3) << 1);
    if (s_inter[q] != 0x7FFFFFFF) {
      c.pred = hevc::CU_INTER;
      c.mv[0] = static_cast<int16_t>(s_mvx[q]);
      c.mv[1] = static_cast<int16_t>(s_mvy[q]);
      if (lg == 3) {  // an 8x8 inter CU: its quadrant's vector of the 16x16 block
        const uint32_t w = s_mv8[q][(gx & 1) | ((gy & 1) << 1)];
        c.mv[0] = static_cast<int16_t>(w & 0xFFFFu);
        c.mv[1] = static_cast<int16_t>(w >> 16);
      }
      c.mv1[0] = static_cast<int16_t>(s_mv1x[q]);
      c.mv1[1] = static_cast<int16_t>(s_mv1y[q]);
      c.dir = static_cast<uint8_t>(s_dir[q] & 3);
      c.pad[0] = static_cast<uint8_t>((s_dir[q] >> 2) & 3);  // list-0 refIdx
    } else {
      c.pred = hevc::CU_INTRA;
      const int idx = lg == 5 ? 0 : (lg == 4 ? 1 + q : 5 + k);
      c.mode = static_cast<uint8_t>(cd[21 + idx]);
      if (lg == 3 && cd[42 + k]) set_nxn(c, cd[42 + k]);
    }
    a.cu[cb * 16 + k] = c;
  }
}

// ============================================================== inter reconstruction
constexpr int kLumaTapsD[4][8] = {{0, 0, 0, 64, 0, 0, 0, 0},
                                  {-1, 4, -10, 58, 17, -5, 1, 0},
                                  {-1, 4, -11, 40, 40, -11, 4, -1},
                                  {0, 1, -5, 17, 58, -10, 4, -1}};
constexpr int kChromaTapsD[8][4] = {{0, 64, 0, 0},    {-2, 58, 10, -2}, {-4, 54, 16, -2}, {-6, 46, 28, -4},
                                    {-4, 36, 36, -4}, {-4, 28, 46, -6}, {-2, 16, 54, -4}, {-2, 10, 58, -2}};

struct InterShared {
  uint16_t win[39 * 39];  // reference window (n + 7)^2
  int tmp[39 * 32];       // horizontal pass
  int R[32 * 32], S[32 * 32];
  int R2[32 * 32];        // luma residual / reconstruction of the quarter-TU alternative
  int16_t lev2[32 * 32];  // its levels
  uint16_t pred[32 * 32];
};

// The default instance's LDS (15.8 KB with the DCT matrix instead of 26.5 KB: 10 workgroups
// per CU instead of 6): the motion-compensation window and horizontal pass live only until
// the residual is formed, the transform scratch S only after, so they share storage; the
// 16-bit intermediates (horizontal pass, the list-0 prediction of bi-prediction) are what
// the standard bounds them to (8.5.3.3.3: 14-bit predSamples, 16-bit first stage)
struct InterSharedLean {
  union {
    struct {
      uint16_t win[39 * 39];
      int16_t tmp[39 * 32];
    };
    int S[32 * 32];
  };
  int R[32 * 32];
  int16_t R2[32 * 32];  // list-0 prediction samples of a bi-predicted block
  uint16_t pred[32 * 32];
};

// rate proxy of a block's levels (bits): ~3 + 2 log2|l| per non-zero level (wave reduction)
__device__ __forceinline__ int level_bits(const int16_t* lev, int stride, int n) {
  int b = 0;
  for (int i = lane_id(); i < n * n; i += 64) {
    const int v = lev[(i / n) * stride + i % n];
    const int m = v < 0 ? -v : v;
    if (m) b += 3 + 2 * (31 - __builtin_clz(m));
  }
  return sum64(b);
}

// SSD of clip(pred + R) against the source block (wave reduction; 64-bit: 32x32 at 10 bits)
template <typename SH>
__device__ __forceinline__ long long recon_ssd(const SH& S, const int* R, const uint16_t* src, int pw, int bx,
                                               int by, int n, int maxv) {
  long long e = 0;
  for (int i = lane_id(); i < n * n; i += 64) {
    const int y = i / n, x = i - y * n;
    int v = S.pred[i] + R[y * 32 + x];
    v = v < 0 ? 0 : (v > maxv ? maxv : v);
    const int d = static_cast<int>(src[static_cast<size_t>(by + y) * pw + bx + x]) - v;
    e += d * d;
  }
  const int lo = static_cast<int>(e & 0x3FFFFFFF), hi = static_cast<int>(e >> 30);
  return (static_cast<long long>(sum64(hi)) << 30) + sum64(lo);
}

// motion-compensated prediction samples predSamplesLX (14-bit intermediate, 8.5.3.3.3
// fractional interpolation) of one n x n block of a component into dst[y * n + x]
template <int NT, typename SH, typename DT>
__device__ __forceinline__ void mc_inter(SH& S, const uint16_t* ref, int pw, int ph, int bx, int by, int n,
                                         int mvx, int mvy, int bd, DT* dst) {
  const int lane = lane_id();
  const int fb = NT == 8 ? 2 : 3;  // fraction bits
  const int half = NT / 2 - 1;     // taps before the sample
  const int fx = mvx & ((1 << fb) - 1), fy = mvy & ((1 << fb) - 1);
  const int ix = bx + (mvx >> fb) - half, iy = by + (mvy >> fb) - half;
  const int wn = n + NT - 1;
  for (int i = lane; i < wn * wn; i += 64) {
    const int r = i / wn, c = i - r * wn;
    const int x = clampi(ix + c, 0, pw - 1), y = clampi(iy + r, 0, ph - 1);
    S.win[r * wn + c] = ref[static_cast<size_t>(y) * pw + x];
  }
  wave_sync();
  const int sh1 = bd - 8 < 4 ? bd - 8 : 4;
  const int wsh = 14 - bd;
  auto tap = [&](int f, int k) { return NT == 8 ? kLumaTapsD[f][k] : kChromaTapsD[f][k]; };
  if (fx != 0 && fy != 0) {  // separable: horizontal pass over n + NT - 1 rows
    for (int i = lane; i < wn * n; i += 64) {
      const int r = i / n, x = i - r * n;
      int s = 0;
#pragma unroll
      for (int k = 0; k < NT; ++k) s += tap(fx, k) * S.win[r * wn + x + k];
      S.tmp[r * 32 + x] = static_cast<std::remove_reference_t<decltype(S.tmp[0])>>(s >> sh1);
    }
    wave_sync();
  }
  for (int i = lane; i < n * n; i += 64) {
    const int y = i / n, x = i - y * n;
    int v;
    if (fx == 0 && fy == 0) {
      v = static_cast<int>(S.win[(y + half) * wn + x + half]) << wsh;
    } else if (fy == 0) {
      int s = 0;
#pragma unroll
      for (int k = 0; k < NT; ++k) s += tap(fx, k) * S.win[(y + half) * wn + x + k];
      v = s >> sh1;
    } else if (fx == 0) {
      int s = 0;
#pragma unroll
      for (int k = 0; k < NT; ++k) s += tap(fy, k) * S.win[(y + k) * wn + x + half];
      v = s >> sh1;
    } else {
      int s = 0;
#pragma unroll
      for (int k = 0; k < NT; ++k) s += tap(fy, k) * S.tmp[(y + k) * 32 + x];
      v = s >> 6;
    }
    dst[i] = static_cast<DT>(v);
  }
  wave_sync();
}

// prediction of one n x n block of a component into S.pred: default weighted sample
// prediction (8.5.3.3.4.2) of one list, or the average of both (bi-prediction)
template <int NT, typename SH>
__device__ __forceinline__ void mc_block(SH& S, const uint16_t* ref0, const uint16_t* ref1, int pw, int ph,
                                         int bx, int by, int n, int dir, int mvx, int mvy, int mv1x, int mv1y, int bd,
                                         int ww = 0, int wo = 0) {
  const int lane = lane_id();
  const int maxv = (1 << bd) - 1;
  if (dir == hevc::DIR_BI) {
    mc_inter<NT>(S, ref0, pw, ph, bx, by, n, mvx, mvy, bd, S.R2);
    mc_inter<NT>(S, ref1, pw, ph, bx, by, n, mv1x, mv1y, bd, S.R);
    const int sh2 = 15 - bd, off2 = 1 << (sh2 - 1);
    for (int i = lane; i < n * n; i += 64) {
      const int v = (S.R2[i] + S.R[i] + off2) >> sh2;
      S.pred[i] = static_cast<uint16_t>(v < 0 ? 0 : (v > maxv ? maxv : v));
    }
  } else {
    const bool l1 = dir == hevc::DIR_L1;
    mc_inter<NT>(S, l1 ? ref1 : ref0, pw, ph, bx, by, n, l1 ? mv1x : mvx, l1 ? mv1y : mvy, bd, S.R);
    if (ww) {  // explicit weighted sample prediction, uni-directional (8.5.3.3.4.3)
      const int lwd = kWpLog2 + 14 - bd, rnd = 1 << (lwd - 1), o = wo * (1 << (bd - 8));
      for (int i = lane; i < n * n; i += 64) {
        const int v = ((S.R[i] * ww + rnd) >> lwd) + o;
        S.pred[i] = static_cast<uint16_t>(v < 0 ? 0 : (v > maxv ? maxv : v));
      }
    } else {
      const int wsh = 14 - bd, woff = 1 << (wsh - 1);
      for (int i = lane; i < n * n; i += 64) {
        const int v = (S.R[i] + woff) >> wsh;
        S.pred[i] = static_cast<uint16_t>(v < 0 ? 0 : (v > maxv ? maxv : v));
      }
    }
  }
  wave_sync();
}

// TSPLIT: the instance with the residual-quadtree choice (its register footprint stays out of
// the default instance)
template <bool TSPLIT>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3, 8))) void hevc_inter_cu(HevcInterArgs a) {
  __shared__ typename std::conditional<TSPLIT, InterShared, InterSharedLean>::type S;
  __shared__ hv::DctLds D;
  const HevcGeom& g = a.g;
  const int task = blockIdx.x, slot = blockIdx.y;
  if (a.run[slot] != 2) return;
  const int ci = task >> 2, q = task & 3;
  const size_t cb = static_cast<size_t>(slot) * g.nctb() + ci;
  const int kq = q * 4;  // z-index of the quadrant's first granule
  CuInfo* cu = a.cu + cb * 16;
  const int pred = cu[kq].pred;
  const int lg = 3 + ((cu[kq].flags >> 1) & 3);
  if (pred != hevc::CU_INTER) return;
  if (lg == 5 && q != 0) return;  // the 32x32 CU is handled by quadrant 0
  hv::dct_lds_init(D);
  __syncthreads();
  const int lane = lane_id();
  const int n = 1 << lg;
  const int rx = ci % g.wctb, ry = ci / g.wctb;
  const int bd = a.bd, maxv = (1 << bd) - 1;
  const int qpy = a.qp[cb], off = 6 * (bd - 8);
  const int qpl = qpy + off, qpc = hevc::chroma_qp_map(clampi(qpy, -off, 57)) + off;
  // a quadrant split into 8x8 inter CUs (x265's minimum CU) codes them one after another
  const int ncu = lg == 3 ? 4 : 1;
  for (int j = 0; j < ncu; ++j) {
  const int kc = kq + j;  // the CU's first granule (z-order)
  const int X0 = rx * 32 + (lg == 5 ? 0 : (q & 1) * 16 + (lg == 3 ? (j & 1) * 8 : 0));
  const int Y0 = ry * 32 + (lg == 5 ? 0 : (q >> 1) * 16 + (lg == 3 ? (j >> 1) * 8 : 0));
  const int mvx = cu[kc].mv[0], mvy = cu[kc].mv[1], mv1x = cu[kc].mv1[0], mv1y = cu[kc].mv1[1];
  const int dir = hevc::cu_dir(cu[kc]);
  const int r0 = cu[kc].pad[0] & 3;  // list-0 refIdx
  // residual quadtree: the luma residual is transformed both as one TU and as four quarter
  // TUs; the cheaper by SSD + lambda * (level-bit proxy + TU overhead) wins, and chroma
  // follows the chosen structure (max_transform_hierarchy_depth_inter 1; 16x16+ CUs)
  int cbfq[4] = {0, 0, 0, 0};  // per quarter: bit c = component c has levels in that quarter's TU
  bool split = false;
  const int h = n >> 1;
  for (int c = 0; c < 3; ++c) {
    const int pw = c ? g.W / 2 : g.W, ph = c ? g.H / 2 : g.H, bs = c ? n / 2 : n;
    const int bx = c ? X0 / 2 : X0, by = c ? Y0 / 2 : Y0;
    const size_t ps = c ? g.csize() : g.ysize();
    const uint16_t* ref = l0_plane(a, c, r0) + slot * ps;
    const uint16_t* ref1 = a.ref1_y ? (c == 0 ? a.ref1_y : (c == 1 ? a.ref1_u : a.ref1_v)) + slot * ps : ref;
    const uint16_t* src = (c == 0 ? a.src_y : (c == 1 ? a.src_u : a.src_v)) + slot * ps;
    uint16_t* rec = (c == 0 ? a.rec_y : (c == 1 ? a.rec_u : a.rec_v)) + slot * ps;
    int16_t* lev = (c == 0 ? a.coef_y : (c == 1 ? a.coef_u : a.coef_v)) + slot * ps + static_cast<size_t>(by) * pw + bx;
    const int ww = (a.wp && dir == hevc::DIR_L0 && r0 == 0) ? a.wp[slot * 6 + 2 * c] : 0;
    const int wo = ww ? a.wp[slot * 6 + 2 * c + 1] : 0;
    if (c == 0) mc_block<8>(S, ref, ref1, pw, ph, bx, by, bs, dir, mvx, mvy, mv1x, mv1y, bd, ww, wo);
    else mc_block<4>(S, ref, ref1, pw, ph, bx, by, bs, dir, mvx, mvy, mv1x, mv1y, bd, ww, wo);
    for (int i = lane; i < bs * bs; i += 64) {
      const int y = i / bs, x = i - y * bs;
      const int r = static_cast<int>(src[static_cast<size_t>(by + y) * pw + bx + x]) - S.pred[i];
      S.R[y * 32 + x] = r;
      if (TSPLIT && c == 0) S.R2[y * 32 + x] = r;
    }
    wave_sync();
    const int l2 = c ? lg - 1 : lg;
    const int qc = c ? qpc : qpl;
    bool coded = false;
    if constexpr (TSPLIT) {
      if (lg >= 4) {
      coded = c == 0 || split;
      if (c == 0) {
        const bool nz = hv::transform_quant_block(D, S.R, S.S, lev, pw, hv::TqParams{l2, bd, qc, false, false, a.sdh ? 0 : -1});
        for (int k = 0; k < 4; ++k) cbfq[k] = nz;
        {
          bool nzq[4];
          for (int k = 0; k < 4; ++k) {
            const int o = (k >> 1) * h * 32 + (k & 1) * h;
            nzq[k] = hv::transform_quant_block(D, S.R2 + o, S.S, S.lev2 + o, 32, hv::TqParams{l2 - 1, bd, qc, false, false, a.sdh ? 0 : -1});
          }
          const bool any = nzq[0] || nzq[1] || nzq[2] || nzq[3];
          if (any) {
            // lambda for SSD (HM: 0.57 * 2^((QP - 12) / 3), at the coded bit depth)
            const float lam = 0.57f * exp2f((qpy - 12) / 3.0f) * static_cast<float>(1 << (2 * (bd - 8)));
            const long long d1 = recon_ssd(S, S.R, src, pw, bx, by, n, maxv);
            const long long d4 = recon_ssd(S, S.R2, src, pw, bx, by, n, maxv);
            const int b1 = level_bits(lev, pw, n) + (nz ? 2 * lg + 2 : 0);
            const int b4 = level_bits(S.lev2, 32, n) + 4 + (nzq[0] + nzq[1] + nzq[2] + nzq[3]) * (2 * lg);
            split = static_cast<float>(d4) + lam * b4 < static_cast<float>(d1) + lam * b1;
          }
          if (split) {
            for (int i = lane; i < n * n; i += 64) {
              const int y = i / n, x = i - y * n;
              lev[y * pw + x] = S.lev2[y * 32 + x];
              S.R[y * 32 + x] = S.R2[y * 32 + x];
            }
            for (int k = 0; k < 4; ++k) cbfq[k] = nzq[k];
          }
          wave_sync();
        }
      } else if (split) {
        const int hc = bs >> 1;
        for (int k = 0; k < 4; ++k) {
          const int o = (k >> 1) * hc * 32 + (k & 1) * hc;
          const bool nz = hv::transform_quant_block(D, S.R + o, S.S, lev + (k >> 1) * hc * pw + (k & 1) * hc, pw,
                                                    hv::TqParams{l2 - 1, bd, qc, false, false, a.sdh ? 0 : -1});
          cbfq[k] |= nz << c;
        }
      }
      }
    }
    if (!coded) {
      const bool nz = hv::transform_quant_block(D, S.R, S.S, lev, pw, hv::TqParams{l2, bd, qc, false, false, a.sdh ? 0 : -1});
      for (int k = 0; k < 4; ++k) cbfq[k] |= nz << c;
    }
    // (a block without levels has an all-zero dequantised residual in R)
    for (int i = lane; i < bs * bs; i += 64) {
      const int y = i / bs, x = i - y * bs;
      int v = S.pred[i] + S.R[y * 32 + x];
      rec[static_cast<size_t>(by + y) * pw + bx + x] = static_cast<uint16_t>(v < 0 ? 0 : (v > maxv ? maxv : v));
    }
    wave_sync();
  }
  // granule records: split flag; cbf = that of the TU covering the granule
  const int ng = lg == 5 ? 16 : (lg == 4 ? 4 : 1);
  if (lane < ng) {
    const int k = lg == 5 ? lane >> 2 : lane;  // z-order: the quarter of a 32x32 CU holds 4 granules
    cu[kc + lane].cbf = static_cast<uint8_t>(split ? cbfq[k] : cbfq[0]);
    if (split) cu[kc + lane].flags |= 16;
  }
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

extern "C" void mivc_launch_hevc_inter(int B, int W, int H, const uint16_t* sy, const uint16_t* su, const uint16_t* sv,
                                       const uint16_t* fy, const uint16_t* fu, const uint16_t* fv, uint16_t* ry,
                                       uint16_t* ru, uint16_t* rv, void* ctu, void* cu, int16_t* cy, int16_t* cu_,
                                       int16_t* cv, const int* qp, const int8_t* run, const int* cand,
                                       const int16_t* mv, const int* me_cost, int bd, int tu_split, int sdh,
                                       int intra_bias, void* stream, const int16_t* mvb, const uint8_t* dirb,
                                       const uint16_t* f1y, const uint16_t* f1u, const uint16_t* f1v,
                                       const int16_t* wp, const uint16_t* const* xref, const int16_t* mv8) {
  HevcInterArgs a;
  a.wp = wp;
  a.mv8 = mv8;
  for (int r = 0; r < 3; ++r) {  // xref: [3 x (y, u, v)] of RefPicList0[1 ..] (null: list-0[0])
    a.xref_y[r] = xref && xref[3 * r] ? xref[3 * r] : fy;
    a.xref_u[r] = xref && xref[3 * r + 1] ? xref[3 * r + 1] : fu;
    a.xref_v[r] = xref && xref[3 * r + 2] ? xref[3 * r + 2] : fv;
  }
  a.g = HevcGeom{B, W, H, W / 32, H / 32};
  a.src_y = sy;
  a.src_u = su;
  a.src_v = sv;
  a.ref_y = fy;
  a.ref_u = fu;
  a.ref_v = fv;
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
  a.mv = mv;
  a.mvb = mvb;
  a.dirb = dirb;
  a.ref1_y = f1y;
  a.ref1_u = f1u;
  a.ref1_v = f1v;
  a.me_cost = me_cost;
  a.bd = bd;
  a.tu_split = tu_split;
  a.sdh = sdh;
  a.intra_bias = intra_bias;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(hevc_p_decide, dim3(a.g.nctb(), B), dim3(64), 0, s, a);
  if (tu_split) hipLaunchKernelGGL(hevc_inter_cu<true>, dim3(a.g.nctb() * 4, B), dim3(64), 0, s, a);
  else hipLaunchKernelGGL(hevc_inter_cu<false>, dim3(a.g.nctb() * 4, B), dim3(64), 0, s, a);
}
