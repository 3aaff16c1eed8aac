// HEVC picture-level kernels: source preparation, in-loop
// deblocking (8.7.2) and sample adaptive offset (8.7.3) with the encoder's SAO
// parameter decision.
//
// Unlike H.264, HEVC deblocking has no raster-order dependency: all vertical edges
// of the picture are filtered first (8-sample grid, decisions read 4 samples and
// modify at most 3 on each side, so edges are independent), then all horizontal
// edges.  Each is one fully parallel launch: a thread owns one 4-sample edge
// segment (luma, plus its 2 chroma lines on the 16-sample chroma grid).  SAO reads the
// deblocked picture and writes every sample of the final reconstruction into a second
// buffer (the encoder ping-pongs the two); one workgroup per
// CTB gathers edge-/band-offset statistics against the source in LDS, picks the
// cheapest of {off, 4 edge classes, band} per component with an SSE + lambda * bits
// estimate, stores the parameters for the CABAC writer and applies them.
#include "kcommon.h"
#include "../common/hevc_tables.h"

namespace mivc {
namespace gpu {

using hevc::CtuInfo;
using hevc::CuInfo;

// ============================================================== source preparation
// Fused source preparation of a whole frame step: the three planes of every slot in
// one launch, 8 output samples (one 16-byte store) per work item, grid-stride (a
// per-row launch issues B x H tiny workgroups and is workgroup-dispatch bound: 1.8 ms
// per plane at B = 64), plus the 8-bit luma proxy the motion search reads (dst8).
struct HevcPrepArgs {
  const uint8_t* src[3];   // frame t of slot 0 per plane; slot b at + b * slot_stride[p]
  long long slot_stride[3];  // bytes
  int pitch[3];              // samples per input row
  int bps;                   // input bytes per sample (1 or 2)
  int w, h;                  // luma display size
  uint16_t* dst[3];          // [B] padded planes (W x H, W/2 x H/2)
  uint8_t* dst8;             // [B] W x H luma proxy = dst >> (bd - 8) (may be null)
  int W, H, B, shift, bd;
};

__global__ __launch_bounds__(256) void hevc_prep_frame(HevcPrepArgs a) {
  const long long ly = static_cast<long long>(a.W / 8) * a.H;       // luma units per slot
  const long long cu = static_cast<long long>(a.W / 16) * (a.H / 2);  // units per chroma plane
  const long long per_slot = ly + 2 * cu;
  const long long total = per_slot * a.B;
  for (long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int b = static_cast<int>(i / per_slot);
    long long r = i - static_cast<long long>(b) * per_slot;
    int p = 0;
    if (r >= ly) {
      r -= ly;
      p = 1 + static_cast<int>(r / cu);
      r -= (p - 1) * cu;
    }
    const int PW = p ? a.W / 2 : a.W, PH = p ? a.H / 2 : a.H;
    const int pw = p ? a.w / 2 : a.w, ph = p ? a.h / 2 : a.h;
    const int upr = PW / 8;
    const int y = static_cast<int>(r / upr), x0 = static_cast<int>(r - static_cast<long long>(y) * upr) * 8;
    const int sy = min(y, ph - 1);
    const uint8_t* row = a.src[p] + b * a.slot_stride[p] + static_cast<long long>(sy) * a.pitch[p] * a.bps;
    uint32_t v[8];
    if (a.bps == 1) {
      if (x0 + 8 <= pw && !(reinterpret_cast<uintptr_t>(row + x0) & 7)) {
        const uint2 wd = *reinterpret_cast<const uint2*>(row + x0);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = ((k < 4 ? wd.x : wd.y) >> (8 * (k & 3))) & 255u;
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = row[min(x0 + k, pw - 1)];
      }
    } else {
      const uint16_t* r16 = reinterpret_cast<const uint16_t*>(row);
      if (x0 + 8 <= pw && !(reinterpret_cast<uintptr_t>(r16 + x0) & 15)) {
        const uint4 wd = *reinterpret_cast<const uint4*>(r16 + x0);
        const uint32_t q[4] = {wd.x, wd.y, wd.z, wd.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = (q[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = r16[min(x0 + k, pw - 1)];
      }
    }
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = (v[2 * k] << a.shift) | ((v[2 * k + 1] << a.shift) << 16);
    uint16_t* d = a.dst[p] + static_cast<size_t>(b) * PW * PH + static_cast<size_t>(y) * PW + x0;
    *reinterpret_cast<uint4*>(d) = make_uint4(o[0], o[1], o[2], o[3]);
    if (p == 0 && a.dst8) {
      const int s8 = a.bd - 8;
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        lo |= (((v[k] << a.shift) >> s8) & 255u) << (8 * k);
        hi |= (((v[k + 4] << a.shift) >> s8) & 255u) << (8 * k);
      }
      *reinterpret_cast<uint2*>(a.dst8 + static_cast<size_t>(b) * PW * PH + static_cast<size_t>(y) * PW + x0) =
          make_uint2(lo, hi);
    }
  }
}

// 8-bit proxy of a u16 plane batch (reference picture for the motion search): 8 samples per item
__global__ __launch_bounds__(256) void hevc_proxy8(const uint16_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                   long long n8, int shift) {
  for (long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n8;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const uint4 w = reinterpret_cast<const uint4*>(src)[i];
    const uint32_t q[4] = {w.x, w.y, w.z, w.w};
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t a0 = ((q[k] & 0xFFFFu) >> shift) & 255u, a1 = ((q[k] >> 16) >> shift) & 255u;
      if (k < 2) lo |= (a0 | (a1 << 8)) << (16 * k);
      else hi |= (a0 | (a1 << 8)) << (16 * (k - 2));
    }
    reinterpret_cast<uint2*>(dst)[i] = make_uint2(lo, hi);
  }
}

// ============================================================== deblocking
struct HevcDbkArgs {
  int B, W, H, wctb, bd;
  uint16_t *y, *u, *v;
  const CuInfo* cu;    // [B, nctb * 16]
  const CtuInfo* ctu;  // [B, nctb]: QpY of the CTB's CUs (qp, qp_pred, qp_first)
  const int8_t* run;   // [B]
  int dir;           // 0 vertical edges, 1 horizontal edges
};

__device__ __forceinline__ const CuInfo& cu_at(const HevcDbkArgs& a, int slot, int x, int y) {
  const int nctb = a.wctb * (a.H / 32);
  const int ci = (y >> 5) * a.wctb + (x >> 5);
  return a.cu[(static_cast<size_t>(slot) * nctb + ci) * 16 + hevc::zorder8((x & 31) >> 3, (y & 31) >> 3)];
}

__device__ __forceinline__ int clip3i(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }

// QpY of the CU covering luma sample (x, y) (8.6.1 with one quantization group per CTB):
// CUs before the CTB's first coded residual keep the group's prediction
__device__ __forceinline__ int qp_at(const HevcDbkArgs& a, int slot, int x, int y) {
  const int nctb = a.wctb * (a.H / 32);
  const CtuInfo& t = a.ctu[static_cast<size_t>(slot) * nctb + (y >> 5) * a.wctb + (x >> 5)];
  return hevc::zorder8((x & 31) >> 3, (y & 31) >> 3) < t.qp_first ? t.qp_pred : t.qp;
}

__global__ void hevc_deblock(HevcDbkArgs a) {
  const int slot = blockIdx.y;
  if (a.run[slot] == 0) return;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  // segments: vertical edges x = 8k (k >= 1), rows of 4; horizontal edges y = 8k, columns of 4
  int xq, yq;
  if (a.dir == 0) {
    const int per_row = a.W / 8 - 1;
    if (idx >= per_row * (a.H / 4)) return;
    xq = (idx % per_row + 1) * 8;
    yq = (idx / per_row) * 4;
  } else {
    const int per_row = a.W / 4;
    if (idx >= per_row * (a.H / 8 - 1)) return;
    xq = (idx % per_row) * 4;
    yq = (idx / per_row + 1) * 8;
  }
  const int xp = a.dir == 0 ? xq - 1 : xq, yp = a.dir == 0 ? yq : yq - 1;
  const CuInfo& Q = cu_at(a, slot, xq, yq);
  const CuInfo& P = cu_at(a, slot, xp, yp);
  const int lq = 3 + ((Q.flags >> 1) & 3) - ((Q.flags >> 4) & 1);  // TU size (inter CUs may split once)
  const int pos = a.dir == 0 ? xq : yq;
  if (pos & ((1 << lq) - 1)) return;  // not a transform / prediction block boundary
  int bs;
  if (P.pred == hevc::CU_INTRA || Q.pred == hevc::CU_INTRA) bs = 2;
  else if ((P.cbf & 1) || (Q.cbf & 1)) bs = 1;
  else {
    // 8.7.2.4: the direction and the refIdx of each used list fix the set of reference pictures
    // (one slice per picture: equal refIdx = the same picture; the B pictures this encoder codes
    // hold different pictures in list 0 and list 1); equal sets compare the vectors list by list
    const int dp = hevc::cu_dir(P), dq = hevc::cu_dir(Q);
    if (dp != dq || ((dp & 1) && P.pad[0] != Q.pad[0]) || ((dp & 2) && P.pad[1] != Q.pad[1])) bs = 1;
    else if ((dp & 1) && (abs(P.mv[0] - Q.mv[0]) >= 4 || abs(P.mv[1] - Q.mv[1]) >= 4)) bs = 1;
    else if ((dp & 2) && (abs(P.mv1[0] - Q.mv1[0]) >= 4 || abs(P.mv1[1] - Q.mv1[1]) >= 4)) bs = 1;
    else bs = 0;
  }
  if (!bs) return;
  const int bd = a.bd, maxv = (1 << bd) - 1;
  const int qpl = (qp_at(a, slot, xp, yp) + qp_at(a, slot, xq, yq) + 1) >> 1;  // 8.7.2.5.3
  const int qb = clip3i(0, 51, qpl), qt = clip3i(0, 53, qpl + 2 * (bs - 1));
  const int beta = hevc::kBetaTable[qb] << (bd - 8), tc = hevc::kTcTable[qt] << (bd - 8);
  const int W = a.W;
  uint16_t* py = a.y + static_cast<size_t>(slot) * W * a.H;
  uint16_t* s0 = py + static_cast<size_t>(yq) * W + xq;
  const int step = a.dir == 0 ? W : 1, across = a.dir == 0 ? 1 : W;
  auto Ps = [&](int l, int i) -> uint16_t& { return s0[l * step - (i + 1) * across]; };
  auto Qs = [&](int l, int i) -> uint16_t& { return s0[l * step + i * across]; };
  const int dp0 = abs(Ps(0, 2) - 2 * Ps(0, 1) + Ps(0, 0)), dp3 = abs(Ps(3, 2) - 2 * Ps(3, 1) + Ps(3, 0));
  const int dq0 = abs(Qs(0, 2) - 2 * Qs(0, 1) + Qs(0, 0)), dq3 = abs(Qs(3, 2) - 2 * Qs(3, 1) + Qs(3, 0));
  const int dpq0 = dp0 + dq0, dpq3 = dp3 + dq3, dp = dp0 + dp3, dq = dq0 + dq3;
  if (dpq0 + dpq3 < beta) {
    auto dsam = [&](int l, int dpq) {
      return 2 * dpq < (beta >> 2) && abs(Ps(l, 3) - Ps(l, 0)) + abs(Qs(l, 0) - Qs(l, 3)) < (beta >> 3) &&
             abs(Ps(l, 0) - Qs(l, 0)) < ((5 * tc + 1) >> 1);
    };
    const bool strong = dsam(0, dpq0) && dsam(3, dpq3);
    const bool dep = dp < ((beta + (beta >> 1)) >> 3), deq = dq < ((beta + (beta >> 1)) >> 3);
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      const int p0 = Ps(l, 0), p1 = Ps(l, 1), p2 = Ps(l, 2), p3 = Ps(l, 3);
      const int q0 = Qs(l, 0), q1 = Qs(l, 1), q2 = Qs(l, 2), q3 = Qs(l, 3);
      if (strong) {
        Ps(l, 0) = static_cast<uint16_t>(clip3i(p0 - 2 * tc, p0 + 2 * tc, (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3));
        Ps(l, 1) = static_cast<uint16_t>(clip3i(p1 - 2 * tc, p1 + 2 * tc, (p2 + p1 + p0 + q0 + 2) >> 2));
        Ps(l, 2) = static_cast<uint16_t>(clip3i(p2 - 2 * tc, p2 + 2 * tc, (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3));
        Qs(l, 0) = static_cast<uint16_t>(clip3i(q0 - 2 * tc, q0 + 2 * tc, (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3));
        Qs(l, 1) = static_cast<uint16_t>(clip3i(q1 - 2 * tc, q1 + 2 * tc, (p0 + q0 + q1 + q2 + 2) >> 2));
        Qs(l, 2) = static_cast<uint16_t>(clip3i(q2 - 2 * tc, q2 + 2 * tc, (p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3));
      } else {
        int delta = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4;
        if (abs(delta) >= tc * 10) continue;
        delta = clip3i(-tc, tc, delta);
        Ps(l, 0) = static_cast<uint16_t>(clip3i(0, maxv, p0 + delta));
        Qs(l, 0) = static_cast<uint16_t>(clip3i(0, maxv, q0 - delta));
        if (dep) Ps(l, 1) = static_cast<uint16_t>(clip3i(0, maxv, p1 + clip3i(-(tc >> 1), tc >> 1, (((p2 + p0 + 1) >> 1) - p1 + delta) >> 1)));
        if (deq) Qs(l, 1) = static_cast<uint16_t>(clip3i(0, maxv, q1 + clip3i(-(tc >> 1), tc >> 1, (((q2 + q0 + 1) >> 1) - q1 - delta) >> 1)));
      }
    }
  }
  // chroma: bS 2 on the 16-luma-sample grid, 2 chroma lines per luma segment
  if (bs == 2 && !(pos & 15)) {
    const int qpc = hevc::chroma_qp_map(qpl);
    const int tcc = hevc::kTcTable[clip3i(0, 53, qpc + 2)] << (bd - 8);
    const int cw = W / 2;
    for (int c = 0; c < 2; ++c) {
      uint16_t* pc = (c == 0 ? a.u : a.v) + static_cast<size_t>(slot) * cw * (a.H / 2);
      uint16_t* q = pc + static_cast<size_t>(yq / 2) * cw + xq / 2;
      const int st = a.dir == 0 ? cw : 1, ac = a.dir == 0 ? 1 : cw;
#pragma unroll
      for (int l = 0; l < 2; ++l) {
        uint16_t* s = q + l * st;
        const int p0 = s[-ac], p1 = s[-2 * ac], q0 = s[0], q1 = s[ac];
        const int delta = clip3i(-tcc, tcc, ((((q0 - p0) << 2) + p1 - q1 + 4) >> 3));
        s[-ac] = static_cast<uint16_t>(clip3i(0, maxv, p0 + delta));
        s[0] = static_cast<uint16_t>(clip3i(0, maxv, q0 - delta));
      }
    }
  }
}

// ============================================================== SAO
struct HevcSaoArgs {
  int B, W, H, wctb, hctb, bd;
  const uint16_t *dy, *du, *dv;   // deblocked copy (input)
  uint16_t *y, *u, *v;            // output (final reconstruction)
  const uint16_t *sy, *su, *sv;   // source
  CtuInfo* ctu;
  const int* qp;   // [B, nctb] QpY per CTB
  const int8_t* run;
  int enable;
  // 64x64 CTUs (one SAO parameter set per CTU): 0 = 32x32 CTBs (statistics, decision and
  // apply per workgroup); 1 = one workgroup per CTU gathers the statistics of its four
  // record blocks, decides and writes the parameters into all four records; 2 = one
  // workgroup per record block applies its CTU's parameters
  int mode;
};

struct SaoShared {
  // the deblocked CTB with a one-sample border (luma 34 x 34, chroma 18 x 18 each): every
  // sample is loaded once; statistics and apply read their neighbours here
  uint16_t tile[34 * 34 + 2 * 18 * 18];
  int eo_cnt[3][4][4], eo_sum[3][4][4];   // [comp][class][category 1..4]
  int bo_cnt[3][32], bo_sum[3][32];
  int type[2], cls[2], band[3];
  int off[3][4];
};

__device__ __forceinline__ int sgn(int v) { return (v > 0) - (v < 0); }

__device__ __forceinline__ int sao_round_div(int s, int n) {
  if (n == 0) return 0;
  const int a = s < 0 ? -s : s;
  const int q = (a + n / 2) / n;
  return s < 0 ? -q : q;
}

// distortion change of adding offset o to n samples whose source - recon sum is s
__device__ __forceinline__ long long sao_dd(int n, int s, int o) {
  return static_cast<long long>(n) * o * o - 2ll * o * s;
}

// SAO decision of a CTB / CTU from the statistics in S (eo_* / bo_*): parameters into S and
// into the records of its nblk record blocks (ci = the first one)
__device__ __forceinline__ void sao_decide(const HevcSaoArgs& a, SaoShared& S, int slot, int ci, int nblk, int tid) {
  const int bd = a.bd;
  // ---- decision.  Every candidate is priced by its own lane (lanes 0-7: edge-offset class k
  // for luma / the chroma pair, lanes 32-127: band position p of Y / Cb / Cr), then lanes 0 / 1
  // pick in the serial order (edge classes 0..3, then the band offsets; the first of equal
  // costs) -- the choice a single-lane scan makes, without 300 serial candidate evaluations
  __shared__ double s_eo_cost[2][4];
  __shared__ int s_eo_off[2][4][2][4];
  __shared__ double s_bo_w[3][32];
  __shared__ int s_bo_off[3][32][4];
  const int qp_ctb = a.qp[static_cast<size_t>(slot) * a.wctb * a.hctb + ci];
  const double lam = 0.57 * exp2((qp_ctb - 12) / 3.0) * static_cast<double>(1 << (2 * (bd - 8)));
  const int cmax = (1 << (min(bd, 10) - 5)) - 1;
  if (a.enable && tid < 8) {  // edge offset class k, components of group tid >> 2
    const int g = tid >> 2, k = tid & 3, c0 = g ? 1 : 0, nc = g ? 2 : 1;
    double cost = lam * (1 + 2);
    for (int cc = 0; cc < nc; ++cc) {
      const int c = c0 + cc;
      for (int e = 0; e < 4; ++e) {
        int v = sao_round_div(S.eo_sum[c][k][e], S.eo_cnt[c][k][e]);
        v = e < 2 ? clampi(v, 0, cmax) : clampi(v, -cmax, 0);
        // shrink while it does not pay
        while (v != 0) {
          const double d0 = static_cast<double>(sao_dd(S.eo_cnt[c][k][e], S.eo_sum[c][k][e], v)) + lam * (v < 0 ? -v : v);
          const int v2 = v > 0 ? v - 1 : v + 1;
          const double d1 = static_cast<double>(sao_dd(S.eo_cnt[c][k][e], S.eo_sum[c][k][e], v2)) + lam * (v2 < 0 ? -v2 : v2);
          if (d1 <= d0) v = v2;
          else break;
        }
        s_eo_off[g][k][cc][e] = v;
        cost += static_cast<double>(sao_dd(S.eo_cnt[c][k][e], S.eo_sum[c][k][e], v)) + lam * ((v < 0 ? -v : v) + 1);
      }
    }
    s_eo_cost[g][k] = cost;
  } else if (a.enable && tid >= 32 && tid < 128) {  // band offset window at position p of component c
    const int c = (tid - 32) >> 5, p = tid & 31;
    double w = lam * 5;
    for (int k = 0; k < 4; ++k) {
      const int b = (p + k) & 31;
      int v = clampi(sao_round_div(S.bo_sum[c][b], S.bo_cnt[c][b]), -cmax, cmax);
      const double dv = static_cast<double>(sao_dd(S.bo_cnt[c][b], S.bo_sum[c][b], v)) + lam * ((v < 0 ? -v : v) + (v != 0));
      if (dv > lam) v = 0;
      s_bo_off[c][p][k] = v;
      w += v ? static_cast<double>(sao_dd(S.bo_cnt[c][b], S.bo_sum[c][b], v)) + lam * ((v < 0 ? -v : v) + 1) : lam;
    }
    s_bo_w[c][p] = w;
  }
  __syncthreads();
  if (tid < 2) {  // lane 0: luma, lane 1: the chroma pair
    const int c0 = tid == 0 ? 0 : 1, nc = tid == 0 ? 1 : 2;
    double best = lam * 1.0;  // "off": no change, ~1 bit for the type
    int btype = 0, bcls = 0, bband[2] = {0, 0}, boff[2][4] = {};
    if (a.enable) {
      for (int k = 0; k < 4; ++k) {
        const double cost = s_eo_cost[tid][k];
        if (cost < best) {
          best = cost;
          btype = 2;
          bcls = k;
          for (int cc = 0; cc < nc; ++cc)
            for (int e = 0; e < 4; ++e) boff[cc][e] = s_eo_off[tid][k][cc][e];
        }
      }
      double cost = lam * 1;
      int pos[2] = {0, 0};
      for (int cc = 0; cc < nc; ++cc) {
        const int c = c0 + cc;
        double bestw = 1e300;
        for (int p = 0; p < 32; ++p)
          if (s_bo_w[c][p] < bestw) {
            bestw = s_bo_w[c][p];
            pos[cc] = p;
          }
        cost += bestw;
      }
      if (cost < best) {
        best = cost;
        btype = 1;
        for (int cc = 0; cc < nc; ++cc) {
          bband[cc] = pos[cc];
          for (int k = 0; k < 4; ++k) boff[cc][k] = s_bo_off[c0 + cc][pos[cc]][k];
        }
      }
    }
    S.type[tid] = btype;
    S.cls[tid] = bcls;
    for (int cc = 0; cc < nc; ++cc) {
      S.band[c0 + cc] = bband[cc];
      for (int k = 0; k < 4; ++k) S.off[c0 + cc][k] = boff[cc][k];
    }
  }
  __syncthreads();
  if (tid < nblk) {  // mode 1: every record block of the CTU carries its parameters
    const int bx = (ci % a.wctb) + (tid & 1), by = (ci / a.wctb) + (tid >> 1);
    if (bx < a.wctb && by < a.hctb) {
      CtuInfo* t = a.ctu + static_cast<size_t>(slot) * a.wctb * a.hctb + by * a.wctb + bx;
      for (int k = 0; k < 2; ++k) {
        t->sao_type[k] = static_cast<uint8_t>(S.type[k]);
        t->sao_class[k] = static_cast<uint8_t>(S.cls[k]);
      }
      for (int c = 0; c < 3; ++c) {
        t->sao_band[c] = static_cast<uint8_t>(S.band[c]);
        for (int k = 0; k < 4; ++k) t->sao_off[c][k] = static_cast<int8_t>(S.type[c ? 1 : 0] ? S.off[c][k] : 0);
      }
    }
  }
}

__global__ __launch_bounds__(256) void hevc_sao(HevcSaoArgs a) {
  __shared__ SaoShared S;
  const int slot = blockIdx.y;
  if (a.run[slot] == 0) return;
  const int tid = threadIdx.x;
  int ci = blockIdx.x, rx = ci % a.wctb, ry = ci / a.wctb;
  int nblk = 1;  // record blocks whose statistics feed the decision
  if (a.mode == 1) {
    const int wctu = (a.wctb + 1) / 2;
    rx = (blockIdx.x % wctu) * 2;
    ry = (blockIdx.x / wctu) * 2;
    ci = ry * a.wctb + rx;
    nblk = 4;
  }
  const int bd = a.bd, maxv = (1 << bd) - 1;
  for (int i = tid; i < 3 * 16; i += 256) {
    (&S.eo_cnt[0][0][0])[i] = 0;
    (&S.eo_sum[0][0][0])[i] = 0;
  }
  for (int i = tid; i < 3 * 32; i += 256) {
    (&S.bo_cnt[0][0])[i] = 0;
    (&S.bo_sum[0][0])[i] = 0;
  }
  // sample (x, y) of component c relative to its CTB block, x, y in [-1, cs]
  auto T = [&](int c, int x, int y) -> int {
    return c == 0 ? S.tile[(y + 1) * 34 + x + 1] : S.tile[34 * 34 + (c - 1) * 18 * 18 + (y + 1) * 18 + x + 1];
  };
  static constexpr int hp[4][2] = {{-1, 1}, {0, 0}, {-1, 1}, {1, -1}};
  static constexpr int vp[4][2] = {{0, 0}, {-1, 1}, {-1, 1}, {-1, 1}};
  for (int j = 0; j < nblk; ++j) {
  if (a.mode == 1) {
    rx = (ci % a.wctb) + (j & 1);
    ry = (ci / a.wctb) + (j >> 1);
    if (rx >= a.wctb || ry >= a.hctb) continue;  // (uniform) partial CTU at the picture edge
    __syncthreads();  // the previous block's statistics are done with the tile
  }
  for (int i = tid; i < 34 * 34 + 2 * 18 * 18; i += 256) {
    int c = 0, k = i;
    if (i >= 34 * 34) {
      c = 1 + (i - 34 * 34) / (18 * 18);
      k = (i - 34 * 34) % (18 * 18);
    }
    const int ts = c ? 18 : 34, cs = c ? 16 : 32;
    const int pw = c ? a.W / 2 : a.W, ph = c ? a.H / 2 : a.H;
    const int X = clampi(rx * cs + k % ts - 1, 0, pw - 1), Y = clampi(ry * cs + k / ts - 1, 0, ph - 1);
    const uint16_t* d = (c == 0 ? a.dy : (c == 1 ? a.du : a.dv)) + slot * static_cast<size_t>(pw) * ph;
    S.tile[i] = d[static_cast<size_t>(Y) * pw + X];  // border samples outside the picture: never used
  }
  __syncthreads();
  // ---- statistics (luma 1024 samples, chroma 2 x 256)
  if (a.enable && a.mode != 2) {
    for (int i = tid; i < 1024 + 512; i += 256) {
      int c, x, y;
      if (i < 1024) {
        c = 0;
        x = i & 31;
        y = i >> 5;
      } else {
        c = 1 + ((i - 1024) >> 8);
        x = (i - 1024) & 15;
        y = ((i - 1024) >> 4) & 15;
      }
      const int pw = c ? a.W / 2 : a.W, ph = c ? a.H / 2 : a.H, cs = c ? 16 : 32;
      const size_t ps = static_cast<size_t>(pw) * ph;
      const uint16_t* s = (c == 0 ? a.sy : (c == 1 ? a.su : a.sv)) + slot * ps;
      const int X = rx * cs + x, Y = ry * cs + y;
      const int v = T(c, x, y);
      const int diff = static_cast<int>(s[static_cast<size_t>(Y) * pw + X]) - v;
      const int b = v >> (bd - 5);
      atomicAdd(&S.bo_cnt[c][b], 1);
      atomicAdd(&S.bo_sum[c][b], diff);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int xa = X + hp[k][0], ya = Y + vp[k][0], xb = X + hp[k][1], yb = Y + vp[k][1];
        if (xa < 0 || ya < 0 || xb < 0 || yb < 0 || xa >= pw || xb >= pw || ya >= ph || yb >= ph) continue;
        int e = 2 + sgn(v - T(c, x + hp[k][0], y + vp[k][0])) + sgn(v - T(c, x + hp[k][1], y + vp[k][1]));
        if (e <= 2) e = (e == 2) ? 0 : e + 1;
        if (!e) continue;
        atomicAdd(&S.eo_cnt[c][k][e - 1], 1);
        atomicAdd(&S.eo_sum[c][k][e - 1], diff);
      }
    }
  }
  }  // record blocks
  __syncthreads();
  if (a.mode == 2) {  // apply the parameters its CTU's first record block carries
    const CtuInfo* t0 = a.ctu + static_cast<size_t>(slot) * a.wctb * a.hctb + (ry & ~1) * a.wctb + (rx & ~1);
    if (tid < 2) {
      S.type[tid] = t0->sao_type[tid];
      S.cls[tid] = t0->sao_class[tid];
    }
    if (tid < 12) S.off[tid >> 2][tid & 3] = t0->sao_off[tid >> 2][tid & 3];
    if (tid < 3) S.band[tid] = t0->sao_band[tid];
  }
  if (a.mode != 2) sao_decide(a, S, slot, ci, nblk, tid);
  if (a.mode == 1) return;  // applied by the per-block launch
  __syncthreads();
  // ---- apply (reads the deblocked copy, writes the output)
  for (int i = tid; i < 1024 + 512; i += 256) {
    int c, x, y;
    if (i < 1024) {
      c = 0;
      x = i & 31;
      y = i >> 5;
    } else {
      c = 1 + ((i - 1024) >> 8);
      x = (i - 1024) & 15;
      y = ((i - 1024) >> 4) & 15;
    }
    const int pw = c ? a.W / 2 : a.W, ph = c ? a.H / 2 : a.H, cs = c ? 16 : 32;
    const size_t ps = static_cast<size_t>(pw) * ph;
    uint16_t* o = (c == 0 ? a.y : (c == 1 ? a.u : a.v)) + slot * ps;
    const int X = rx * cs + x, Y = ry * cs + y;
    const int v = T(c, x, y);
    const int type = S.type[c ? 1 : 0];
    int r = v;
    if (type == 1) {
      const int k = ((v >> (bd - 5)) - S.band[c]) & 31;
      if (k < 4) r = clampi(v + S.off[c][k], 0, maxv);
    } else if (type == 2) {
      const int k = S.cls[c ? 1 : 0];
      const int xa = X + hp[k][0], ya = Y + vp[k][0], xb = X + hp[k][1], yb = Y + vp[k][1];
      if (!(xa < 0 || ya < 0 || xb < 0 || yb < 0 || xa >= pw || xb >= pw || ya >= ph || yb >= ph)) {
        int e = 2 + sgn(v - T(c, x + hp[k][0], y + vp[k][0])) + sgn(v - T(c, x + hp[k][1], y + vp[k][1]));
        if (e <= 2) e = (e == 2) ? 0 : e + 1;
        if (e) r = clampi(v + S.off[c][e - 1], 0, maxv);
      }
    }
    o[static_cast<size_t>(Y) * pw + X] = static_cast<uint16_t>(r);
  }
}


// ---- 64x64 CTUs: statistics without an LDS tile.  Lane = column (luma: 64 columns; chroma:
// 32 columns per half wave), each lane walks its rows with the rows above / below in
// registers and the horizontal neighbours by lane shuffles (the CTU's edge columns load theirs);
// edge-offset counts and sums accumulate in registers and reach LDS once per wave, the band
// histogram takes one 64-bit LDS add per sample (count in bits 0-15, sum above).  Integer sums:
// the statistics, and so the decision, equal those of hevc_sao's tile pass.
__global__ __launch_bounds__(256) void hevc_sao_stats64(HevcSaoArgs a) {
  __shared__ SaoShared S;
  __shared__ unsigned long long bo64[3][32];
  const int slot = blockIdx.y;
  if (a.run[slot] == 0) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wctu = (a.wctb + 1) / 2;
  const int rx = (blockIdx.x % wctu) * 2, ry = (blockIdx.x / wctu) * 2;
  const int ci = ry * a.wctb + rx;
  for (int i = tid; i < 3 * 16; i += 256) {
    (&S.eo_cnt[0][0][0])[i] = 0;
    (&S.eo_sum[0][0][0])[i] = 0;
  }
  if (tid < 96) (&bo64[0][0])[tid] = 0;
  __syncthreads();
  if (a.enable) {
    const int bd = a.bd;
#pragma unroll 1
    for (int c = 0; c < 3; ++c) {
      const int pw = c ? a.W / 2 : a.W, ph = c ? a.H / 2 : a.H;
      const size_t ps = static_cast<size_t>(pw) * ph;
      const uint16_t* d = (c == 0 ? a.dy : (c == 1 ? a.du : a.dv)) + slot * ps;
      const uint16_t* src = (c == 0 ? a.sy : (c == 1 ? a.su : a.sv)) + slot * ps;
      const int xw = c ? 32 : 64;               // shuffle segment = one CTU row of this component
      const int x = c ? (lane & 31) : lane;
      const int nrows = c ? 4 : 16;
      const int X = (c ? rx * 16 : rx * 32) + x;
      const int Y0 = (c ? ry * 16 + (w * 2 + (lane >> 5)) * 4 : ry * 32 + w * 16);
      const bool xin = X < pw;
      auto ld = [&](int xx, int yy) -> int {
        return d[static_cast<size_t>(clampi(yy, 0, ph - 1)) * pw + clampi(xx, 0, pw - 1)];
      };
      // neighbour columns X - 1 / X + 1 of a row: lane shuffles inside the CTU row, loads at its edges
      auto lft = [&](int v, int yy) { const int t = __shfl_up(v, 1, xw); return x == 0 ? ld(X - 1, yy) : t; };
      auto rgt = [&](int v, int yy) { const int t = __shfl_down(v, 1, xw); return x == xw - 1 ? ld(X + 1, yy) : t; };
      int cnt[4][4], sm[4][4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) cnt[k][e] = sm[k][e] = 0;
      int cp = ld(X, Y0 - 1), cc = ld(X, Y0);
      int lp = lft(cp, Y0 - 1), rp = rgt(cp, Y0 - 1), lc = lft(cc, Y0), rc = rgt(cc, Y0);
      const bool hx = X - 1 >= 0 && X + 1 < pw;
#pragma unroll 1
      for (int i = 0; i < nrows; ++i) {
        const int Y = Y0 + i;
        const int cn = ld(X, Y + 1);
        const int ln = lft(cn, Y + 1), rn = rgt(cn, Y + 1);
        if (xin && Y < ph) {
          const int v = cc;
          const int diff = static_cast<int>(src[static_cast<size_t>(Y) * pw + X]) - v;
          atomicAdd(&bo64[c][v >> (bd - 5)],
                    (static_cast<unsigned long long>(static_cast<long long>(diff)) << 16) + 1ull);
          const bool hy = Y - 1 >= 0 && Y + 1 < ph;
          const int A[4] = {lc, cp, lp, rp}, Bn[4] = {rc, cn, rn, ln};
          const bool ok[4] = {hx, hy, hx && hy, hx && hy};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            int e = 2 + sgn(v - A[k]) + sgn(v - Bn[k]);
            e = e < 2 ? e + 1 : (e == 2 ? 0 : e);
            e = ok[k] ? e : 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const bool hit = e == q + 1;
              cnt[k][q] += hit;
              sm[k][q] += hit ? diff : 0;
            }
          }
        }
        cp = cc;
        cc = cn;
        lp = lc;
        lc = ln;
        rp = rc;
        rc = rn;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int n = sum64(cnt[k][q]), t = sum64(sm[k][q]);
          if (lane == 0 && n) {
            atomicAdd(&S.eo_cnt[c][k][q], n);
            atomicAdd(&S.eo_sum[c][k][q], t);
          }
        }
    }
  }
  __syncthreads();
  if (tid < 96) {
    const unsigned long long v = (&bo64[0][0])[tid];
    (&S.bo_cnt[0][0])[tid] = static_cast<int>(v & 0xFFFFull);
    (&S.bo_sum[0][0])[tid] = static_cast<int>(static_cast<long long>(v) >> 16);
  }
  __syncthreads();
  sao_decide(a, S, slot, ci, 4, tid);
}

// ---- apply: one lane per 4 horizontally adjacent samples of every plane, parameters from the
// sample's record block, neighbours straight from the deblocked picture (L1 / L2 hits)
__global__ __launch_bounds__(256) void hevc_sao_apply(HevcSaoArgs a) {
  const int slot = blockIdx.y;
  if (a.run[slot] == 0) return;
  const int gwl = a.W / 4, gwc = a.W / 8;
  const int gl = gwl * a.H, gc = gwc * (a.H / 2);
  int gi = blockIdx.x * 256 + threadIdx.x;
  if (gi >= gl + 2 * gc) return;
  int c, X, Y;
  if (gi < gl) {
    c = 0;
    Y = gi / gwl;
    X = (gi - Y * gwl) * 4;
  } else {
    gi -= gl;
    c = 1 + (gi >= gc);
    gi -= (c - 1) * gc;
    Y = gi / gwc;
    X = (gi - Y * gwc) * 4;
  }
  const int pw = c ? a.W / 2 : a.W, ph = c ? a.H / 2 : a.H;
  const size_t ps = static_cast<size_t>(pw) * ph;
  const uint16_t* d = (c == 0 ? a.dy : (c == 1 ? a.du : a.dv)) + slot * ps;
  uint16_t* o = (c == 0 ? a.y : (c == 1 ? a.u : a.v)) + slot * ps;
  const int bsh = c ? 4 : 5;  // record block of the sample (32 luma / 16 chroma samples)
  const CtuInfo& t = a.ctu[static_cast<size_t>(slot) * a.wctb * a.hctb + (Y >> bsh) * a.wctb + (X >> bsh)];
  const int type = t.sao_type[c ? 1 : 0];
  const size_t ro = static_cast<size_t>(Y) * pw + X;
  const uint2 cw = *reinterpret_cast<const uint2*>(d + ro);
  int v[4] = {static_cast<int>(cw.x & 0xFFFF), static_cast<int>(cw.x >> 16), static_cast<int>(cw.y & 0xFFFF),
              static_cast<int>(cw.y >> 16)};
  const int maxv = (1 << a.bd) - 1;
  int r[4] = {v[0], v[1], v[2], v[3]};
  if (type == 1) {
    const int band = t.sao_band[c];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = ((v[i] >> (a.bd - 5)) - band) & 31;
      if (k < 4) r[i] = clampi(v[i] + t.sao_off[c][k], 0, maxv);
    }
  } else if (type == 2) {
    const int k = t.sao_class[c ? 1 : 0];
    // the 6 samples X - 1 .. X + 4 of row yy (clamped loads; unavailable ones are never used)
    auto row6 = [&](int yy, int* q) {
      const uint16_t* rp = d + static_cast<size_t>(clampi(yy, 0, ph - 1)) * pw;
      const uint2 m = *reinterpret_cast<const uint2*>(rp + X);
      q[0] = rp[X > 0 ? X - 1 : 0];
      q[1] = m.x & 0xFFFF;
      q[2] = m.x >> 16;
      q[3] = m.y & 0xFFFF;
      q[4] = m.y >> 16;
      q[5] = rp[X + 4 < pw ? X + 4 : pw - 1];
    };
    int up[6], mid[6], dn[6];
    row6(Y, mid);
    if (k != 0) {
      row6(Y - 1, up);
      row6(Y + 1, dn);
    }
    // class k's neighbour pair of sample i with constant register indices (k: 0 horizontal,
    // 1 vertical, 2 135 degrees, 3 45 degrees)
    const bool hx0 = X > 0, hx1 = X + 4 < pw, hy = Y > 0 && Y + 1 < ph;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool lok = i > 0 || hx0, rok = i < 3 || hx1;
      int A, Bv;
      bool ok;
      if (k == 0) {
        A = mid[i];
        Bv = mid[i + 2];
        ok = lok && rok;
      } else if (k == 1) {
        A = up[i + 1];
        Bv = dn[i + 1];
        ok = hy;
      } else if (k == 2) {
        A = up[i];
        Bv = dn[i + 2];
        ok = hy && lok && rok;
      } else {
        A = up[i + 2];
        Bv = dn[i];
        ok = hy && lok && rok;
      }
      if (!ok) continue;
      int e = 2 + sgn(v[i] - A) + sgn(v[i] - Bv);
      if (e <= 2) e = (e == 2) ? 0 : e + 1;
      if (e) r[i] = clampi(v[i] + t.sao_off[c][e - 1], 0, maxv);
    }
  }
  *reinterpret_cast<uint2*>(o + ro) = make_uint2(static_cast<uint32_t>(r[0]) | static_cast<uint32_t>(r[1]) << 16,
                                                 static_cast<uint32_t>(r[2]) | static_cast<uint32_t>(r[3]) << 16);
}

// ============================================================== adaptive quantisation
// Per-CTB QP (x265 --aq-mode 1 --qg-size 32, the libx265 default family of the
// reference's "265" preset, server.go:67-68): each 16x16 block gets x264's variance-AQ
// offset strength * 1.0397 * (log2(AC energy) - 14.427 - 2 (bd - 8)), energy = var(Y
// 16x16) + var(Cb 8x8) + var(Cr 8x8) at the coded bit depth (+ an optional per-block
// float offset, e.g. MB-tree); the CTB's QP offset is the rounded mean of its four
// blocks (x265 averages the AQ partitions of a quantization group), clamped to +-12 so
// that consecutive CTBs stay within CuQpDeltaVal's range.  One wave per 16x16 block.
__global__ __launch_bounds__(256) void hevc_aq_ctb(int W, int H, int bd, const uint16_t* __restrict__ sy,
                                                   const uint16_t* __restrict__ su, const uint16_t* __restrict__ sv,
                                                   const int* __restrict__ qp, float strength,
                                                   const float* __restrict__ extra, long long extra_stride,
                                                   int extra_rows, int* __restrict__ ctb_qp,
                                                   int8_t* __restrict__ mb_aq) {
  __shared__ float s_off[4];
  const int wctb = W / 32, nctb = wctb * (H / 32), wmb = W / 16, nmb = wmb * (H / 16);
  const int ci = blockIdx.x, slot = blockIdx.y;
  const int q = wave_id(), l = lane_id();
  const int mx = (ci % wctb) * 2 + (q & 1), my = (ci / wctb) * 2 + (q >> 1);
  const uint16_t* py = sy + static_cast<size_t>(slot) * W * H + static_cast<size_t>(my * 16 + (l >> 2)) * W + mx * 16 + (l & 3) * 4;
  const uint2 wy = *reinterpret_cast<const uint2*>(py);
  const int cw = W / 2;
  const uint16_t* pc = (l < 32 ? su : sv) + static_cast<size_t>(slot) * cw * (H / 2) +
                       static_cast<size_t>(my * 8 + ((l & 31) >> 2)) * cw + mx * 8 + (l & 3) * 2;
  const uint32_t wc = *reinterpret_cast<const uint32_t*>(pc);
  const int y0 = wy.x & 0xFFFF, y1 = wy.x >> 16, y2 = wy.y & 0xFFFF, y3 = wy.y >> 16;
  const int c0 = wc & 0xFFFF, c1 = wc >> 16;
  const int s = sum64(y0 + y1 + y2 + y3), cs = sum32(c0 + c1);
  const int ss = sum64(y0 * y0 + y1 * y1 + y2 * y2 + y3 * y3), css = sum32(c0 * c0 + c1 * c1);
  const int cs_v = __shfl(cs, 32, 64), css_v = __shfl(css, 32, 64);
  if (l == 0) {
    const long long e = (ss - ((static_cast<long long>(s) * s) >> 8)) + (css - ((static_cast<long long>(cs) * cs) >> 6)) +
                        (css_v - ((static_cast<long long>(cs_v) * cs_v) >> 6));
    float adj = 0.0f;
    if (strength > 0.0f)
      adj = strength * 1.0397f * (log2f(static_cast<float>(e > 1 ? e : 1)) - (14.427f + 2.0f * (bd - 8)));
    if (extra && my < extra_rows) adj += extra[slot * extra_stride + my * wmb + mx];
    s_off[q] = adj;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int off = clampi(static_cast<int>(rintf(0.25f * (s_off[0] + s_off[1] + s_off[2] + s_off[3]))), -12, 12);
    const int base = qp[slot];
    const int v = clampi(base + off, 0, 51);
    ctb_qp[static_cast<size_t>(slot) * nctb + ci] = v;
    if (mb_aq) {
      const int r0 = (ci / wctb) * 2, c0i = (ci % wctb) * 2;
      int8_t* m = mb_aq + static_cast<size_t>(slot) * nmb;
      m[r0 * wmb + c0i] = m[r0 * wmb + c0i + 1] = m[(r0 + 1) * wmb + c0i] = m[(r0 + 1) * wmb + c0i + 1] =
          static_cast<int8_t>(v - base);
    }
  }
}

// QpY bookkeeping after reconstruction (8.6.1, one quantization group per CTB): the
// group's prediction is the QpY of the previous CTB in decoding order (the slice QP at
// the start of the slice and, with WPP, of every CTB row); the CTB's delta is coded in
// its first CU with a coded residual, earlier CUs keep the prediction, and a CTB
// without any coded residual takes the prediction as its QpY.  Deblocking and the
// CABAC writer read the result.  One thread per CTB row (WPP) or per slot.
//
// 64x64 CTUs (ctu64): the 32x32 record blocks are the quantization groups (diff_cu_qp_delta_depth
// 1) of a CTU, coded in z-order; a group's prediction averages the QpY left of and above it
// when those lie in the same CTU (the right column's top granule of the left block, the
// bottom row's left granule of the block above), each replaced by qPY_PREV otherwise.
__device__ __forceinline__ int qg_granule_qp(const CtuInfo& t, int z) { return z >= t.qp_first ? t.qp : t.qp_pred; }

__global__ __launch_bounds__(256) void hevc_qp_fixup(int wctb, int hctb, CtuInfo* __restrict__ ctu,
                                                     const CuInfo* __restrict__ cu, const int* __restrict__ qp,
                                                     const int8_t* __restrict__ run, int wpp, int ctu64) {
  const int slot = blockIdx.x;
  if (run[slot] == 0) return;
  const int nctb = wctb * hctb;
  auto first_coded = [&](size_t c) {
    const CuInfo* g = cu + c * 16;
    int first = 16;
    for (int k = 15; k >= 0; --k)
      if (g[k].cbf) first = k;
    if (first < 16) {  // QpY is per CU: the whole CU whose TU carries the delta takes it
      const int lgc = (g[first].flags >> 1) & 3;
      first &= ~((1 << (2 * lgc)) - 1);
    }
    return first;
  };
  if (ctu64) {
    const int wctu = (wctb + 1) / 2, hctu = (hctb + 1) / 2;
    const int rows_per = wpp ? 1 : hctu;
    for (int r0 = threadIdx.x * rows_per; r0 < hctu; r0 += blockDim.x * rows_per) {
      int prev = qp[slot];
      for (int r = r0; r < r0 + rows_per; ++r)
        for (int x = 0; x < wctu; ++x)
          for (int q = 0; q < 4; ++q) {
            const int bx = 2 * x + (q & 1), by = 2 * r + (q >> 1);
            if (bx >= wctb || by >= hctb) continue;
            const size_t base = static_cast<size_t>(slot) * nctb;
            const size_t c = base + by * wctb + bx;
            const int first = first_coded(c);
            const int qa = (q & 1) ? qg_granule_qp(ctu[base + by * wctb + bx - 1], 5) : prev;
            const int qb = (q & 2) ? qg_granule_qp(ctu[base + (by - 1) * wctb + bx], 10) : prev;
            const int pred = (qa + qb + 1) >> 1;
            CtuInfo& t = ctu[c];
            t.qp_pred = static_cast<int8_t>(pred);
            t.qp_first = static_cast<uint8_t>(first);
            if (first == 16) t.qp = static_cast<int8_t>(pred);
            prev = t.qp;
          }
    }
    return;
  }
  const int rows_per = wpp ? 1 : hctb;
  for (int r0 = threadIdx.x * rows_per; r0 < hctb; r0 += blockDim.x * rows_per) {
    int prev = qp[slot];
    for (int r = r0; r < r0 + rows_per; ++r)
      for (int x = 0; x < wctb; ++x) {
        const size_t c = static_cast<size_t>(slot) * nctb + r * wctb + x;
        const int first = first_coded(c);
        CtuInfo& t = ctu[c];
        t.qp_pred = static_cast<int8_t>(prev);
        t.qp_first = static_cast<uint8_t>(first);
        if (first == 16) t.qp = static_cast<int8_t>(prev);
        prev = t.qp;
      }
  }
}


// ============================================================== sparse level hand-off
// Only the non-zero 4x4 blocks of the quantised levels go to the host CABAC writer
// (hevc::PackedLevels, hevc_codec.h): hevc_nz_map finds them per CTB (one wave: lane =
// luma 4x4 block, lanes 0..31 = chroma blocks, ballots give the masks), hevc_nz_scan turns
// the per-CTB block counts into offsets (one workgroup per slot), hevc_nz_pack copies each
// non-zero block (32 bytes) to its rank in the slot's packed buffer, which is pinned host
// memory: the picture's levels cross PCIe once and only where they are non-zero.
__global__ __launch_bounds__(64) void hevc_nz_map(int W, int H, const int16_t* __restrict__ cy,
                                                  const int16_t* __restrict__ cb, const int16_t* __restrict__ cr,
                                                  unsigned long long* __restrict__ nzmap, int* __restrict__ cnt) {
  const int wctb = W / 32, nctb = wctb * (H / 32);
  const int ci = blockIdx.x, slot = blockIdx.y, l = lane_id();
  const int rx = ci % wctb, ry = ci / wctb;
  const int16_t* py = cy + static_cast<size_t>(slot) * W * H + static_cast<size_t>(ry * 32 + (l >> 3) * 4) * W + rx * 32 + (l & 7) * 4;
  uint64_t a = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) a |= *reinterpret_cast<const uint64_t*>(py + static_cast<size_t>(r) * W);
  const unsigned long long lm = __ballot(a != 0);
  const int cw = W / 2;
  uint64_t c = 0;
  if (l < 32) {
    const int k = l & 15;
    const int16_t* pc = (l < 16 ? cb : cr) + static_cast<size_t>(slot) * cw * (H / 2) +
                        static_cast<size_t>(ry * 16 + (k >> 2) * 4) * cw + rx * 16 + (k & 3) * 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) c |= *reinterpret_cast<const uint64_t*>(pc + static_cast<size_t>(r) * cw);
  }
  const unsigned long long cm = __ballot(l < 32 && c != 0) & 0xFFFFFFFFull;
  if (l == 0) {
    const size_t o = static_cast<size_t>(slot) * nctb + ci;
    nzmap[2 * o] = lm;
    nzmap[2 * o + 1] = cm;
    cnt[o] = __popcll(lm) + __popcll(cm);
  }
}

// per slot: exclusive scan of the block counts (chunked serial sums + Hillis-Steele)
__global__ __launch_bounds__(1024) void hevc_nz_scan(int nctb, const int* __restrict__ cnt, unsigned* __restrict__ off,
                                                     long long cap, int* __restrict__ err) {
  const int slot = blockIdx.x;
  __shared__ int s_sum[1024];
  const int per = (nctb + blockDim.x - 1) / blockDim.x;
  const int i0 = threadIdx.x * per, i1 = min(nctb, i0 + per);
  const size_t base = static_cast<size_t>(slot) * nctb;
  int sum = 0;
  for (int i = i0; i < i1; ++i) sum += cnt[base + i];
  s_sum[threadIdx.x] = sum;
  __syncthreads();
  for (int d = 1; d < blockDim.x; d <<= 1) {
    const int v = threadIdx.x >= d ? s_sum[threadIdx.x - d] : 0;
    __syncthreads();
    s_sum[threadIdx.x] += v;
    __syncthreads();
  }
  int run = threadIdx.x > 0 ? s_sum[threadIdx.x - 1] : 0;
  for (int i = i0; i < i1; ++i) {
    off[base + i] = static_cast<unsigned>(run);
    run += cnt[base + i];
  }
  if (threadIdx.x == blockDim.x - 1 && s_sum[threadIdx.x] > cap) atomicAdd(err, 1);  // cannot happen: cap = all blocks
}

__global__ __launch_bounds__(64) void hevc_nz_pack(int W, int H, const int16_t* __restrict__ cy,
                                                   const int16_t* __restrict__ cb, const int16_t* __restrict__ cr,
                                                   const unsigned long long* __restrict__ nzmap,
                                                   const unsigned* __restrict__ off, long long cap,
                                                   int16_t* __restrict__ out) {
  const int wctb = W / 32, nctb = wctb * (H / 32);
  const int ci = blockIdx.x, slot = blockIdx.y, l = lane_id();
  const int rx = ci % wctb, ry = ci / wctb;
  const size_t o = static_cast<size_t>(slot) * nctb + ci;
  const unsigned long long lm = nzmap[2 * o], cm = nzmap[2 * o + 1];
  int16_t* dst = out + (static_cast<size_t>(slot) * cap + off[o]) * 16;
  const int nl = __popcll(lm);
  if ((lm >> l) & 1ull) {
    const int rank = __popcll(lm & ((1ull << l) - 1ull));
    const int16_t* py = cy + static_cast<size_t>(slot) * W * H + static_cast<size_t>(ry * 32 + (l >> 3) * 4) * W + rx * 32 + (l & 7) * 4;
    uint64_t* d = reinterpret_cast<uint64_t*>(dst + rank * 16);
#pragma unroll
    for (int r = 0; r < 4; ++r) d[r] = *reinterpret_cast<const uint64_t*>(py + static_cast<size_t>(r) * W);
  }
  if (l < 32 && ((cm >> l) & 1ull)) {
    const int rank = nl + __popcll(cm & ((1ull << l) - 1ull));
    const int k = l & 15, cw = W / 2;
    const int16_t* pc = (l < 16 ? cb : cr) + static_cast<size_t>(slot) * cw * (H / 2) +
                        static_cast<size_t>(ry * 16 + (k >> 2) * 4) * cw + rx * 16 + (k & 3) * 4;
    uint64_t* d = reinterpret_cast<uint64_t*>(dst + rank * 16);
#pragma unroll
    for (int r = 0; r < 4; ++r) d[r] = *reinterpret_cast<const uint64_t*>(pc + static_cast<size_t>(r) * cw);
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

static unsigned grid_for(long long items) {
  const long long g = (items + 255) / 256;
  return static_cast<unsigned>(g < 8192 ? (g > 0 ? g : 1) : 8192);  // 32 x 256 CUs, grid-stride beyond
}

// src*: frame t of slot 0 per plane; strides in bytes, pitches in samples.  W % 16 == 0, H % 2 == 0.
extern "C" int mivc_launch_hevc_prep_frame(int B, const void* sy, const void* su, const void* sv, long long ss_y,
                                           long long ss_c, int pitch_y, int pitch_c, int bps, int w, int h,
                                           uint16_t* dy, uint16_t* du, uint16_t* dv, uint8_t* d8, int W, int H,
                                           int shift, int bd, void* stream) {
  if ((W & 15) || (H & 1) || w > W || h > H || (bps != 1 && bps != 2) || bd < 8) return -1;
  HevcPrepArgs a{};
  a.src[0] = static_cast<const uint8_t*>(sy);
  a.src[1] = static_cast<const uint8_t*>(su);
  a.src[2] = static_cast<const uint8_t*>(sv);
  a.slot_stride[0] = ss_y;
  a.slot_stride[1] = a.slot_stride[2] = ss_c;
  a.pitch[0] = pitch_y;
  a.pitch[1] = a.pitch[2] = pitch_c;
  a.bps = bps;
  a.w = w;
  a.h = h;
  a.dst[0] = dy;
  a.dst[1] = du;
  a.dst[2] = dv;
  a.dst8 = d8;
  a.W = W;
  a.H = H;
  a.B = B;
  a.shift = shift;
  a.bd = bd;
  const long long items = static_cast<long long>(B) * (W / 8) * H * 3 / 2;
  hipLaunchKernelGGL(hevc_prep_frame, dim3(grid_for(items)), dim3(256), 0, static_cast<hipStream_t>(stream), a);
  return 0;
}

extern "C" int mivc_launch_hevc_proxy8(const uint16_t* src, uint8_t* dst, long long n, int shift, void* stream) {
  if (n % 8) return -1;
  hipLaunchKernelGGL(hevc_proxy8, dim3(grid_for(n / 8)), dim3(256), 0, static_cast<hipStream_t>(stream), src, dst,
                     n / 8, shift);
  return 0;
}

extern "C" void mivc_launch_hevc_deblock(int B, int W, int H, int bd, uint16_t* y, uint16_t* u, uint16_t* v,
                                         const void* cu, const void* ctu, const int8_t* run, void* stream) {
  HevcDbkArgs a{B, W, H, W / 32, bd, y, u, v, static_cast<const CuInfo*>(cu), static_cast<const CtuInfo*>(ctu), run, 0};
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int nv = (W / 8 - 1) * (H / 4), nh = (W / 4) * (H / 8 - 1);
  if (nv > 0) hipLaunchKernelGGL(hevc_deblock, dim3((nv + 255) / 256, B), dim3(256), 0, s, a);
  a.dir = 1;
  if (nh > 0) hipLaunchKernelGGL(hevc_deblock, dim3((nh + 255) / 256, B), dim3(256), 0, s, a);
}

extern "C" void mivc_launch_hevc_sao(int B, int W, int H, int bd, const uint16_t* dy, const uint16_t* du,
                                     const uint16_t* dv, uint16_t* y, uint16_t* u, uint16_t* v, const uint16_t* sy,
                                     const uint16_t* su, const uint16_t* sv, void* ctu, const int* qp,
                                     const int8_t* run, int enable, void* stream, int ctu64) {
  HevcSaoArgs a{B, W, H, W / 32, H / 32, bd, dy, du, dv, y, u, v, sy, su, sv, static_cast<CtuInfo*>(ctu), qp, run, enable,
                0};
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (!ctu64) {
    hipLaunchKernelGGL(hevc_sao, dim3((W / 32) * (H / 32), B), dim3(256), 0, s, a);
    return;
  }
  static const bool tile_pass = [] {  // MIVC_HEVC_SAO_TILE=1: the LDS-tile pass (A/B switch)
    const char* e = std::getenv("MIVC_HEVC_SAO_TILE");
    return e && std::atoi(e) == 1;
  }();
  a.mode = 1;
  if (tile_pass) {
    hipLaunchKernelGGL(hevc_sao, dim3(((W / 32 + 1) / 2) * ((H / 32 + 1) / 2), B), dim3(256), 0, s, a);
    a.mode = 2;
    hipLaunchKernelGGL(hevc_sao, dim3((W / 32) * (H / 32), B), dim3(256), 0, s, a);
    return;
  }
  hipLaunchKernelGGL(hevc_sao_stats64, dim3(((W / 32 + 1) / 2) * ((H / 32 + 1) / 2), B), dim3(256), 0, s, a);
  const int groups = (W / 4) * H + 2 * (W / 8) * (H / 2);
  hipLaunchKernelGGL(hevc_sao_apply, dim3((groups + 255) / 256, B), dim3(256), 0, s, a);
}

// ctb_qp: [B, nctb] int32 out; mb_aq: [B, nmb16] int8 out (may be null); extra: optional
// per-16x16 float offsets of slot s at extra + s * extra_stride, rows [0, extra_rows) of
// the W / 16 wide grid (the lookahead's grid may stop short of the 32-aligned height)
extern "C" void mivc_launch_hevc_aq(int B, int W, int H, int bd, const uint16_t* sy, const uint16_t* su,
                                    const uint16_t* sv, const int* qp, float strength, const float* extra,
                                    long long extra_stride, int extra_rows, int* ctb_qp, int8_t* mb_aq, void* stream) {
  hipLaunchKernelGGL(hevc_aq_ctb, dim3((W / 32) * (H / 32), B), dim3(256), 0, static_cast<hipStream_t>(stream), W, H,
                     bd, sy, su, sv, qp, strength, extra, extra_stride, extra_rows, ctb_qp, mb_aq);
}

extern "C" void mivc_launch_hevc_qp_fixup(int B, int W, int H, void* ctu, const void* cu, const int* qp,
                                          const int8_t* run, int wpp, void* stream, int ctu64) {
  hipLaunchKernelGGL(hevc_qp_fixup, dim3(B), dim3(256), 0, static_cast<hipStream_t>(stream), W / 32, H / 32,
                     static_cast<CtuInfo*>(ctu), static_cast<const CuInfo*>(cu), qp, run, wpp, ctu64);
}

// levels of B slots -> packed form: nzmap [B, nctb, 2] u64, off [B, nctb] u32, out: B slots of
// cap_blocks 4x4 blocks (pinned host memory, device-visible); cnt: [B, nctb] int scratch.
// out == null: the sub-block maps only (the GPU entropy coder reads the level planes)
extern "C" void mivc_launch_hevc_pack_levels(int B, int W, int H, const int16_t* cy, const int16_t* cb,
                                             const int16_t* cr, unsigned long long* nzmap, int* cnt, unsigned* off,
                                             long long cap_blocks, int16_t* out, int* err, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int nctb = (W / 32) * (H / 32);
  hipLaunchKernelGGL(hevc_nz_map, dim3(nctb, B), dim3(64), 0, s, W, H, cy, cb, cr, nzmap, cnt);
  if (!out) return;
  hipLaunchKernelGGL(hevc_nz_scan, dim3(B), dim3(1024), 0, s, nctb, cnt, off, cap_blocks, err);
  hipLaunchKernelGGL(hevc_nz_pack, dim3(nctb, B), dim3(64), 0, s, W, H, cy, cb, cr, nzmap, off, cap_blocks, out);
}
