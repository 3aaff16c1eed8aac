// Motion estimation for P macroblocks:
//   1. search centre = best (SAD + mv cost) of the temporal predictors of this MB and
//      its left/top/right neighbours and the zero vector;
//   2. integer full search in a (2R+1)^2 window around it, SAD with v_sad_u8 on a
//      reference window staged in LDS (row words re-aligned with v_alignbyte_b32);
//   3. half- then quarter-sample refinement around the best integer vector on the
//      G/b/h/j planes of clause 8.4.2.2.1 built in LDS from the same window;
//      cost = SATD (4x4 Hadamard) + lambda * |mvd| bits;
//   4. the final luma prediction and an open-loop Intra16x16 SATD estimate.
//
// Latency structure (the v1 kernel spent most of its time waiting on ~30
// serialised global loads per MB): every global access is issued in one batch per
// phase -- the source MB, its intra neighbours and the 5 candidate blocks together,
// then the whole reference window as aligned dwords (at most 15 in flight per
// lane) -- and the window carries enough margin that the sub-pel planes come from
// LDS.  Quarter-sample interpolation is branch-free: every position is the
// rounded average of two samples of the 4 planes (kQOff), so the four 16-lane
// candidate groups of a wave never diverge.
//
// One wave64 per macroblock; the workgroup id is remapped so each XCD walks a
// contiguous run of MBs (window rows are shared through that XCD's L2).
#include "kcommon.h"

#include <cstdio>
#include <cstdlib>

namespace mivc {
namespace gpu {

struct MeArgs {
  Geom g;
  const uint8_t* src_y;    // [B, H, W]
  const uint8_t* ref_y;    // [B, H, W]
  const int16_t* pred_mv;  // [B, nmb, 2] quarter-pel predictor (may be null)
  int16_t* out_mv;         // [B, nmb, 2]
  int* out_cost;           // [B, nmb]
  uint8_t* out_pred;       // [B, nmb, 256] final luma prediction (raster 16x16)
  int* out_intra_cost;     // [B, nmb] open-loop Intra16x16 SATD estimate (source neighbours)
  const int* qp;           // [B] frame QP per slot
  int range;               // integer radius, <= 16
  int subpel;              // 0 none, 1 half, 2 quarter
  const uint8_t* hp;       // [B, 3, H + 8, W + 8] b / h / j half-sample planes of ref_y (margin 4)
  const int8_t* aq;        // [B, nmb] adaptive-quantisation QP offsets (nullable)
  int early_sad;           // > 0: skip the integer search when the best candidate's SAD <= this
  // MBs whose cost from an earlier decision (gate_cost: a farther reference's list-0[0] search,
  // a B picture's temporal direct) is already <= gate_thresh (< 0: -gate_thresh * lambda) are
  // not searched (out_cost = kNoCost, out_intra_cost = kNoCost, nothing else written)
  const int* gate_cost;    // [B, nmb] (nullable)
  int gate_thresh;
  // mvd costs against this vector instead of pred_mv (nullable): a farther picture's search is
  // centred on the distance-scaled list-0[0] vector, while its mvd is coded against the
  // neighbours' vectors (which mostly point to RefPicList0[0])
  const int16_t* cost_mv;
  // routing (route.h; rt null: uniform launch): ref_y / hp are pools [B, nbuf, plane], the
  // searched picture is role `role` of each slot, and only slots coding a `want` picture (and,
  // for RefPicList0[role], with more than `role` active entries) are searched
  const SlotRoute* rt;
  int nbuf, role, want;
  // an extra candidate per MB (nullable): [B, nmb, 2] quarter-pel, the lookahead's lowres vector
  // scaled to this picture's reference distance (x264 seeds its search from the lowres motion)
  const int16_t* seed_mv;
};

constexpr int kNoCost = 0x3FFFFFFF;

constexpr int kHpM = 4;  // half-sample plane margin (samples); coordinates clamp into it exactly

constexpr int kMaxR = 16;
constexpr int kML = 4;                                   // window margin left/top (6-tap + qpel)
constexpr int kMR = 6;                                   // margin right/bottom
constexpr int kWinPitch = 17;                            // words per LDS row (odd: bank spread)

// quarter-sample position (xf, yf) -> two LDS offsets into the plane block P[4][20 rows x
// kPP bytes] (plane 0 = G integer, 1 = b half-x, 2 = h half-y, 3 = j centre); sample =
// (A + B + 1) >> 1.  Plane rows are staged as aligned words (kPP = 24 bytes), so a
// plane sample (u, v) sits at byte v * kPP + u + sh, sh = the region's misalignment.
constexpr int kPP = 24;
constexpr int kPlane = 20 * kPP;
#define QO(p, du, dv) ((p) * kPlane + (dv) * kPP + (du))
__constant__ short kQOff[16][2] = {
    {QO(0, 0, 0), QO(0, 0, 0)}, {QO(0, 0, 0), QO(1, 0, 0)}, {QO(1, 0, 0), QO(1, 0, 0)}, {QO(0, 1, 0), QO(1, 0, 0)},
    {QO(0, 0, 0), QO(2, 0, 0)}, {QO(1, 0, 0), QO(2, 0, 0)}, {QO(3, 0, 0), QO(1, 0, 0)}, {QO(1, 0, 0), QO(2, 1, 0)},
    {QO(2, 0, 0), QO(2, 0, 0)}, {QO(3, 0, 0), QO(2, 0, 0)}, {QO(3, 0, 0), QO(3, 0, 0)}, {QO(3, 0, 0), QO(2, 1, 0)},
    {QO(0, 0, 1), QO(2, 0, 0)}, {QO(1, 0, 1), QO(2, 0, 0)}, {QO(3, 0, 0), QO(1, 0, 1)}, {QO(1, 0, 1), QO(2, 1, 0)},
};
#undef QO

// Exp-Golomb length of se(v) with a count-leading-zeros instead of a loop
__device__ __forceinline__ int mvbits(int v) {
  uint32_t x = (v <= 0 ? static_cast<uint32_t>(-2 * v) : static_cast<uint32_t>(2 * v - 1)) + 1u;
  return 2 * (31 - __clz(x)) + 1;
}

// per-byte rounding average (a + b + 1) >> 1 of two packed words
__device__ __forceinline__ uint32_t avg4(uint32_t a, uint32_t b) {
  return (a | b) - (((a ^ b) >> 1) & 0x7F7F7F7Fu);
}

__device__ __forceinline__ int wave_min_key(int key) { return min64(key); }
__device__ __forceinline__ int wave_sum(int v) { return sum64(v); }

// LDS of one workgroup, sized for the largest radius its kernel instance accepts
// (me_p16x16<8> fits 31 workgroups per CU by LDS instead of 22 for radius 16).
template <int MAXR>
struct MeShared {
  static constexpr int kRows = 16 + 2 * MAXR + kML + kMR;
  static constexpr int kLoads = (kRows * 16 + 63) / 64;  // window words per lane (16 words per row at most)
  union {                                  // the window is dead once the sub-pel planes are staged
    uint32_t win[kRows * kWinPitch];       // reference window, aligned words
    uint32_t P32[4 * kPlane / 4 + 4];      // G, b, h, j planes (20 rows x kPP bytes each) + pad
  };
  alignas(16) uint32_t src[64];            // source MB (16 rows x 4 words)
  int nb[36];                              // source intra neighbours: top[16], left[16], tl
  short qoff[32];                          // kQOff copy (lane-varying index -> LDS, not constant)
};

// Stage rows [wy, wy+rows) x bytes [xa, xa + 4*words) of the reference, clamped to the frame.
// All loads are issued before the first LDS store.  WORDS > 0: compile-time row width
// (the lane -> (row, word) split is then a multiply, not a 30-instruction division).
template <int WORDS, class SH>
__device__ __forceinline__ void stage_window(SH& S, const uint8_t* ref, int W, int H, int xa, int wy,
                                             int rows, int words_rt, int lane) {
  const int words = WORDS > 0 ? WORDS : words_rt;
  const int n = rows * words;
  constexpr int kLoadsPerLane = SH::kLoads;
  uint32_t v[kLoadsPerLane];
  const bool inside = xa >= 0 && xa + 4 * words <= W;
  if (inside) {
#pragma unroll
    for (int k = 0; k < kLoadsPerLane; ++k) {
      int i = lane + 64 * k;
      int r = i / words, w = i - r * words;
      int yy = clampi(wy + r, 0, H - 1);
      v[k] = i < n ? *reinterpret_cast<const uint32_t*>(ref + static_cast<size_t>(yy) * W + xa + 4 * w) : 0u;
    }
  } else {
#pragma unroll
    for (int k = 0; k < kLoadsPerLane; ++k) {
      int i = lane + 64 * k;
      int r = i / words, w = i - r * words;
      const uint8_t* row = ref + static_cast<size_t>(clampi(wy + r, 0, H - 1)) * W;
      uint32_t word = 0;
      if (i < n) {
#pragma unroll
        for (int b = 0; b < 4; ++b) word |= static_cast<uint32_t>(row[clampi(xa + 4 * w + b, 0, W - 1)]) << (8 * b);
      }
      v[k] = word;
    }
  }
#pragma unroll
  for (int k = 0; k < kLoadsPerLane; ++k) {
    int i = lane + 64 * k;
    int r = i / words, w = i - r * words;
    if (i < n) S.win[r * kWinPitch + w] = v[k];
  }
}

// 4 bytes of a frame row at byte column x (any alignment, x .. x+3 inside the row)
__device__ __forceinline__ uint32_t load4u(const uint8_t* row, int x) {
  const int a = x & ~3, sh = x & 3;
  const uint32_t w0 = *reinterpret_cast<const uint32_t*>(row + a);
  if (sh == 0) return w0;
  return __builtin_amdgcn_alignbyte(*reinterpret_cast<const uint32_t*>(row + a + 4), w0, sh);
}

// Integer search for a compile-time radius: lane = (dx, dy-group of DYN rows).  The lane
// keeps DYN realigned window rows in registers as a sliding window over the source rows,
// so each window row is read from LDS once (5 words) and feeds DYN candidates' SADs:
// ~5x less LDS traffic per candidate than one-candidate-per-lane.  Source rows are LDS
// broadcasts.
template <int R, class SH>
__device__ __forceinline__ int int_search_fixed(const SH& S, int sh0, int lane, int lambda, int cx, int cy,
                                                int pmx, int pmy) {
  constexpr int side = 2 * R + 1;
  constexpr int G = 64 / side;
  constexpr int DYN = (side + G - 1) / G;
  const int g = lane / side, dx = lane - g * side;
  const int dy0 = g * DYN;
  const int bo = sh0 + kML + dx;
  const int w0 = bo >> 2, sh = bo & 3;
  const int rowbase = g < G ? kML + dy0 : kML;  // idle lanes read valid rows
  // wv[j] = realigned words of window row (rowbase + r + j) while processing source row r
  uint32_t wv[DYN][4];
  auto loadrow = [&](int row, uint32_t (&o)[4]) {
    const uint32_t* rp = S.win + row * kWinPitch + w0;
    const uint32_t a0 = rp[0], a1 = rp[1], a2 = rp[2], a3 = rp[3], a4 = rp[4];
    o[0] = __builtin_amdgcn_alignbyte(a1, a0, sh);
    o[1] = __builtin_amdgcn_alignbyte(a2, a1, sh);
    o[2] = __builtin_amdgcn_alignbyte(a3, a2, sh);
    o[3] = __builtin_amdgcn_alignbyte(a4, a3, sh);
  };
#pragma unroll
  for (int j = 0; j < DYN; ++j) loadrow(rowbase + j, wv[j]);
  uint32_t acc[DYN];
#pragma unroll
  for (int j = 0; j < DYN; ++j) acc[j] = 0;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const uint4 sv = *reinterpret_cast<const uint4*>(S.src + 4 * r);  // LDS broadcast
#pragma unroll
    for (int j = 0; j < DYN; ++j) {
      acc[j] = sad4(sv.x, wv[j][0], acc[j]);
      acc[j] = sad4(sv.y, wv[j][1], acc[j]);
      acc[j] = sad4(sv.z, wv[j][2], acc[j]);
      acc[j] = sad4(sv.w, wv[j][3], acc[j]);
    }
    // pin the row's SADs here: the sad intrinsic is pure, and without this the IR
    // optimiser sinks every SAD below all window loads (194 VGPRs live instead of 46)
#pragma unroll
    for (int j = 0; j < DYN; ++j) asm volatile("" : "+v"(acc[j]));
    if (r < 15) {
#pragma unroll
      for (int j = 0; j + 1 < DYN; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) wv[j][k] = wv[j + 1][k];
      loadrow(rowbase + r + DYN, wv[DYN - 1]);
    }
  }
  int best = 0x7FFFFFFF;
#pragma unroll
  for (int j = 0; j < DYN; ++j) {
    const int dy = dy0 + j;
    const int mvx = (cx + dx - R) * 4, mvy = (cy + dy - R) * 4;
    const int cost = static_cast<int>(acc[j]) + lambda * (mvbits(mvx - pmx) + mvbits(mvy - pmy));
    const int key = (g < G && dy < side) ? ((cost << 12) | (dy * side + dx)) : 0x7FFFFFFF;
    best = key < best ? key : best;
  }
  return best;
}

// Frame-level half-sample planes of a reference batch (clause 8.4.2.2.1): for every
// integer position (x, y) of a (W + 8) x (H + 8) grid (margin kHpM, coordinates of the
// reference clamped to the picture = the normative edge extension):
//   b = half between x and x+1, h = half between y and y+1, j = centre.
// Values outside the margin equal the margin's (all 6 taps replicate), so a consumer
// clamps coordinates into [-4, W+3] x [-4, H+3] exactly.
// Grid (column quads / 64, row groups / 4, slot); a thread produces 4 columns x kHpRows
// rows, sliding a 6-row window of source rows and horizontal intermediates down.
constexpr int kHpRows = 8;

__device__ __forceinline__ void hp_load_row(const uint8_t* fr, int W, int H, int y, int x0, bool xin, int* p) {
  const uint8_t* row = fr + static_cast<size_t>(clampi(y, 0, H - 1)) * W;
  if (xin) {
    const uint32_t w0 = *reinterpret_cast<const uint32_t*>(row + x0 - 4);
    const uint32_t w1 = *reinterpret_cast<const uint32_t*>(row + x0);
    const uint32_t w2 = *reinterpret_cast<const uint32_t*>(row + x0 + 4);
    p[0] = __builtin_amdgcn_ubfe(w0, 16, 8);
    p[1] = __builtin_amdgcn_ubfe(w0, 24, 8);
#pragma unroll
    for (int k = 0; k < 4; ++k) p[2 + k] = __builtin_amdgcn_ubfe(w1, 8 * k, 8);
#pragma unroll
    for (int k = 0; k < 3; ++k) p[6 + k] = __builtin_amdgcn_ubfe(w2, 8 * k, 8);
  } else {
#pragma unroll
    for (int c = 0; c < 9; ++c) p[c] = row[clampi(x0 - 2 + c, 0, W - 1)];
  }
}

// routed (rt): the current picture of every slot coding a reference picture (SF_REF), from and
// into the pools [B, nbuf, plane]
__global__ __launch_bounds__(256) void me_halfpel_planes(const uint8_t* __restrict__ ref, int W, int H,
                                                         uint8_t* __restrict__ hp, const SlotRoute* rt, int nbuf) {
  const int PW = W + 2 * kHpM, PH = H + 2 * kHpM;
  const int q = blockIdx.x * 64 + (threadIdx.x & 63);
  const int py0 = (blockIdx.y * 4 + (threadIdx.x >> 6)) * kHpRows;
  if (q >= PW / 4 || py0 >= PH) return;
  const int slot = blockIdx.z;
  if (rt && (rt[slot].kind < 0 || !(rt[slot].flags & SF_REF))) return;
  const size_t pslot = route_index(rt, nbuf, slot, RO_CUR);
  const int x0 = 4 * q - kHpM, y0 = py0 - kHpM;
  const uint8_t* fr = ref + pslot * W * H;
  const bool xin = x0 - 4 >= 0 && x0 + 8 <= W;
  // window: source rows y-2 .. y+3 (p) and their horizontal 6-tap sums (b1)
  int p[6][9], b1[6][4];
#pragma unroll
  for (int r = 0; r < 5; ++r) {
    hp_load_row(fr, W, H, y0 - 2 + r, x0, xin, p[r + 1]);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      b1[r + 1][k] = h264::tap6(p[r + 1][k], p[r + 1][k + 1], p[r + 1][k + 2], p[r + 1][k + 3], p[r + 1][k + 4],
                                p[r + 1][k + 5]);
  }
  const size_t plane = static_cast<size_t>(PW) * PH;
  uint8_t* o = hp + pslot * 3 * plane + static_cast<size_t>(py0) * PW + 4 * q;
#pragma unroll
  for (int t = 0; t < kHpRows; ++t) {
#pragma unroll
    for (int r = 0; r < 5; ++r) {
#pragma unroll
      for (int c = 0; c < 9; ++c) p[r][c] = p[r + 1][c];
#pragma unroll
      for (int k = 0; k < 4; ++k) b1[r][k] = b1[r + 1][k];
    }
    hp_load_row(fr, W, H, y0 + t + 3, x0, xin, p[5]);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      b1[5][k] = h264::tap6(p[5][k], p[5][k + 1], p[5][k + 2], p[5][k + 3], p[5][k + 4], p[5][k + 5]);
    int bv[4], hv[4], jv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      bv[k] = h264::clip1((b1[2][k] + 16) >> 5);
      hv[k] = h264::clip1((h264::tap6(p[0][k + 2], p[1][k + 2], p[2][k + 2], p[3][k + 2], p[4][k + 2],
                                      p[5][k + 2]) + 16) >> 5);
      jv[k] = h264::clip1((h264::tap6(b1[0][k], b1[1][k], b1[2][k], b1[3][k], b1[4][k], b1[5][k]) + 512) >> 10);
    }
    // byte packing through v_perm: a shift/or packing of clip((x + r) >> n) values gets
    // selected to gfx950's v_ashr_pk_u8_i32, whose high half the backend assumes is zero
    // (it is not): bytes 2-3 came out 255 on some inputs (test_me_halfpel_planes_match_numpy)
    if (py0 + t < PH) {
      *reinterpret_cast<uint32_t*>(o) = pack4_u8(bv);
      *reinterpret_cast<uint32_t*>(o + plane) = pack4_u8(hv);
      *reinterpret_cast<uint32_t*>(o + 2 * plane) = pack4_u8(jv);
    }
    o += PW;
  }
}

#ifdef MIVC_ME_PROFILE
__device__ unsigned long long g_me_prof[64][12];
#define MPROF(ph) do { if (lin < 64 && lane == 0) g_me_prof[lin][ph] = clock64(); } while (0)
#else
#define MPROF(ph) do {} while (0)
#endif

// 8 waves per SIMD (64 VGPRs + a 20-byte spill; the compiler chose 5 at 65 VGPRs + 20 AGPRs):
// me_p 180 -> 170 and me_b 265 -> 248 ms per headline step (profiles/r5_occupancy_ab.md)
template <int MAXR>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8, 8))) void me_p16x16(MeArgs a) {
  const Geom& g = a.g;
  // XCD-aware remap: hardware deals workgroups round-robin over the 8 XCDs; give each XCD
  // a contiguous range of (slot, MB) so neighbouring windows share its L2.
  const int nmb = g.nmb();
  const int total = nmb * g.B;
  int lin = blockIdx.y * gridDim.x + blockIdx.x;
  if ((total & 7) == 0) lin = (lin & 7) * (total >> 3) + (lin >> 3);
  const int slot = lin / nmb, mb = lin - slot * nmb;
  const int mx = mb % g.wmb, my = mb / g.wmb;
  const int lane = threadIdx.x;
  const int X0 = mx * 16, Y0 = my * 16;
  if (a.rt) {  // wave-uniform: this slot codes another picture type / has no such reference
    const SlotRoute& rr = a.rt[slot];
    if (rr.kind != a.want || (a.role < RO_L1 && a.role >= rr.n0)) return;
  }
  const size_t rslot = route_index(a.rt, a.nbuf, slot, a.role);
  const uint8_t* src = a.src_y + slot * g.ysize();
  const uint8_t* ref = a.ref_y + rslot * g.ysize();
  const int W = g.W, H = g.H;
  const int qp = clampi(a.qp[slot] + (a.aq ? a.aq[static_cast<size_t>(slot) * nmb + mb] : 0), 0, 51);
  const int lambda = h264::kLambda[qp];
  const int R = a.range < MAXR ? a.range : MAXR;

  __shared__ MeShared<MAXR> S;
  if (a.gate_cost) {
    const size_t og = static_cast<size_t>(slot) * nmb + mb;
    // gate_thresh < 0: -gate_thresh lambdas of this MB's QP
    const int thr = a.gate_thresh >= 0 ? a.gate_thresh : -a.gate_thresh * lambda;
    if (a.gate_cost[og] <= thr) {  // wave-uniform
      if (lane == 0) {
        a.out_cost[og] = kNoCost;
        if (a.out_intra_cost) a.out_intra_cost[og] = kNoCost;  // the gate's candidate is good: no intra
      }
      return;
    }
  }

  MPROF(0);
  // ---- phase 0: source MB, its intra neighbours, candidate vectors (one batch of loads)
  const int r4 = lane >> 2, c4 = (lane & 3) * 4;
  const uint32_t my_src = *reinterpret_cast<const uint32_t*>(src + static_cast<size_t>(Y0 + r4) * W + X0 + c4);
  int nbv = 0;
  if (lane < 16) nbv = my > 0 ? src[static_cast<size_t>(Y0 - 1) * W + X0 + lane] : 0;
  else if (lane < 32) nbv = mx > 0 ? src[static_cast<size_t>(Y0 + lane - 16) * W + X0 - 1] : 0;
  else if (lane == 32) nbv = (mx > 0 && my > 0) ? src[static_cast<size_t>(Y0 - 1) * W + X0 - 1] : 0;
  int pmx = 0, pmy = 0;
  int cand_x[6] = {0, 0, 0, 0, 0, 0}, cand_y[6] = {0, 0, 0, 0, 0, 0};
  if (a.seed_mv) {
    const size_t so = (static_cast<size_t>(slot) * nmb + mb) * 2;
    cand_x[5] = (a.seed_mv[so] + 2) >> 2;
    cand_y[5] = (a.seed_mv[so + 1] + 2) >> 2;
  }
  if (a.pred_mv) {
    const int16_t* pm = a.pred_mv + static_cast<size_t>(slot) * nmb * 2;
    pmx = pm[mb * 2];
    pmy = pm[mb * 2 + 1];
    cand_x[0] = (pmx + 2) >> 2;
    cand_y[0] = (pmy + 2) >> 2;
    if (a.cost_mv) {
      pmx = a.cost_mv[(static_cast<size_t>(slot) * nmb + mb) * 2];
      pmy = a.cost_mv[(static_cast<size_t>(slot) * nmb + mb) * 2 + 1];
    }
    if (mx > 0) { cand_x[1] = (pm[(mb - 1) * 2] + 2) >> 2; cand_y[1] = (pm[(mb - 1) * 2 + 1] + 2) >> 2; }
    if (my > 0) { cand_x[2] = (pm[(mb - g.wmb) * 2] + 2) >> 2; cand_y[2] = (pm[(mb - g.wmb) * 2 + 1] + 2) >> 2; }
    if (mx < g.wmb - 1) { cand_x[3] = (pm[(mb + 1) * 2] + 2) >> 2; cand_y[3] = (pm[(mb + 1) * 2 + 1] + 2) >> 2; }
  }
  uint32_t cref[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    cand_x[k] = clampi(cand_x[k], -128, 128);
    cand_y[k] = clampi(cand_y[k], -128, 128);
    const uint8_t* rp = ref + static_cast<size_t>(clampi(Y0 + r4 + cand_y[k], 0, H - 1)) * W;
    const int xs = X0 + c4 + cand_x[k];
    uint32_t w = 0;
    if (xs >= 0 && xs + 4 <= W) {
      w = load4u(rp, xs);
    } else {
#pragma unroll
      for (int b = 0; b < 4; ++b) w |= static_cast<uint32_t>(rp[clampi(xs + b, 0, W - 1)]) << (8 * b);
    }
    cref[k] = w;
  }
  S.src[lane] = my_src;
  if (lane < 33) S.nb[lane] = nbv;
  if (lane < 32) S.qoff[lane] = kQOff[lane >> 1][lane & 1];
  wave_sync();
  // MFMA SATD operands shared by the intra estimate and the sub-sample search (see the
  // sub-sample section below for the formulation)
  typedef float v4f __attribute__((ext_vector_type(4)));
  typedef _Float16 v4h __attribute__((ext_vector_type(4)));
  const int mg = lane >> 4, mn = lane & 15, mb_b = mn & 3;
  v4h negH;  // A operand: -H16[row mn][k = 4 mg + j], j = 0..3
#pragma unroll
  for (int j = 0; j < 4; ++j) negH[j] = (__builtin_popcount(mn & (4 * mg + j)) & 1) ? _Float16(1.0f) : _Float16(-1.0f);
  auto as_h = [](uint32_t w) -> v4h {  // 4 samples -> f16 1024 + sample
    const uint32_t lo = __builtin_amdgcn_perm(0x64646464u, w, 0x04010400u);
    const uint32_t hi = __builtin_amdgcn_perm(0x64646464u, w, 0x04030402u);
    const unsigned long long v = (static_cast<unsigned long long>(hi) << 32) | lo;
    return __builtin_bit_cast(v4h, v);
  };
  // ---- open-loop Intra16x16 estimate on source pixels, on MFMA like the sub-sample SATD:
  // column n = (mode = n >> 2, block column b), lane group g = row g of block row t.
  // Every mode is written as pred(x, y) = clip((K + CX[x] + RY[y]) >> 5) (V: CX = 32 top,
  // H: RY = 32 left, DC: K = 32 dc + 16, plane: the linear form); the neighbour sums
  // behind DC and plane are row reductions of the neighbour registers (H = sum (t - 7)
  // top[t] - 8 tl, V alike).  Runs while the candidate reference loads are in flight.
  int intra_key = 0x3FFFFFFF;
  if (a.out_intra_cost) {  // null: the caller already has this picture's estimate (B pictures' L1 search)
    const int mode = mn >> 2;
    const bool has_top = my > 0, has_left = mx > 0;
    const bool ok = (mode == 0 && has_top) || (mode == 1 && has_left) || mode == 2 || (mode == 3 && has_top && has_left);
    const int pk = sum16(lane < 32 ? nbv * ((lane & 15) - 7) + (nbv << 16) : 0);  // weighted + 65536 * plain
    const int ptop = __builtin_amdgcn_readlane(pk, 0), pleft = __builtin_amdgcn_readlane(pk, 16);
    const int tl = __builtin_amdgcn_readlane(nbv, 32);
    const int st = (ptop + 32768) >> 16, sl = (pleft + 32768) >> 16;
    const int Hs = ptop - st * 65536 - 8 * tl, Vs = pleft - sl * 65536 - 8 * tl;
    const int pa = 16 * (__builtin_amdgcn_readlane(nbv, 31) + __builtin_amdgcn_readlane(nbv, 15));
    const int pb = (5 * Hs + 32) >> 6, pc = (5 * Vs + 32) >> 6;
    const int dc = (has_top && has_left) ? (st + sl + 16) >> 5 : (has_left ? (sl + 8) >> 4 : (has_top ? (st + 8) >> 4 : 128));
    const int4 top4 = *reinterpret_cast<const int4*>(S.nb + 4 * mb_b);
    const int cxv[4] = {mode == 0 ? 32 * top4.x : 0, mode == 0 ? 32 * top4.y : (mode == 3 ? pb : 0),
                        mode == 0 ? 32 * top4.z : (mode == 3 ? 2 * pb : 0), mode == 0 ? 32 * top4.w : (mode == 3 ? 3 * pb : 0)};
    const int K = mode == 2 ? 32 * dc + 16 : (mode == 3 ? pa + pb * (4 * mb_b - 7) + 16 : 16);
    float acc = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int y = 4 * t + mg;
      const int ry = mode == 1 ? 32 * S.nb[16 + y] : (mode == 3 ? pc * (y - 7) : 0);
      int pv[4];
#pragma unroll
      for (int x = 0; x < 4; ++x) pv[x] = clampi((K + cxv[x] + ry) >> 5, 0, 255);
      const uint32_t lo = (static_cast<uint32_t>(pv[0]) | (static_cast<uint32_t>(pv[1]) << 16)) | 0x64006400u;
      const uint32_t hi = (static_cast<uint32_t>(pv[2]) | (static_cast<uint32_t>(pv[3]) << 16)) | 0x64006400u;
      const v4h ph = __builtin_bit_cast(v4h, (static_cast<unsigned long long>(hi) << 32) | lo);
      const v4f cs = -__builtin_amdgcn_mfma_f32_16x16x16f16(negH, as_h(S.src[y * 4 + mb_b]), v4f{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      const v4f d = __builtin_amdgcn_mfma_f32_16x16x16f16(negH, ph, cs, 0, 0, 0);
      acc += __builtin_fabsf(d[0]) + __builtin_fabsf(d[1]) + __builtin_fabsf(d[2]) + __builtin_fabsf(d[3]);
    }
    int sv = static_cast<int>(acc);
    sv += __shfl_xor(sv, 1, 64);
    sv += __shfl_xor(sv, 2, 64);
    sv += __shfl_xor(sv, 16, 64);
    sv += __shfl_xor(sv, 32, 64);
    intra_key = min64(ok ? (sv + 1) >> 1 : 0x3FFFFFFF);
  }
  int cx = 0, cy = 0, best_sad = 0x7FFFFFFF;
  {
    // per-lane SADs are <= 1020, so two candidates share one wave reduction (16-bit halves)
    int csad[6];
    {
      const uint32_t p01 = static_cast<uint32_t>(wave_sum(static_cast<int>(sad4(my_src, cref[0], 0) | (sad4(my_src, cref[1], 0) << 16))));
      const uint32_t p23 = static_cast<uint32_t>(wave_sum(static_cast<int>(sad4(my_src, cref[2], 0) | (sad4(my_src, cref[3], 0) << 16))));
      const uint32_t p45 = static_cast<uint32_t>(wave_sum(static_cast<int>(sad4(my_src, cref[4], 0) | (sad4(my_src, cref[5], 0) << 16))));
      csad[0] = p01 & 0xFFFFu;
      csad[1] = p01 >> 16;
      csad[2] = p23 & 0xFFFFu;
      csad[3] = p23 >> 16;
      csad[4] = p45 & 0xFFFFu;
      csad[5] = p45 >> 16;
    }
    int best = 0x7FFFFFFF;
    const int ncand = a.seed_mv ? 6 : 5;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      if (k >= ncand) break;
      int sad = csad[k];
      int cost = sad + lambda * (mvbits(cand_x[k] * 4 - pmx) + mvbits(cand_y[k] * 4 - pmy));
      if (cost < best) {
        best = cost;
        cx = cand_x[k];
        cy = cand_y[k];
        best_sad = sad;
      }
    }
  }

  // early termination (x264-style): a candidate already predicting the MB to within
  // early_sad skips the window and the integer search; the sub-sample refinement below
  // still runs around it (wave-uniform: the SADs are wave reductions)
  const bool early = a.early_sad > 0 && best_sad <= a.early_sad;
  int bx = cx, by = cy;  // integer displacement
  if (!early) {
  MPROF(1);
  // ---- phase 1: reference window around the centre, with margins for the sub-pel planes
  const int wrows = 16 + 2 * R + kML + kMR;
  int wx = X0 + cx - R - kML;
  int xa = wx & ~3, sh0 = wx - xa;
  const int wwords = (wrows + 3) / 4 + 1;
  if (R == 8) stage_window<(16 + 16 + kML + kMR + 3) / 4 + 1>(S, ref, W, H, xa, Y0 + cy - R - kML, wrows, wwords, lane);
  else if (R == 4) stage_window<(16 + 8 + kML + kMR + 3) / 4 + 1>(S, ref, W, H, xa, Y0 + cy - R - kML, wrows, wwords, lane);
  else stage_window<0>(S, ref, W, H, xa, Y0 + cy - R - kML, wrows, wwords, lane);
  __syncthreads();

  MPROF(2);
  // ---- phase 2: integer full search
  const int side = 2 * R + 1;
  int best_key;
  if (R == 8) {
    best_key = int_search_fixed<8>(S, sh0, lane, lambda, cx, cy, pmx, pmy);
  } else if (R == 4) {  // B pictures: 81 candidates around the temporal-direct predictor
    best_key = int_search_fixed<4>(S, sh0, lane, lambda, cx, cy, pmx, pmy);
  } else {
    const int ncand = side * side;
    best_key = 0x7FFFFFFF;
    for (int p = lane; p < ncand; p += 64) {
      int dy = p / side, dx = p - dy * side;
      int bo = sh0 + kML + dx;
      int w0 = bo >> 2, sh = bo & 3;
      uint32_t sad = 0;
#pragma unroll 4
      for (int r = 0; r < 16; ++r) {
        const uint32_t* rowp = S.win + (kML + dy + r) * kWinPitch + w0;
        const uint4 sv = *reinterpret_cast<const uint4*>(S.src + r * 4);
        uint32_t a0 = rowp[0], a1 = rowp[1], a2 = rowp[2], a3 = rowp[3], a4 = rowp[4];
        sad = sad4(sv.x, __builtin_amdgcn_alignbyte(a1, a0, sh), sad);
        sad = sad4(sv.y, __builtin_amdgcn_alignbyte(a2, a1, sh), sad);
        sad = sad4(sv.z, __builtin_amdgcn_alignbyte(a3, a2, sh), sad);
        sad = sad4(sv.w, __builtin_amdgcn_alignbyte(a4, a3, sh), sad);
      }
      int mvx = (cx + dx - R) * 4, mvy = (cy + dy - R) * 4;
      int cost = static_cast<int>(sad) + lambda * (mvbits(mvx - pmx) + mvbits(mvy - pmy));
      int key = (cost << 12) | p;
      best_key = key < best_key ? key : best_key;
    }
  }
  // the zero vector lies outside the window only when the centre is more than R away
  const bool zero_outside = cx < -R || cx > R || cy < -R || cy > R;
  if (zero_outside) {
    int sad = wave_sum(static_cast<int>(sad4(my_src, *reinterpret_cast<const uint32_t*>(
                                                          ref + static_cast<size_t>(Y0 + r4) * W + X0 + c4), 0)));
    int cost = sad + lambda * (mvbits(-pmx) + mvbits(-pmy));
    int key = (cost << 12) | 4095;
    best_key = key < best_key ? key : best_key;
  }
  best_key = wave_min_key(best_key);
  const int bp = best_key & 4095;
  if (bp == 4095) {
    bx = 0;
    by = 0;
  } else {
    by = bp / side;
    bx = cx + (bp - by * side) - R;
    by = cy + by - R;
  }
  }  // !early
  int best_mvx = bx * 4, best_mvy = by * 4;

  MPROF(3);
  // ---- phase 3: sub-pel planes around (bx, by): G from the reference, b, h, j (clause
  // 8.4.2.2.1 half-sample planes) from the frame-level planes built once per reference
  // picture by me_halfpel_planes (the per-MB 6-tap filtering they replace was ~20% of
  // this kernel's instructions).  P(u, v) = plane at (X0+bx-2+u, Y0+by-2+v).
  {
    const int PW = W + 2 * kHpM, PH = H + 2 * kHpM;
    const uint8_t* hp = a.hp + rslot * 3 * PW * PH;
    const int x0 = X0 + bx - 2, y0 = Y0 + by - 2;  // frame coordinates of P(0, 0)
    // aligned words covering bytes x0 .. x0 + 19 of every row: 6 per row from xa = x0 & ~3
    const int xa = x0 & ~3;
    const bool gin = xa >= 0 && xa + kPP <= W;                      // reference row, no clamping
    const bool xin = xa + kHpM >= 0 && xa + kHpM + kPP <= PW;       // half-sample plane row
    // 4 planes (G from the reference itself, b / h / j from hp) x 20 rows x 6 words =
    // 480 words, one batch of loads; lane item i -> (plane, row, word)
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = lane + 64 * k;
      const int pl = i / 120, rem = i - pl * 120, r = rem / 6, w = rem - r * 6;
      uint32_t word = 0;
      if (i < 480) {
        if (pl == 0) {
          const uint8_t* row = ref + static_cast<size_t>(clampi(y0 + r, 0, H - 1)) * W;
          if (gin) {
            word = *reinterpret_cast<const uint32_t*>(row + xa + 4 * w);
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) word |= static_cast<uint32_t>(row[clampi(xa + 4 * w + q, 0, W - 1)]) << (8 * q);
          }
        } else {
          const int yy = clampi(y0 + r, -kHpM, H + kHpM - 1) + kHpM;
          const uint8_t* row = hp + static_cast<size_t>(pl - 1) * PW * PH + static_cast<size_t>(yy) * PW;
          if (xin) {
            word = *reinterpret_cast<const uint32_t*>(row + xa + kHpM + 4 * w);
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q)
              word |= static_cast<uint32_t>(row[clampi(xa + 4 * w + q, -kHpM, W + kHpM - 1) + kHpM]) << (8 * q);
          }
        }
      }
      v[k] = word;
    }
    wave_sync();  // last window reads (integer search) before the planes overwrite it
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = lane + 64 * k;
      if (i < 480) S.P32[i] = v[k];  // plane p starts at word 120 * p; rows of 6 words
    }
  }
  if (lane < 4) S.P32[4 * kPlane / 4 + lane] = 0;
  const int psh = (X0 + bx - 2) & 3;  // misalignment of the staged plane rows
  __syncthreads();

  MPROF(4);
  // 4 consecutive plane bytes at byte offset `off` (any alignment) as one word
  auto load4 = [&](int off) -> uint32_t {
    const int w = off >> 2;
    return __builtin_amdgcn_alignbyte(S.P32[w + 1], S.P32[w], off & 3);
  };
  // 4 predicted samples of a row starting at plane coords (u, v) (G(u,v) = pixel (bx-2+u, by-2+v))
  auto pred4 = [&](int u, int v, int offa, int offb) -> uint32_t {
    const int base = v * kPP + u + psh;
    return avg4(load4(base + offa), load4(base + offb));
  };
  // ---- sub-sample SATD on MFMA.  One v_mfma_f32_16x16x16_f16 evaluates one 4x4-block row
  // (blocks (b, t), b = 0..3) of 4 candidates: output column n = lane & 15 = (candidate
  // c = n >> 2, block b = n & 3) holds the 16 Hadamard coefficients (H4 (x) H4 = the
  // Sylvester H16, entries (-1)^popcount(i & k)) of the residual s - p:
  //     D = C_t + (-H16) . (p + 1024),   C_t = H16 (s + 1024) = H16 s + 16384 e_0
  // with u8 samples entering as the f16 value 1024 + u8 (one v_perm puts the 0x64 exponent
  // byte beside two samples); the 1024 offsets cancel in the DC row and every value is an
  // integer below 2^24, so the f32 accumulation is exact.  K = 16: lane group g = lane >> 4
  // holds row g of its block -- the prediction goes from the LDS planes straight into the B
  // operand, with no residual or Hadamard butterflies on the VALU; |D| sums use the f32
  // abs source modifier.  SATD = (sum |D| + 1) / 2, the scalar form up to per-block rounding.
  v4f cS[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) cS[t] = -__builtin_amdgcn_mfma_f32_16x16x16f16(negH, as_h(S.src[(t * 4 + mg) * 4 + mb_b]),
                                                                             v4f{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  // SATD of this lane's candidate (quarter offsets (dqx, dqy) relative to (4bx, 4by))
  auto satd_cand = [&](int dqx, int dqy) -> int {
    const int q = (dqy & 3) * 4 + (dqx & 3), ox = dqx >> 2, oy = dqy >> 2;
    const int offa = S.qoff[2 * q], offb = S.qoff[2 * q + 1];
    const int u = mb_b * 4 + ox + 2;
    float acc = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const v4f d = __builtin_amdgcn_mfma_f32_16x16x16f16(negH, as_h(pred4(u, t * 4 + mg + oy + 2, offa, offb)), cS[t],
                                                          0, 0, 0);
      acc += __builtin_fabsf(d[0]) + __builtin_fabsf(d[1]) + __builtin_fabsf(d[2]) + __builtin_fabsf(d[3]);
    }
    // the candidate's 16 lanes: block bits 0-1 and row-group bits 4-5
    int s = static_cast<int>(acc);
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    return (s + 1) >> 1;
  };
  // candidate c of a 3x3 ring (0 = centre, 1..8 = the 8 neighbours) -> offsets in units of `step`
  auto ring = [](int c, int step, int* dx, int* dy) {
    int idx = c == 0 ? 4 : (c <= 4 ? c - 1 : c);
    *dx = (idx % 3 - 1) * step;
    *dy = (idx / 3 - 1) * step;
  };
  int best_cost;
  int hx = 0, hy = 0;
  {
    int bkey = 0x7FFFFFFF;
    const int ncand_h = a.subpel >= 1 ? 9 : 1;
    for (int base = 0; base < ncand_h; base += 4) {
      int ci = base + (mn >> 2);
      int c = ci < ncand_h ? ci : 0;
      int ox, oy;
      ring(c, 2, &ox, &oy);
      int s = satd_cand(ox, oy);
      int mvx = best_mvx + ox, mvy = best_mvy + oy;
      int cost = s + lambda * (mvbits(mvx - pmx) + mvbits(mvy - pmy));
      int key = ci < ncand_h ? ((cost << 4) | c) : 0x7FFFFFFF;
      bkey = key < bkey ? key : bkey;
    }
    bkey = wave_min_key(bkey);
    best_cost = bkey >> 4;
    ring(bkey & 15, 2, &hx, &hy);
    MPROF(5);
    if (a.subpel >= 2) {
      int qkey = (best_cost << 4) | 0;
      for (int base = 1; base < 9; base += 4) {
        int ci = base + (mn >> 2);
        int ox, oy;
        ring(ci, 1, &ox, &oy);
        int s = satd_cand(hx + ox, hy + oy);
        int mvx = best_mvx + hx + ox, mvy = best_mvy + hy + oy;
        int cost = s + lambda * (mvbits(mvx - pmx) + mvbits(mvy - pmy));
        int key = (cost << 4) | ci;
        qkey = key < qkey ? key : qkey;
      }
      qkey = wave_min_key(qkey);
      best_cost = qkey >> 4;
      int qx, qy;
      ring(qkey & 15, 1, &qx, &qy);
      hx += qx;
      hy += qy;
    }
    MPROF(6);
    best_mvx += hx;
    best_mvy += hy;
  }
  const size_t o = static_cast<size_t>(slot) * nmb + mb;
  MPROF(7);
  // ---- phase 4: final luma prediction for the chosen vector (lane = row lane>>2, 4 columns)
  {
    int dqx = best_mvx - 4 * bx, dqy = best_mvy - 4 * by;
    int q = (dqy & 3) * 4 + (dqx & 3), ox = dqx >> 2, oy = dqy >> 2;
    int offa = S.qoff[2 * q], offb = S.qoff[2 * q + 1];
    reinterpret_cast<uint32_t*>(a.out_pred + o * 256)[lane] = pred4(c4 + ox + 2, r4 + oy + 2, offa, offb);
  }
  MPROF(8);
  if (lane == 0) {
    a.out_mv[o * 2] = static_cast<int16_t>(best_mvx);
    a.out_mv[o * 2 + 1] = static_cast<int16_t>(best_mvy);
    a.out_cost[o] = best_cost;
    if (a.out_intra_cost) a.out_intra_cost[o] = intra_key + lambda * 4;
  }
  MPROF(9);
}
// Reference selection of P macroblocks (x264 --ref N): the list-0[0] decision (16x16 search,
// P_Skip-aware refinement and 8x8 partitions: mv / mv8 / cost / pred) against the 16x16
// searches of RefPicList0[1 .. nref-1]; cost + lambda * ref_idx bits (CABAC unary: about 1,
// 3, 4, 5 bits).  A farther picture that wins overwrites the decision with its vector (one
// partition), cost and luma prediction and records its index in mref.  One wave per MB.
struct RefSelArgs {
  Geom g;
  int nref;
  int16_t* mv;                 // [B, nmb, 2]
  int16_t* mv8;                // [B, nmb, 4, 2] (nullable)
  int* cost;                   // [B, nmb]
  uint8_t* pred;               // [B, nmb, 256]
  const int16_t* xmv;          // [nref - 1, B, nmb, 2]
  const int* xcost;            // [nref - 1, B, nmb] (kNoCost: not searched)
  const uint8_t* xpred;        // [nref - 1, B, nmb, 256]
  int8_t* mref;                // [B, nmb]
  const int* qp;               // [B]
  const int8_t* aq;            // [B, nmb] (nullable)
  const SlotRoute* rt;         // routed: P slots only, each with its own active list-0 size
};

__global__ __launch_bounds__(64) void me_ref_select(RefSelArgs a) {
  const int nmb = a.g.nmb();
  const int mb = blockIdx.x, slot = blockIdx.y, lane = threadIdx.x;
  if (!route_active(a.rt, slot, SK_P)) return;
  const int nref = a.rt ? min(a.nref, static_cast<int>(a.rt[slot].n0)) : a.nref;
  const size_t o = static_cast<size_t>(slot) * nmb + mb;
  const size_t plane = static_cast<size_t>(a.g.B) * nmb;
  const int qp = clampi(a.qp[slot] + (a.aq ? a.aq[o] : 0), 0, 51);
  const int lambda = h264::kLambda[qp];
  int best = a.cost[o] + lambda, bk = 0;
  for (int k = 1; k < nref; ++k) {
    const int c = a.xcost[(k - 1) * plane + o];
    if (c >= kNoCost) continue;
    const int ck = c + lambda * (k + 2);
    if (ck < best) {
      best = ck;
      bk = k;
    }
  }
  if (bk > 0) {
    const size_t xo = (bk - 1) * plane + o;
    reinterpret_cast<uint32_t*>(a.pred + o * 256)[lane] = reinterpret_cast<const uint32_t*>(a.xpred + xo * 256)[lane];
    if (lane == 0) {
      const int16_t vx = a.xmv[xo * 2], vy = a.xmv[xo * 2 + 1];
      a.mv[o * 2] = vx;
      a.mv[o * 2 + 1] = vy;
      if (a.mv8) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          a.mv8[o * 8 + q * 2] = vx;
          a.mv8[o * 8 + q * 2 + 1] = vy;
        }
      }
      a.cost[o] = a.xcost[xo];
    }
  }
  if (lane == 0) a.mref[o] = static_cast<int8_t>(bk);
}

#ifdef MIVC_ME_PROFILE
extern "C" void mivc_me_prof_read(unsigned long long* out) {
  hipMemcpyFromSymbol(out, HIP_SYMBOL(g_me_prof), sizeof(unsigned long long) * 64 * 12);
}
#endif

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

// b / h / j planes of B reference pictures into hp ([B, 3, H + 8, W + 8], margin 4)
// b / h / j planes of B reference pictures into hp ([B, 3, H + 8, W + 8], margin 4)
extern "C" void mivc_launch_me_halfpel(int B, int W, int H, const uint8_t* ref_y, uint8_t* hp, void* stream,
                                       const void* route, int nbuf) {
  const int PW = W + 2 * kHpM, PH = H + 2 * kHpM;
  const dim3 grid((PW / 4 + 63) / 64, (PH + 4 * kHpRows - 1) / (4 * kHpRows), B);
  hipLaunchKernelGGL(me_halfpel_planes, grid, dim3(256), 0, static_cast<hipStream_t>(stream), ref_y, W, H, hp,
                     static_cast<const SlotRoute*>(route), nbuf);
}

extern "C" void mivc_launch_me(int B, int wmb, int hmb, const uint8_t* src_y, const uint8_t* ref_y,
                               const int16_t* pred_mv, int16_t* out_mv, int* out_cost, uint8_t* out_pred,
                               int* out_intra_cost, const int* qp, int range, int subpel, uint8_t* hp_buf,
                               const int8_t* aq, int planes_ready, int early_sad, void* stream,
                               const int* gate_cost, int gate_thresh, const int16_t* cost_mv, const void* route,
                               int nbuf, int role, int want, const int16_t* seed_mv) {
  // hp_buf: caller-owned [B, 3, H + 8, W + 8] (+64 bytes slack) half-sample plane scratch,
  // resident across frames; nullptr -> stream-ordered scratch for this call only.
  // planes_ready: hp_buf already holds ref_y's planes (an anchor's planes are built once
  // and shared by the P picture and the B pictures that reference it).
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int W = wmb * 16, H = hmb * 16;
  uint8_t* hp = hp_buf;
  if (!hp) {
    const size_t hp_bytes = static_cast<size_t>(B) * 3 * (W + 2 * kHpM) * (H + 2 * kHpM) + 64;
    keep_async_pool();
    if (hipMallocAsync(reinterpret_cast<void**>(&hp), hp_bytes, s) != hipSuccess) {
      fprintf(stderr, "mivc_launch_me: hipMallocAsync(%zu) failed\n", hp_bytes);
      abort();
    }
  }
  if (route && !(planes_ready && hp_buf)) {
    fprintf(stderr, "mivc_launch_me: a routed search needs the resident half-sample pool\n");
    abort();
  }
  if (!(planes_ready && hp_buf)) mivc_launch_me_halfpel(B, W, H, ref_y, hp, stream, nullptr, 0);
  MeArgs a;
  a.g = Geom{B, wmb, hmb, W, H};
  a.src_y = src_y;
  a.ref_y = ref_y;
  a.pred_mv = pred_mv;
  a.out_mv = out_mv;
  a.out_cost = out_cost;
  a.out_pred = out_pred;
  a.out_intra_cost = out_intra_cost;
  a.qp = qp;
  a.range = range < kMaxR ? range : kMaxR;
  a.subpel = subpel;
  a.hp = hp;
  a.aq = aq;
  a.early_sad = early_sad;
  a.gate_cost = gate_cost;
  a.gate_thresh = gate_thresh;
  a.cost_mv = cost_mv;
  a.rt = static_cast<const SlotRoute*>(route);
  a.nbuf = nbuf;
  a.role = role;
  a.want = want;
  a.seed_mv = seed_mv;
  if (a.range <= 8) hipLaunchKernelGGL(me_p16x16<8>, dim3(wmb * hmb, B), dim3(64), 0, s, a);
  else hipLaunchKernelGGL(me_p16x16<kMaxR>, dim3(wmb * hmb, B), dim3(64), 0, s, a);
  if (!hp_buf) (void)hipFreeAsync(hp, s);
}

extern "C" void mivc_launch_me_ref_select(int B, int wmb, int hmb, int nref, int16_t* mv, int16_t* mv8, int* cost,
                                          uint8_t* pred, const int16_t* xmv, const int* xcost, const uint8_t* xpred,
                                          int8_t* mref, const int* qp, const int8_t* aq, void* stream,
                                          const void* route) {
  RefSelArgs a;
  a.rt = static_cast<const SlotRoute*>(route);
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.nref = nref;
  a.mv = mv;
  a.mv8 = mv8;
  a.cost = cost;
  a.pred = pred;
  a.xmv = xmv;
  a.xcost = xcost;
  a.xpred = xpred;
  a.mref = mref;
  a.qp = qp;
  a.aq = aq;
  hipLaunchKernelGGL(me_ref_select, dim3(wmb * hmb, B), dim3(64), 0, static_cast<hipStream_t>(stream), a);
}
