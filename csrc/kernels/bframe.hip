// B-picture motion: temporal direct derivation and the B_16x16 mode decision
// (x264's default --bframes 3 behind the reference's `-vcodec libx264`, server.go:69-70).
//
// The GPU codes B pictures with *temporal* direct prediction (direct_spatial_mv_pred_flag
// = 0, x264 --direct temporal): the direct motion of a macroblock depends only on the
// co-located macroblock of RefPicList1[0] and on POC distances (clause 8.4.1.2.3), never
// on its neighbours in the current picture, so every MB of every slot decides in parallel
// (spatial direct needs the neighbours' final motion: a raster-order dependency).
//
//   b_direct_mv  (thread per MB)   direct MVs per list / 8x8 quadrant + the ME predictors
//   b_decide     (wave per MB)     candidates B_L0_16x16 / B_L1_16x16 (the two ME searches),
//                                  B_Bi_16x16 (both ME vectors) and B_Direct_16x16 (B_Skip
//                                  when no residual survives): luma motion compensation from
//                                  the anchors' frame-level half-sample planes, 4x4 SATD,
//                                  cost = SATD + lambda * bits; writes the winner's MbHeader
//                                  motion fields and its luma prediction for encode_inter.
// and two P-picture passes after the 16x16 search:
//   p_mv_refine  (wave per MB)     P_Skip-aware vector choice (Jacobi passes)
//   p_part8x8    (wave per MB)     8x8 quadrant vectors: P_8x8 / P_16x8 / P_8x16 partitions
#include "kcommon.h"

namespace mivc {
namespace gpu {

using h264::MbHeader;

constexpr int kHpMargin = 4;  // me_halfpel_planes margin (csrc/kernels/me.hip)

constexpr int kMaxRefs = 4;  // list-0 pictures an encoder P picture may reference (x264 --ref)

struct BDirectArgs {
  Geom g;
  const MbHeader* col;      // [B, nmb] records of RefPicList1[0] (a P anchor)
  // per refIdxL0 r = refIdxCol (the anchor's list 0 and the B picture's list 0 order the same
  // past anchors, so MapColToList0 is the identity): DistScaleFactor, ignored when direct_copy
  int dsf[kMaxRefs];
  int direct_copy[kMaxRefs];  // td == 0: mvL0 = mvCol, mvL1 = 0
  int16_t* dmv;             // [B, nmb, 2, 4, 2] direct vectors (list, quadrant, xy)
  int8_t* dref;             // [B, nmb, 4] refIdxL0 of each quadrant's direct prediction (nullable: all 0)
  int16_t* pm0;             // [B, nmb, 2] ME predictor L0 (mean of the direct vectors)
  int16_t* pm1;             // [B, nmb, 2] ME predictor L1
  // routed (route.h): col is the record pool [B, nbuf, nmb]; B slots only, each with its own
  // co-located picture (RefPicList1[0]) and its own dsf / direct_copy (SlotRoute)
  const SlotRoute* rt;
  int nbuf;
  // spatial direct (nullable): colZeroFlag of the four quadrants (bit q; 8.4.1.2.2: the
  // co-located block is inter, its refIdxCol is 0 and both vector components are in -1..1)
  uint8_t* czero;
};

__global__ __launch_bounds__(256) void b_direct_mv(BDirectArgs a) {
  const int mb = blockIdx.x * 256 + threadIdx.x, slot = blockIdx.y;
  const int nmb = a.g.nmb();
  if (mb >= nmb || !route_active(a.rt, slot, SK_B)) return;
  const size_t o = static_cast<size_t>(slot) * nmb + mb;
  const MbHeader& c = a.col[route_index(a.rt, a.nbuf, slot, RO_L1) * nmb + mb];
  // a B picture as the co-located one (b-pyramid): a block without list-0 motion gives its
  // list-1 motion (8.4.1.2.1); a P anchor predicts from list 0 only
  const bool col_l1 = a.rt && a.rt[slot].col_l1;
  const bool intra = h264::mbk_is_intra(c.kind);
  int v[2][4][2];
  int rq[4];
  int s[2][2] = {{0, 0}, {0, 0}};
  int cz = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    // direct_8x8_inference: the corner 4x4 block of co-located quadrant q, i.e. its vector;
    // a P anchor predicts from list 0 only
    const int cl = (col_l1 && c.ref[0][q] < 0) ? 1 : 0;
    const bool none = intra || c.ref[cl][q] < 0;
    const int cx = none ? 0 : c.mv[cl][q][0];
    const int cy = none ? 0 : c.mv[cl][q][1];
    const int r = none ? 0 : min(static_cast<int>(c.ref[cl][q]), kMaxRefs - 1);
    rq[q] = r;
    if (!none && c.ref[cl][q] == 0 && abs(cx) <= 1 && abs(cy) <= 1) cz |= 1 << q;
    int l0x, l0y;
    const int dcp = a.rt ? a.rt[slot].dcopy[r] : a.direct_copy[r], dsf = a.rt ? a.rt[slot].dsf[r] : a.dsf[r];
    if (dcp) {
      l0x = cx;
      l0y = cy;
    } else {
      l0x = (dsf * cx + 128) >> 8;
      l0y = (dsf * cy + 128) >> 8;
    }
    v[0][q][0] = l0x;
    v[0][q][1] = l0y;
    v[1][q][0] = dcp ? 0 : l0x - cx;
    v[1][q][1] = dcp ? 0 : l0y - cy;
#pragma unroll
    for (int l = 0; l < 2; ++l) {
      s[l][0] += v[l][q][0];
      s[l][1] += v[l][q][1];
    }
  }
  int16_t* d = a.dmv + o * 16;
#pragma unroll
  for (int l = 0; l < 2; ++l)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      d[l * 8 + q * 2] = static_cast<int16_t>(v[l][q][0]);
      d[l * 8 + q * 2 + 1] = static_cast<int16_t>(v[l][q][1]);
    }
  if (a.dref) {
    const uint32_t rw = static_cast<uint32_t>(rq[0]) | (static_cast<uint32_t>(rq[1]) << 8) |
                        (static_cast<uint32_t>(rq[2]) << 16) | (static_cast<uint32_t>(rq[3]) << 24);
    *reinterpret_cast<uint32_t*>(a.dref + o * 4) = rw;
  }
  if (a.czero) a.czero[o] = static_cast<uint8_t>(cz);
  a.pm0[o * 2] = static_cast<int16_t>((s[0][0] + 2) >> 2);
  a.pm0[o * 2 + 1] = static_cast<int16_t>((s[0][1] + 2) >> 2);
  a.pm1[o * 2] = static_cast<int16_t>((s[1][0] + 2) >> 2);
  a.pm1[o * 2 + 1] = static_cast<int16_t>((s[1][1] + 2) >> 2);
}

struct BDecideArgs {
  Geom g;
  const uint8_t* src_y;            // [B, H, W]
  const uint8_t *ref0, *ref1;      // anchors' luma (RefPicList0[0], RefPicList1[0])
  const uint8_t *hp0, *hp1;        // their b / h / j planes [B, 3, H + 8, W + 8]
  const int16_t *mv0, *mv1;        // [B, nmb, 2] ME vectors per list
  const int *cost0, *cost1;        // ME costs (SATD + lambda * mv bits)
  const uint8_t *pred0, *pred1;    // ME luma predictions [B, nmb, 256]
  const int16_t *pm0, *pm1;        // ME predictors
  const int16_t* dmv;              // [B, nmb, 2, 4, 2]
  const int* qp;                   // [B]
  const int8_t* aq;                // [B, nmb] (nullable)
  MbHeader* hdr;                   // out: kind / ref / mv
  uint8_t* pred_out;               // out: [B, nmb, 256]
  int* cost_out;                   // out: [B, nmb] the winner's cost (vs the intra estimate)
  // implicit bi-prediction weight of list 1 (32: plain average) per refIdxL0 (the list-1
  // picture is always RefPicList1[0]); the ME candidates use entry 0
  int w1[kMaxRefs];
  // direct prediction from RefPicList0[r] (r = dref per quadrant, nullable: all 0):
  // luma / half-sample planes of every list-0 picture (entry 0 = ref0 / hp0)
  const int8_t* dref;
  const uint8_t* ref0k[kMaxRefs];
  const uint8_t* hp0k[kMaxRefs];
  // direct_only: the pre-pass before the two ME searches -- only the direct candidate's cost
  // (SATD + lambda) goes to cost_out; MBs whose direct cost is already low skip the searches
  // (me.hip gate) and their list costs come back as kNoCost
  int direct_only;
  // the pre-pass ran (direct_only = 1 before the searches): pred_out / cost_out hold every MB's
  // direct prediction and cost -- unsearched MBs keep them, the others skip the direct MC
  int have_direct;
  int bparts;  // x264 --partitions b8x8: per-quadrant candidates (B_16x8 / B_8x16 / B_8x8)
  // spatial direct 1 (wavefront decision): searched MBs keep their best explicit candidate (no
  // direct MB / quadrant); b_spatial_decide weighs it against the exact spatial direct motion
  // in decoding order.  2 (fast): direct is priced in parallel with the pre-pass's estimate of
  // the spatial motion (needs the pre-pass); b_spatial_exact / b_spatial_fixup make it exact
  int spatial;
  int dbias;  // direct preferred by dbias * lambda in the 16x16 choice (cost_out stays unbiased)
  const uint8_t* czero;  // spatial == 2: colZeroFlag bits per MB (b_direct_mv)
  // routed (route.h): ref0 / ref1 / hp0 / hp1 / ref0k / hp0k are pool bases, the roles come from
  // each B slot's SlotRoute (list-0 entries, list-1 entry, implicit weights)
  const SlotRoute* rt;
  int nbuf;
};

constexpr int kNoCostB = 0x3FFFFFFF;  // me.hip kNoCost: the MB was not searched

// Quarter-sample luma position (xf, yf) = two (plane, du, dv) taps averaged (the G/b/h/j
// form of clause 8.4.2.2.1 used by me.hip): plane 0 = integer samples, 1 = b (half x),
// 2 = h (half y), 3 = j (centre).
__constant__ int8_t kQTap[16][2][3] = {
    {{0, 0, 0}, {0, 0, 0}}, {{0, 0, 0}, {1, 0, 0}}, {{1, 0, 0}, {1, 0, 0}}, {{0, 1, 0}, {1, 0, 0}},
    {{0, 0, 0}, {2, 0, 0}}, {{1, 0, 0}, {2, 0, 0}}, {{3, 0, 0}, {1, 0, 0}}, {{1, 0, 0}, {2, 1, 0}},
    {{2, 0, 0}, {2, 0, 0}}, {{3, 0, 0}, {2, 0, 0}}, {{3, 0, 0}, {3, 0, 0}}, {{3, 0, 0}, {2, 1, 0}},
    {{0, 0, 1}, {2, 0, 0}}, {{1, 0, 1}, {2, 0, 0}}, {{3, 0, 0}, {1, 0, 1}}, {{1, 0, 1}, {2, 1, 0}},
};

__device__ __forceinline__ uint32_t avg4b(uint32_t a, uint32_t b) { return (a | b) - (((a ^ b) >> 1) & 0x7F7F7F7Fu); }

// implicit weighted bi-prediction of 4 packed samples (8.4.2.3.2 with logWD 5, offsets 0):
// (a * (64 - w1) + b * w1 + 32) >> 6; w1 = 32 is the plain rounded average
__device__ __forceinline__ uint32_t wavg4b(uint32_t a, uint32_t b, int w1) {
  if (w1 == 32) return avg4b(a, b);
  const int w0 = 64 - w1;
  uint32_t o = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int v = (static_cast<int>((a >> (8 * k)) & 255u) * w0 + static_cast<int>((b >> (8 * k)) & 255u) * w1 + 32) >> 6;
    o |= static_cast<uint32_t>(clampi(v, 0, 255)) << (8 * k);
  }
  return o;
}

// 4 consecutive samples (u .. u+3, v) of one plane; coordinates clamp to the plane's
// extension (integer plane: the picture; half-sample planes: their 4-sample margin)
__device__ __forceinline__ uint32_t plane4(const uint8_t* G, const uint8_t* hp, int W, int H, int pl, int u, int v) {
  const uint8_t* row;
  int lo, hi, base;
  if (pl == 0) {
    row = G + static_cast<size_t>(clampi(v, 0, H - 1)) * W;
    lo = 0;
    hi = W - 1;
    base = 0;
  } else {
    const int PW = W + 2 * kHpMargin, PH = H + 2 * kHpMargin;
    row = hp + static_cast<size_t>(pl - 1) * PW * PH +
          static_cast<size_t>(clampi(v, -kHpMargin, H + kHpMargin - 1) + kHpMargin) * PW;
    lo = -kHpMargin;
    hi = W + kHpMargin - 1;
    base = kHpMargin;
  }
  const int x = u + base, a = x & ~3;
  if (u >= lo && u + 3 <= hi && a + 8 <= hi + base + 1) {
    const uint32_t w0 = *reinterpret_cast<const uint32_t*>(row + a);
    const uint32_t w1 = *reinterpret_cast<const uint32_t*>(row + a + 4);
    return __builtin_amdgcn_alignbyte(w1, w0, x & 3);
  }
  uint32_t w = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) w |= static_cast<uint32_t>(row[clampi(u + k, lo, hi) + base]) << (8 * k);
  return w;
}

// predicted samples (x .. x+3, y) of a 16x16 block displaced by the quarter-sample vector
__device__ __forceinline__ uint32_t mc4(const uint8_t* G, const uint8_t* hp, int W, int H, int x, int y, int mvx,
                                        int mvy) {
  const int q = (mvy & 3) * 4 + (mvx & 3);
  const int xi = x + (mvx >> 2), yi = y + (mvy >> 2);
  const uint32_t A = plane4(G, hp, W, H, kQTap[q][0][0], xi + kQTap[q][0][1], yi + kQTap[q][0][2]);
  const uint32_t Bv = plane4(G, hp, W, H, kQTap[q][1][0], xi + kQTap[q][1][1], yi + kQTap[q][1][2]);
  return avg4b(A, Bv);
}

__device__ __forceinline__ int mvbits_se(int v) {
  const uint32_t x = (v <= 0 ? static_cast<uint32_t>(-2 * v) : static_cast<uint32_t>(2 * v - 1)) + 1u;
  return 2 * (31 - __clz(x)) + 1;
}

struct NbMv16 {
  bool avail;
  int ref;
  int mv[2];
};

__device__ __forceinline__ int med3i(int a, int b, int c) { return max(min(a, b), min(max(a, b), c)); }

// Spatial direct of one list (8.4.1.2.2): refIdx = MinPositive over the neighbours A, B, C
// (C replaced by D by the caller), the vector = the 16x16 motion-vector predictor of that
// reference (8.4.1.3: a single neighbour on it gives its vector, else the median, with A
// standing in for B and C when only A is available)
__device__ __forceinline__ void spatial_pmv(NbMv16 A, NbMv16 B, NbMv16 C, int& ref, int& px, int& py) {
  auto minpos = [](int p, int qv) { return (p >= 0 && qv >= 0) ? min(p, qv) : max(p, qv); };
  ref = minpos(A.ref, minpos(B.ref, C.ref));
  px = py = 0;
  if (ref < 0) return;
  if (!B.avail && !C.avail && A.avail) {
    B = A;
    C = A;
  }
  const int match = (A.ref == ref) + (B.ref == ref) + (C.ref == ref);
  if (match == 1) {
    const NbMv16& m = A.ref == ref ? A : (B.ref == ref ? B : C);
    px = m.mv[0];
    py = m.mv[1];
  } else {
    px = med3i(A.mv[0], B.mv[0], C.mv[0]);
    py = med3i(A.mv[1], B.mv[1], C.mv[1]);
  }
}

// Four MBs per wave, one 16-lane row each: a lane owns one 4x4 block (raster order) of its MB
// and prices it for every candidate from registers; quadrant sums go through a pair DPP and a
// small LDS table.  The pass is a chain of dependent loads per MB (vectors -> predictions ->
// costs), so MBs in flight set its speed (one MB per wave, the round-3 layout, was half as
// fast for p_mv_refine).
constexpr int kDecideMbsPerWave = 4;

// 4x4 SATD of this lane's block against 4 packed prediction rows
__device__ __forceinline__ int blk_satd4(const uint32_t (&src)[4], const uint32_t (&pw)[4]) {
  return satd4x4_u8(src, pw);  // packed 16-bit (kcommon.h), = h264::satd4x4 of the residual
}

// The main pass of b_decide after the direct-only pre-pass, for a searched MB (the caller
// returned for gated ones): the same candidates, costs and decisions as the general path,
// computed with one candidate's rows live at a time.
template <class W1>
__device__ __forceinline__ void b_decide_main(const BDecideArgs& a, const uint32_t (&src)[4], size_t o, int slot,
                                              int mb, int lane, int wrow, int q, int X, int Y, uint8_t* pout,
                                              MbHeader* hrec, uint32_t drw, const int16_t* dm, const uint8_t* G0,
                                              const uint8_t* G1, const uint8_t* H0, const uint8_t* H1, W1 w1of) {
  const Geom& g = a.g;
  const int W = g.W, H = g.H;
  const int m0x = a.mv0[o * 2], m0y = a.mv0[o * 2 + 1];
  const int m1x = a.mv1[o * 2], m1y = a.mv1[o * 2 + 1];
  const int by4 = (lane >> 2) * 4, bx4 = (lane & 3) * 4;
  const uint8_t* pr0 = a.pred0 + o * 256 + by4 * 16 + bx4;
  const uint8_t* pr1 = a.pred1 + o * 256 + by4 * 16 + bx4;
  __shared__ int s_pair[kDecideMbsPerWave][4][16];
  uint32_t pb[4];
  {
    uint32_t t[4];
#pragma unroll
    for (int y = 0; y < 4; ++y) t[y] = *reinterpret_cast<const uint32_t*>(pout + 16 * y);
    const int s0 = blk_satd4(src, t);
    s_pair[wrow][0][lane] = s0 + dpp<kDppQuadXor1>(s0);
#pragma unroll
    for (int y = 0; y < 4; ++y) t[y] = *reinterpret_cast<const uint32_t*>(pr0 + 16 * y);
    const int s2 = blk_satd4(src, t);
    s_pair[wrow][2][lane] = s2 + dpp<kDppQuadXor1>(s2);
#pragma unroll
    for (int y = 0; y < 4; ++y) t[y] = *reinterpret_cast<const uint32_t*>(pr1 + 16 * y);
    const int s3 = blk_satd4(src, t);
    s_pair[wrow][3][lane] = s3 + dpp<kDppQuadXor1>(s3);
  }
  const int w10 = w1of(0);
#pragma unroll
  for (int y = 0; y < 4; ++y)
    pb[y] = wavg4b(mc4(G0, H0, W, H, X, Y + y, m0x, m0y), mc4(G1, H1, W, H, X, Y + y, m1x, m1y), w10);
  {
    const int s1 = blk_satd4(src, pb);
    s_pair[wrow][1][lane] = s1 + dpp<kDppQuadXor1>(s1);
  }
  wave_sync();
  int qsat[4][4];  // [candidate][quadrant]
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int l0 = (qq >> 1) * 8 + (qq & 1) * 2;
      qsat[c][qq] = s_pair[wrow][c][l0] + s_pair[wrow][c][l0 + 4];
    }
  const int satd_direct = qsat[0][0] + qsat[0][1] + qsat[0][2] + qsat[0][3];
  const int satd_bi = qsat[1][0] + qsat[1][1] + qsat[1][2] + qsat[1][3];
  const int qp = clampi(a.qp[slot] + (a.aq ? a.aq[o] : 0), 0, 51);
  const int lambda = h264::kLambda[qp];
  const int c_direct = satd_direct + lambda * 1;
  const int c_l0 = a.cost0[o] + lambda * 3;
  const int c_l1 = a.cost1[o] + lambda * 3;
  const int mvb0 = mvbits_se(m0x - a.pm0[o * 2]) + mvbits_se(m0y - a.pm0[o * 2 + 1]);
  const int mvb1 = mvbits_se(m1x - a.pm1[o * 2]) + mvbits_se(m1y - a.pm1[o * 2 + 1]);
  const int c_bi = satd_bi + lambda * (6 + mvb0 + mvb1);
  const bool no_direct = a.spatial == 1;  // (searched)
  const int dbias = no_direct ? 0 : a.dbias * lambda;
  int mode = 0, best = no_direct ? kNoCostB : c_direct - dbias;  // 0 direct, 1 L0, 2 L1, 3 Bi
  if (c_l0 < best) { mode = 1; best = c_l0; }
  if (c_l1 < best) { mode = 2; best = c_l1; }
  if (c_bi < best) { mode = 3; best = c_bi; }
  int qm[4] = {mode == 0 ? 0 : (mode == 3 ? 1 : mode + 1), 0, 0, 0};  // per quadrant: 0 D, 1 Bi, 2 L0, 3 L1
  qm[1] = qm[2] = qm[3] = qm[0];
  int kind = mode == 0 ? h264::MBK_BDIRECT : h264::MBK_B16x16;
  if (a.bparts) {
    int sum = 0, used0 = 0, used1 = 0, pm[4];
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int cd = no_direct ? kNoCostB : qsat[0][qq] + lambda * 1, cb = qsat[1][qq] + lambda * 7;
      const int c0q = qsat[2][qq] + lambda * 4, c1q = qsat[3][qq] + lambda * 4;
      int m = 0, bc = cd;
      if (cb < bc) { m = 1; bc = cb; }
      if (c0q < bc) { m = 2; bc = c0q; }
      if (c1q < bc) { m = 3; bc = c1q; }
      pm[qq] = m;
      sum += bc;
      used0 |= m == 1 || m == 2;
      used1 |= m == 1 || m == 3;
    }
    const bool anyd = pm[0] == 0 || pm[1] == 0 || pm[2] == 0 || pm[3] == 0;
    const bool h2 = pm[0] == pm[1] && pm[2] == pm[3], v2 = pm[0] == pm[2] && pm[1] == pm[3];
    const bool uni = h2 && v2;
    if (!uni) {
      const int shape_bits = (!anyd && (h2 || v2)) ? 7 : 6;
      const int c_part = sum + lambda * (shape_bits + (used0 ? mvb0 : 0) + (used1 ? mvb1 : 0));
      if (c_part < best) {
        best = c_part;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) qm[qq] = pm[qq];
        kind = (!anyd && h2) ? h264::MBK_B16x8 : ((!anyd && v2) ? h264::MBK_B8x16 : h264::MBK_B8x8);
      }
    }
  }
  // the winner's prediction of this lane's block (direct: pred_out holds it already)
  const int lm = qm[q];
  if (lm != 0) {
    const uint8_t* srcp = lm == 2 ? pr0 : pr1;
#pragma unroll
    for (int y = 0; y < 4; ++y)
      *reinterpret_cast<uint32_t*>(pout + 16 * y) = lm == 1 ? pb[y] : *reinterpret_cast<const uint32_t*>(srcp + 16 * y);
  }
  if (lane == 0) {
    // direct motion per quadrant: temporal from b_direct_mv's vectors (dref: refIdxL0), the
    // fast spatial path's estimate from the record the pre-pass wrote
    uint32_t dw[2][4];
    uint32_t dr8[2];
    if (a.spatial == 2) {
      const uint2 hr = *reinterpret_cast<const uint2*>(&hrec->ref[0][0]);
      const uint4 hm0 = *reinterpret_cast<const uint4*>(&hrec->mv[0][0][0]);
      const uint4 hm1 = *reinterpret_cast<const uint4*>(&hrec->mv[1][0][0]);
      dr8[0] = hr.x;
      dr8[1] = hr.y;
      dw[0][0] = hm0.x; dw[0][1] = hm0.y; dw[0][2] = hm0.z; dw[0][3] = hm0.w;
      dw[1][0] = hm1.x; dw[1][1] = hm1.y; dw[1][2] = hm1.z; dw[1][3] = hm1.w;
    } else {
      const uint4 d0 = reinterpret_cast<const uint4*>(dm)[0], d1 = reinterpret_cast<const uint4*>(dm)[1];
      dr8[0] = drw;
      dr8[1] = 0;
      dw[0][0] = d0.x; dw[0][1] = d0.y; dw[0][2] = d0.z; dw[0][3] = d0.w;
      dw[1][0] = d1.x; dw[1][1] = d1.y; dw[1][2] = d1.z; dw[1][3] = d1.w;
    }
    MbHeader* h = hrec;
    h->kind = static_cast<uint8_t>(kind);
    int sd_ = 0;
    uint32_t w[2][4];
    uint32_t rfw[2] = {0, 0};
    const uint32_t v0 = (static_cast<uint32_t>(m0x) & 0xFFFFu) | (static_cast<uint32_t>(m0y) << 16);
    const uint32_t v1 = (static_cast<uint32_t>(m1x) & 0xFFFFu) | (static_cast<uint32_t>(m1y) << 16);
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int m = qm[qq];
      uint32_t r0, r1;
      if (m == 0) {  // direct (the whole MB or a B_Direct_8x8 quadrant)
        w[0][qq] = dw[0][qq];
        w[1][qq] = dw[1][qq];
        r0 = (dr8[0] >> (8 * qq)) & 255u;
        r1 = (dr8[1] >> (8 * qq)) & 255u;
        sd_ |= 1 << qq;
      } else {
        const bool u0 = m != 3, u1 = m != 2;
        w[0][qq] = u0 ? v0 : 0u;
        w[1][qq] = u1 ? v1 : 0u;
        r0 = u0 ? 0u : 255u;
        r1 = u1 ? 0u : 255u;
      }
      rfw[0] |= r0 << (8 * qq);
      rfw[1] |= r1 << (8 * qq);
    }
    h->sub_direct = static_cast<uint8_t>(kind == h264::MBK_B8x8 ? sd_ : 0);
    *reinterpret_cast<uint2*>(&h->ref[0][0]) = make_uint2(rfw[0], rfw[1]);
    uint4* mvp = reinterpret_cast<uint4*>(&h->mv[0][0][0]);  // 16-byte aligned
    mvp[0] = make_uint4(w[0][0], w[0][1], w[0][2], w[0][3]);
    mvp[1] = make_uint4(w[1][0], w[1][1], w[1][2], w[1][3]);
    a.cost_out[o] = best + (kind == h264::MBK_BDIRECT ? dbias : 0);
  }
}

// K: 0 general (any flags), 1 the direct-only pre-pass, 2 the main pass after the pre-pass
// (have_direct: the default configuration).  K = 2 keeps only the bi-predicted candidate in
// registers -- direct's prediction is already in pred_out, the list predictions are re-read
// from the ME's buffers for the winner, and the direct motion is re-read for the record -- so
// the kernel fits 64 VGPRs (8 waves per SIMD instead of 4 for this chain of dependent loads).
template <int K>
__global__ __launch_bounds__(64) void b_decide(BDecideArgs a) {
  const Geom& g = a.g;
  const int nmb = g.nmb();
  int unit, slot;
  xcd_unit_slot(unit, slot);
  if (!route_active(a.rt, slot, SK_B)) return;
  const int lane = threadIdx.x & 15, wrow = threadIdx.x >> 4;
  const int mb = unit * kDecideMbsPerWave + wrow;
  if (mb >= nmb) return;   // whole rows only: the DPP below stays row-local
  const size_t o = static_cast<size_t>(slot) * nmb + mb;
  const int mx = mb % g.wmb, my = mb / g.wmb;
  const int W = g.W, H = g.H;
  const int by4 = (lane >> 2) * 4, bx4 = (lane & 3) * 4;
  const int X = mx * 16 + bx4, Y = my * 16 + by4;
  const int q = (by4 >> 3) * 2 + (bx4 >> 3);  // 8x8 quadrant of this lane's block
  const size_t yo = static_cast<size_t>(slot) * g.ysize();
  const size_t hps = hp_plane_bytes(W, H);
  const size_t s0 = route_index(a.rt, a.nbuf, slot, RO_L0), s1 = route_index(a.rt, a.nbuf, slot, RO_L1);
  const uint8_t *G0 = a.ref0 + s0 * g.ysize(), *G1 = a.ref1 + s1 * g.ysize(), *H0 = a.hp0 + s0 * hps,
                *H1 = a.hp1 + s1 * hps;
  const int16_t* w1t = a.rt ? a.rt[slot].w1 : nullptr;
  auto w1of = [&](int rr) { return w1t ? static_cast<int>(w1t[rr & 3]) : a.w1[rr & 3]; };
  const int16_t* dm = a.dmv + o * 16;
  const bool donly = (K == 1 || K == 3) ? true : (K == 2 ? false : static_cast<bool>(a.direct_only));
  const bool have_direct = K == 2 ? true : ((K == 1 || K == 3) ? false : static_cast<bool>(a.have_direct));
  const bool sfast = a.spatial == 2;
  const int m0x = donly ? 0 : a.mv0[o * 2], m0y = donly ? 0 : a.mv0[o * 2 + 1];
  const int m1x = donly ? 0 : a.mv1[o * 2], m1y = donly ? 0 : a.mv1[o * 2 + 1];
  uint32_t src[4];
#pragma unroll
  for (int y = 0; y < 4; ++y) src[y] = *reinterpret_cast<const uint32_t*>(a.src_y + yo + static_cast<size_t>(Y + y) * W + X);
  MbHeader* hrec = a.hdr + o;
  // The direct candidate per quadrant and list: refIdx (-1: list unused) and vector.
  //   temporal: the co-located block's scaled motion (b_direct_mv), list 1 from RefPicList1[0];
  //   spatial (fast, spatial == 2): the pre-pass estimates 8.4.1.2.2 from the neighbours'
  //     temporal-direct motion standing in for their final motion (colZeroFlag exact) and
  //     leaves it in the record; the main pass prices it; b_spatial_exact later derives the
  //     exact motion in decoding order and b_spatial_fixup re-predicts where it differs.
  int dref_[2][4], dvx[2][4], dvy[2][4];
  uint32_t drw = 0;  // refIdxL0 of the four temporal-direct quadrants (bytes)
  if (a.dref) drw = *reinterpret_cast<const uint32_t*>(a.dref + o * 4);
  if (K == 2 || K == 3) {
    // the lean passes: nothing here (each lane reads its own quadrant's direct motion, lane 0
    // re-reads it for the record)
  } else if (!sfast) {
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      dref_[0][qq] = (drw >> (8 * qq)) & 255;
      dref_[1][qq] = 0;
      dvx[0][qq] = dm[qq * 2];
      dvy[0][qq] = dm[qq * 2 + 1];
      dvx[1][qq] = dm[8 + qq * 2];
      dvy[1][qq] = dm[8 + qq * 2 + 1];
    }
  } else if (donly) {
    auto tmot = [&](int n, int l, int qq, bool avail) -> NbMv16 {
      NbMv16 m{avail, -1, {0, 0}};
      if (!avail) return m;
      const size_t on = static_cast<size_t>(slot) * nmb + n;
      m.ref = l == 0 ? (a.dref ? static_cast<int>(a.dref[on * 4 + qq]) : 0) : 0;
      m.mv[0] = a.dmv[on * 16 + l * 8 + qq * 2];
      m.mv[1] = a.dmv[on * 16 + l * 8 + qq * 2 + 1];
      return m;
    };
    const bool aA = mx > 0, aB = my > 0, aC = my > 0 && mx + 1 < g.wmb, aD = mx > 0 && my > 0;
    int sref[2], spx[2], spy[2];
#pragma unroll
    for (int l = 0; l < 2; ++l) {
      const NbMv16 A = tmot(mb - 1, l, 1, aA);
      const NbMv16 Bn = tmot(mb - g.wmb, l, 2, aB);
      const NbMv16 C = aC ? tmot(mb - g.wmb + 1, l, 2, true) : tmot(mb - g.wmb - 1, l, 3, aD);
      spatial_pmv(A, Bn, C, sref[l], spx[l], spy[l]);
    }
    const bool zero = sref[0] < 0 && sref[1] < 0;
    const int cz = a.czero ? a.czero[o] : 0;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq)
#pragma unroll
      for (int l = 0; l < 2; ++l) {
        int rf = sref[l], vx = spx[l], vy = spy[l];
        if (zero) {
          rf = 0;
          vx = vy = 0;
        } else if (rf < 0 || (rf == 0 && ((cz >> qq) & 1))) {
          vx = vy = 0;
        }
        dref_[l][qq] = rf;
        dvx[l][qq] = vx;
        dvy[l][qq] = vy;
      }
  } else {  // the pre-pass's estimate, left in the record
    const uint2 hr = *reinterpret_cast<const uint2*>(&hrec->ref[0][0]);
    const uint4 hm0 = *reinterpret_cast<const uint4*>(&hrec->mv[0][0][0]);
    const uint4 hm1 = *reinterpret_cast<const uint4*>(&hrec->mv[1][0][0]);
    const uint32_t w0[4] = {hm0.x, hm0.y, hm0.z, hm0.w}, w1_[4] = {hm1.x, hm1.y, hm1.z, hm1.w};
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      dref_[0][qq] = static_cast<int8_t>((hr.x >> (8 * qq)) & 255u);
      dref_[1][qq] = static_cast<int8_t>((hr.y >> (8 * qq)) & 255u);
      dvx[0][qq] = static_cast<int16_t>(w0[qq] & 0xFFFFu);
      dvy[0][qq] = static_cast<int16_t>(w0[qq] >> 16);
      dvx[1][qq] = static_cast<int16_t>(w1_[qq] & 0xFFFFu);
      dvy[1][qq] = static_cast<int16_t>(w1_[qq] >> 16);
    }
  }
  const bool searched = !donly && a.cost0[o] < kNoCostB && a.cost1[o] < kNoCostB;
  uint8_t* pout = a.pred_out + o * 256 + by4 * 16 + bx4;   // row y at pout + 16 * y
  if (!donly && !searched && have_direct) {
    // gated MB: B_Direct_16x16 with the pre-pass's prediction and cost
    if (lane == 0) {
      hrec->kind = h264::MBK_BDIRECT;
      hrec->sub_direct = 0;
      if (!sfast) {  // (spatial: the estimate is in the record already)
        *reinterpret_cast<uint2*>(&hrec->ref[0][0]) = make_uint2(drw, 0u);
        uint4* mvp = reinterpret_cast<uint4*>(&hrec->mv[0][0][0]);
        const uint4* dv = reinterpret_cast<const uint4*>(dm);  // [list][quadrant][xy] int16
        mvp[0] = dv[0];
        mvp[1] = dv[1];
      }
    }
    return;
  }
  if constexpr (K == 2) {
    b_decide_main(a, src, o, slot, mb, lane, wrow, q, X, Y, pout, hrec, drw, dm, G0, G1, H0, H1, w1of);
    return;
  }
  if constexpr (K == 3) {
    // the temporal-direct pre-pass: this lane's quadrant only
    const int dr = (drw >> (8 * q)) & 255;
    const int dvx0 = dm[q * 2], dvy0 = dm[q * 2 + 1], dvx1 = dm[8 + q * 2], dvy1 = dm[8 + q * 2 + 1];
    const size_t sd = route_index(a.rt, a.nbuf, slot, RO_L0 + (dr & 3));
    const uint8_t *GD = dr ? a.ref0k[dr] + (a.rt ? sd : slot) * g.ysize() : G0,
                  *HD = dr ? a.hp0k[dr] + (a.rt ? sd : slot) * hps : H0;
    const int w1 = w1of(dr);
    uint32_t pd[4];
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      pd[y] = wavg4b(mc4(GD, HD, W, H, X, Y + y, dvx0, dvy0), mc4(G1, H1, W, H, X, Y + y, dvx1, dvy1), w1);
      *reinterpret_cast<uint32_t*>(pout + 16 * y) = pd[y];
    }
    const int sat = sum16(satd4x4_u8(src, pd));
    if (lane == 0) {
      const int qp = clampi(a.qp[slot] + (a.aq ? a.aq[o] : 0), 0, 51);
      a.cost_out[o] = sat + h264::kLambda[qp] * 1;
    }
    return;
  }
  const int dr = dref_[0][q] < 0 ? 0 : dref_[0][q];  // this lane's quadrant
  const bool du0 = dref_[0][q] >= 0, du1 = dref_[1][q] >= 0;
  const size_t sd = route_index(a.rt, a.nbuf, slot, RO_L0 + (dr & 3));
  const uint8_t *GD = dr ? a.ref0k[dr] + (a.rt ? sd : slot) * g.ysize() : G0,
                *HD = dr ? a.hp0k[dr] + (a.rt ? sd : slot) * hps : H0;
  uint32_t pd[4], pb[4], p0w[4], p1w[4];
#pragma unroll
  for (int y = 0; y < 4; ++y) {
    if (!donly && have_direct) {
      pd[y] = *reinterpret_cast<const uint32_t*>(pout + 16 * y);
    } else {
      const uint32_t pl0 = du0 ? mc4(GD, HD, W, H, X, Y + y, dvx[0][q], dvy[0][q]) : 0u;
      const uint32_t pl1 = du1 ? mc4(G1, H1, W, H, X, Y + y, dvx[1][q], dvy[1][q]) : 0u;
      pd[y] = (du0 && du1) ? wavg4b(pl0, pl1, w1of(dr)) : (du0 ? pl0 : pl1);
    }
    if (donly) *reinterpret_cast<uint32_t*>(pout + 16 * y) = pd[y];
    pb[y] = donly ? pd[y]
                  : wavg4b(mc4(G0, H0, W, H, X, Y + y, m0x, m0y), mc4(G1, H1, W, H, X, Y + y, m1x, m1y), w1of(0));
    // candidates: 0 direct, 1 bi (the two ME vectors), 2 L0, 3 L1 (the ME predictions; not
    // needed by the direct-only pre-pass or for MBs the gate left unsearched)
    p0w[y] = searched ? *reinterpret_cast<const uint32_t*>(a.pred0 + o * 256 + (by4 + y) * 16 + bx4) : pd[y];
    p1w[y] = searched ? *reinterpret_cast<const uint32_t*>(a.pred1 + o * 256 + (by4 + y) * 16 + bx4) : pd[y];
  }
  auto blk_satd = [&](const uint32_t* pw) {
    const uint32_t w4[4] = {pw[0], pw[1], pw[2], pw[3]};
    return satd4x4_u8(src, w4);
  };
  // per 8x8 quadrant and candidate: horizontal block pairs by DPP, then the two pair rows of
  // each quadrant from LDS (pair sums at lanes 8 * qy + 4 * {0, 1} + 2 * qx)
  __shared__ int s_pair[kDecideMbsPerWave][4][16];
  const int ncand = donly ? 1 : 4;  // the pre-pass prices direct only
  {
    const int s0 = blk_satd(pd);
    s_pair[wrow][0][lane] = s0 + dpp<kDppQuadXor1>(s0);
    if (!donly) {
      const int s1 = blk_satd(pb), s2 = blk_satd(p0w), s3 = blk_satd(p1w);
      s_pair[wrow][1][lane] = s1 + dpp<kDppQuadXor1>(s1);
      s_pair[wrow][2][lane] = s2 + dpp<kDppQuadXor1>(s2);
      s_pair[wrow][3][lane] = s3 + dpp<kDppQuadXor1>(s3);
    }
  }
  wave_sync();
  int qsat[4][4];  // [candidate][quadrant] (the pre-pass: candidate 0 only)
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int l0 = (qq >> 1) * 8 + (qq & 1) * 2;
      qsat[c][qq] = c < ncand ? s_pair[wrow][c][l0] + s_pair[wrow][c][l0 + 4] : 0;
    }
  const int satd_direct = qsat[0][0] + qsat[0][1] + qsat[0][2] + qsat[0][3];
  const int satd_bi = qsat[1][0] + qsat[1][1] + qsat[1][2] + qsat[1][3];
  const int qp = clampi(a.qp[slot] + (a.aq ? a.aq[o] : 0), 0, 51);
  const int lambda = h264::kLambda[qp];
  // mb_type / motion bits (CABAC-ish): direct "0"; L0 / L1 "10x"; Bi "110000" + two mvds
  const int c_direct = satd_direct + lambda * 1;
  if (donly) {
    if (lane == 0) {
      if (a.spatial == 1) {
        // spatial direct decided in the wavefront (b_spatial_decide): only MBs whose co-located
        // motion is static in every quadrant (temporal direct vectors within +-1, refIdxL0 0)
        // may skip the searches -- there spatial direct predicts zero motion too (colZeroFlag)
        bool stat = drw == 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) stat = stat && dm[k] >= -1 && dm[k] <= 1;
        a.cost_out[o] = stat ? c_direct : kNoCostB;
      } else {
        a.cost_out[o] = c_direct;
      }
      if (sfast) {  // the estimate, for the main pass (and for gated MBs: their motion)
#pragma unroll
        for (int l = 0; l < 2; ++l)
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            hrec->ref[l][qq] = static_cast<int8_t>(dref_[l][qq]);
            hrec->mv[l][qq][0] = static_cast<int16_t>(dvx[l][qq]);
            hrec->mv[l][qq][1] = static_cast<int16_t>(dvy[l][qq]);
          }
      }
    }
    return;
  }
  const int c_l0 = a.cost0[o] + lambda * 3;
  const int c_l1 = a.cost1[o] + lambda * 3;
  const int mvb0 = mvbits_se(m0x - a.pm0[o * 2]) + mvbits_se(m0y - a.pm0[o * 2 + 1]);
  const int mvb1 = mvbits_se(m1x - a.pm1[o * 2]) + mvbits_se(m1y - a.pm1[o * 2 + 1]);
  const int c_bi = satd_bi + lambda * (6 + mvb0 + mvb1);
  const bool no_direct = a.spatial == 1 && searched;
  const int dbias = no_direct ? 0 : a.dbias * lambda;
  int mode = 0, best = no_direct ? kNoCostB : c_direct - dbias;  // 0 direct, 1 L0, 2 L1, 3 Bi
  if (c_l0 < best) { mode = 1; best = c_l0; }
  if (c_l1 < best) { mode = 2; best = c_l1; }
  if (searched && c_bi < best) { mode = 3; best = c_bi; }
  // x264 --partitions b8x8: every quadrant picks its own candidate among the MB's motion
  // (direct quadrant, L0, L1, bi with the two searched vectors): B_16x8 / B_8x16 when the
  // halves agree and no quadrant is direct, else B_8x8 (direct quadrants as B_Direct_8x8).
  // Bits: sub_mb_type (direct 1, L0 / L1 3, bi 5 bins), one full mvd per list in use, 1 bin
  // per later partition repeating it, and the B_8x8 mb_type (~6 bins) / 16x8 pair codes.
  int qm[4] = {mode == 0 ? 0 : (mode == 3 ? 1 : mode + 1), 0, 0, 0};  // per quadrant: 0 D, 1 Bi, 2 L0, 3 L1
  qm[1] = qm[2] = qm[3] = qm[0];
  int kind = mode == 0 ? h264::MBK_BDIRECT : h264::MBK_B16x16;
  if (a.bparts && searched) {
    int sum = 0, used0 = 0, used1 = 0, pm[4];
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int cd = no_direct ? kNoCostB : qsat[0][qq] + lambda * 1, cb = qsat[1][qq] + lambda * 7;
      const int c0q = qsat[2][qq] + lambda * 4, c1q = qsat[3][qq] + lambda * 4;
      int m = 0, bc = cd;
      if (cb < bc) { m = 1; bc = cb; }
      if (c0q < bc) { m = 2; bc = c0q; }
      if (c1q < bc) { m = 3; bc = c1q; }
      pm[qq] = m;
      sum += bc;
      used0 |= m == 1 || m == 2;
      used1 |= m == 1 || m == 3;
    }
    const bool anyd = pm[0] == 0 || pm[1] == 0 || pm[2] == 0 || pm[3] == 0;
    const bool h2 = pm[0] == pm[1] && pm[2] == pm[3], v2 = pm[0] == pm[2] && pm[1] == pm[3];
    const bool uni = h2 && v2;
    if (!uni) {
      const int shape_bits = (!anyd && (h2 || v2)) ? 7 : 6;
      const int c_part = sum + lambda * (shape_bits + (used0 ? mvb0 : 0) + (used1 ? mvb1 : 0));
      if (c_part < best) {
        best = c_part;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) qm[qq] = pm[qq];
        kind = (!anyd && h2) ? h264::MBK_B16x8 : ((!anyd && v2) ? h264::MBK_B8x16 : h264::MBK_B8x8);
      }
    }
  }
  const int lm = qm[q];  // this lane's quadrant
#pragma unroll
  for (int y = 0; y < 4; ++y)
    *reinterpret_cast<uint32_t*>(pout + 16 * y) = lm == 0 ? pd[y] : (lm == 1 ? pb[y] : (lm == 2 ? p0w[y] : p1w[y]));
  if (lane == 0) {
    MbHeader* h = hrec;
    h->kind = static_cast<uint8_t>(kind);
    int sd_ = 0;
    uint32_t w[2][4];
    int8_t rf[2][4];
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int m = qm[qq];
      int x0 = 0, y0 = 0, x1 = 0, y1 = 0;
      if (m == 0) {  // direct (the whole MB or a B_Direct_8x8 quadrant)
        x0 = dvx[0][qq]; y0 = dvy[0][qq]; x1 = dvx[1][qq]; y1 = dvy[1][qq];
        rf[0][qq] = static_cast<int8_t>(dref_[0][qq]);
        rf[1][qq] = static_cast<int8_t>(dref_[1][qq]);
        sd_ |= 1 << qq;
      } else {
        const bool u0 = m != 3, u1 = m != 2;
        if (u0) { x0 = m0x; y0 = m0y; }
        if (u1) { x1 = m1x; y1 = m1y; }
        rf[0][qq] = u0 ? 0 : -1;
        rf[1][qq] = u1 ? 0 : -1;
      }
      w[0][qq] = (static_cast<uint32_t>(x0) & 0xFFFFu) | (static_cast<uint32_t>(y0) << 16);
      w[1][qq] = (static_cast<uint32_t>(x1) & 0xFFFFu) | (static_cast<uint32_t>(y1) << 16);
    }
    h->sub_direct = static_cast<uint8_t>(kind == h264::MBK_B8x8 ? sd_ : 0);
#pragma unroll
    for (int l = 0; l < 2; ++l)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) h->ref[l][qq] = rf[l][qq];
    uint4* mvp = reinterpret_cast<uint4*>(&h->mv[0][0][0]);  // 16-byte aligned
    mvp[0] = make_uint4(w[0][0], w[0][1], w[0][2], w[0][3]);
    mvp[1] = make_uint4(w[1][0], w[1][1], w[1][2], w[1][3]);
    a.cost_out[o] = best + (kind == h264::MBK_BDIRECT ? dbias : 0);
  }
}

// ---------------------------------------------------------------- spatial direct (x264 --direct spatial)
// 8.4.1.2.2: the direct motion of a macroblock follows its neighbours A (left), B (above) and
// C (above-right, else D above-left) in the *current* picture: refIdxLX = MinPositive over
// them, the 16x16 motion-vector predictor of that reference, zeroed per 8x8 quadrant where the
// co-located block of RefPicList1[0] is static (colZeroFlag).  Neighbours' final motion exists
// only in decoding order, so the direct-vs-explicit decision runs in an MB wavefront (one wave
// per MB row, the row above two MBs ahead): b_decide (spatial = 1) leaves each searched
// MB's best explicit candidate (B_L0/L1/Bi 16x16, 16x8, 8x16, B_8x8 without direct quadrants)
// with its cost, and b_spatial_decide derives the exact direct motion from the final
// neighbours, prices it (SATD of its bi-prediction + lambda) and takes it when not dearer.
// MBs the gate left unsearched (b_decide wrote them B_Direct) are always direct.
struct BSpatialArgs {
  Geom g;
  MbHeader* hdr;         // [B, nmb] current picture (in / out)
  const MbHeader* col;   // [B, nmb] RefPicList1[0]'s records
  int* err;
  // encode_inter turns an MB intra when intra_cost < cost (the final decision): such MBs are
  // intra neighbours for the derivation
  const int* intra_cost;
  int* cost;             // in: the explicit candidate's cost (unsearched: the temporal estimate); out: final
  const uint8_t* src_y;
  const uint8_t *ref1, *hp1;
  const uint8_t* ref0k[kMaxRefs];
  const uint8_t* hp0k[kMaxRefs];
  int w1[kMaxRefs];
  uint8_t* pred_out;     // [B, nmb, 256] rewritten for MBs that become direct
  const int* qp;
  const int8_t* aq;
  int bias;              // direct taken when cost_d <= cost_e + bias * lambda
  const SlotRoute* rt;   // routed (route.h): pools for col / ref1 / hp1 / ref0k / hp0k, B slots only
  int nbuf;
};

__device__ __forceinline__ NbMv16 nb16(const MbHeader* h, bool avail, bool intra, int l, int q) {
  NbMv16 n{avail, -1, {0, 0}};
  if (!avail || intra || h264::mbk_is_intra(h->kind)) return n;
  n.ref = h->ref[l][q];
  if (n.ref >= 0) {
    n.mv[0] = h->mv[l][q][0];
    n.mv[1] = h->mv[l][q][1];
  }
  return n;
}

constexpr int kSpatialMaxCols = 480;  // MB columns (8K)
constexpr int kSpatialWaves = 16;  // 16 row chains per slot: the chain (wmb + 2 hmb MBs) bounds it, not the MB count

// packed motion of one quadrant and list: ref (low 8 bits, signed) | mvx << 8 (12 bits) |
// mvy << 20 -- the encoder's vectors stay within +-2048 quarter samples
__device__ __forceinline__ int pk_ref(int v) { return static_cast<int8_t>(v & 255); }
__device__ __forceinline__ int pk_mx(int v) { return (v << 12) >> 20; }
__device__ __forceinline__ int pk_my(int v) { return v >> 20; }

__device__ __forceinline__ NbMv16 nb_packed(bool avail, bool intra, int v) {
  NbMv16 n{avail, -1, {0, 0}};
  if (!avail || intra) return n;
  n.ref = pk_ref(v);
  if (n.ref >= 0) {
    n.mv[0] = pk_mx(v);
    n.mv[1] = pk_my(v);
  }
  return n;
}

// The row above hands its final motion on through LDS, never through global memory: per MB
// column the intra flag and the bottom quadrants (2, 3) of both lists, double-buffered by row
// parity (row y + 1 overwrites column x of row y - 1's entries only after row y has passed
// column x + 1, the last step that reads it).  The left neighbour stays in registers.
// Each wave runs two MB rows in lock step (half-waves: row 2w + 32k in lanes 0..31, the row
// below in lanes 32..63 two MBs behind), 8 samples per lane, so 16 waves cover 32 rows and
// the per-wave serial work (not the wavefront chain) stops bounding the kernel.
__global__ __launch_bounds__(64 * kSpatialWaves) void b_spatial_decide(BSpatialArgs a) {
  const Geom& g = a.g;
  const int slot = blockIdx.x, nmb = g.nmb();
  if (!route_active(a.rt, slot, SK_B)) return;  // uniform per workgroup
  __shared__ int prog[kMaxRows];
  __shared__ int s_res[kSpatialWaves][2][256];
  __shared__ int nbq[2][kSpatialMaxCols][5];  // [row parity][column]: intra, L0 q2, L0 q3, L1 q2, L1 q3
  for (int i = threadIdx.x; i < g.hmb; i += blockDim.x) prog[i] = 0;
  __syncthreads();
  const int w = wave_id(), lane = lane_id();
  const int half = lane >> 5, hl = lane & 31;
  const int r = hl >> 1, c0 = (hl & 1) * 8, q = (r >> 3) * 2 + (c0 >> 3);
  const int W = g.W, Hh = g.H, wmb = g.wmb, hmb = g.hmb;
  const size_t yo = static_cast<size_t>(slot) * g.ysize();
  const size_t hps = hp_plane_bytes(W, Hh);
  size_t sk[kMaxRefs];
#pragma unroll
  for (int k = 0; k < kMaxRefs; ++k) sk[k] = route_index(a.rt, a.nbuf, slot, RO_L0 + k);
  const size_t s1 = route_index(a.rt, a.nbuf, slot, RO_L1);
  const int16_t* w1t = a.rt ? a.rt[slot].w1 : nullptr;
  const bool col_l1 = a.rt && a.rt[slot].col_l1;
  MbHeader* H = a.hdr + static_cast<size_t>(slot) * nmb;
  const MbHeader* C0 = a.col + s1 * nmb;
  const int* IC = a.intra_cost + static_cast<size_t>(slot) * nmb;
  int* CB = a.cost + static_cast<size_t>(slot) * nmb;
  int* res = s_res[w][half];
  const int lam_base = a.qp[slot];
  for (int yu = 2 * w; yu < hmb; yu += 2 * kSpatialWaves) {
    const int y = yu + half;
    const bool row_ok = y < hmb;
    int* cur_row = &nbq[y & 1][0][0];
    const int* up_row = &nbq[(y & 1) ^ 1][0][0];
    int left_intra = 0, left_q1[2] = {0, 0};  // lanes 0 / 32: the left MB's intra flag / quadrant 1
    for (int step = 0; step < wmb + 2; ++step) {
      const int x = half ? step - 2 : step;
      const bool act = row_ok && x >= 0 && x < wmb;
      const int xs = act ? x : 0, ys = act ? y : 0;  // in-range addresses for idle halves
      const int mb = ys * wmb + xs;
      const size_t o = static_cast<size_t>(slot) * nmb + mb;
      // chain-independent inputs first (in flight during the wait)
      const int ic = IC[mb];
      const int cost_e = CB[mb];
      const bool forced = H[mb].kind == h264::MBK_BDIRECT;
      // b_decide's explicit record (kept when direct loses)
      const uint2 href = *reinterpret_cast<const uint2*>(&H[mb].ref[0][0]);
      const uint4 hmv0 = *reinterpret_cast<const uint4*>(&H[mb].mv[0][0][0]);
      const uint4 hmv1 = *reinterpret_cast<const uint4*>(&H[mb].mv[1][0][0]);
      const int lambda = h264::kLambda[clampi(lam_base + (a.aq ? a.aq[o] : 0), 0, 51)];
      const MbHeader& c = C0[mb];
      const uint2 cref = *reinterpret_cast<const uint2*>(&c.ref[0][0]);  // ref[2][4]
      const uint4 cmv = *reinterpret_cast<const uint4*>(&c.mv[0][0][0]);  // list-0 vectors
      const uint4 cmv1 = col_l1 ? *reinterpret_cast<const uint4*>(&c.mv[1][0][0]) : make_uint4(0u, 0u, 0u, 0u);
      const int ckind = c.kind;
      const int X = xs * 16 + c0, Y = ys * 16 + r;
      const uint2 src = *reinterpret_cast<const uint2*>(a.src_y + yo + static_cast<size_t>(Y) * W + X);
      // the upper row waits on the row above (the previous wave's lower row); the lower row's
      // dependency, the upper half two MBs ahead, is met by the lock step
      if (yu > 0) row_wait_lds(prog, yu - 1, min(step + 2, wmb), a.err);
      int pk[4][2] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
      if (hl == 0 && act) {
        const bool aA = x > 0, aB = y > 0, aC = y > 0 && x + 1 < wmb, aD = x > 0 && y > 0;
        const int* uB = up_row + x * 5;
        const int* uC = up_row + (x + 1) * 5;
        const int* uD = up_row + (x - 1) * 5;
        int refs[2], pmv[2][2] = {{0, 0}, {0, 0}};
        for (int l = 0; l < 2; ++l) {
          NbMv16 A = nb_packed(aA, left_intra, left_q1[l]);
          NbMv16 B = aB ? nb_packed(true, uB[0], uB[1 + 2 * l]) : NbMv16{false, -1, {0, 0}};
          NbMv16 C = aC ? nb_packed(true, uC[0], uC[1 + 2 * l])
                        : (aD ? nb_packed(true, uD[0], uD[2 + 2 * l]) : NbMv16{false, -1, {0, 0}});
          auto minpos = [](int p, int qv) { return (p >= 0 && qv >= 0) ? min(p, qv) : max(p, qv); };
          refs[l] = minpos(A.ref, minpos(B.ref, C.ref));
          if (refs[l] < 0) continue;
          if (!B.avail && !C.avail && A.avail) {
            B = A;
            C = A;
          }
          const int rr = refs[l];
          const int match = (A.ref == rr) + (B.ref == rr) + (C.ref == rr);
          if (match == 1) {
            const NbMv16& m = A.ref == rr ? A : (B.ref == rr ? B : C);
            pmv[l][0] = m.mv[0];
            pmv[l][1] = m.mv[1];
          } else {
            pmv[l][0] = med3i(A.mv[0], B.mv[0], C.mv[0]);
            pmv[l][1] = med3i(A.mv[1], B.mv[1], C.mv[1]);
          }
        }
        const bool zero = refs[0] < 0 && refs[1] < 0;
        const bool cintra = h264::mbk_is_intra(ckind);
        const uint32_t cmw[4] = {cmv.x, cmv.y, cmv.z, cmv.w};
        const uint32_t cmw1[4] = {cmv1.x, cmv1.y, cmv1.z, cmv1.w};
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          // 8.4.1.2.1: the co-located block's list-0 motion, or its list-1 motion when it has
          // none (only a B picture -- b-pyramid -- can be list-1 only)
          const int cr0 = static_cast<int8_t>((cref.x >> (8 * qq)) & 255u);
          const bool use1 = col_l1 && cr0 < 0;
          const int cr = use1 ? static_cast<int8_t>((cref.y >> (8 * qq)) & 255u) : cr0;
          const uint32_t cw_ = use1 ? cmw1[qq] : cmw[qq];
          const int cx = static_cast<int16_t>(cw_ & 0xFFFFu), cy = static_cast<int16_t>(cw_ >> 16);
          const bool col_zero = !cintra && cr == 0 && abs(cx) <= 1 && abs(cy) <= 1;
#pragma unroll
          for (int l = 0; l < 2; ++l) {
            int rf = refs[l], mx = pmv[l][0], my = pmv[l][1];
            if (zero) {
              rf = 0;
              mx = my = 0;
            } else if (rf < 0 || (rf == 0 && col_zero)) {
              mx = my = 0;
            }
            pk[qq][l] = (rf & 255) | ((mx & 4095) << 8) | (my << 20);
          }
        }
      }
      int mine[2] = {0, 0};
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
#pragma unroll
        for (int l = 0; l < 2; ++l) {
          const int vu = __builtin_amdgcn_readlane(pk[qq][l], 0), vl = __builtin_amdgcn_readlane(pk[qq][l], 32);
          if (qq == q) mine[l] = half ? vl : vu;
        }
      const int r0 = pk_ref(mine[0]), r1 = pk_ref(mine[1]);
      uint32_t pw[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        uint32_t p0 = 0, p1 = 0;
        if (r0 >= 0)
          p0 = mc4(a.ref0k[r0 & 3] + sk[r0 & 3] * g.ysize(), a.hp0k[r0 & 3] + sk[r0 & 3] * hps, W, Hh, X + 4 * k, Y,
                   pk_mx(mine[0]), pk_my(mine[0]));
        if (r1 >= 0) p1 = mc4(a.ref1 + s1 * g.ysize(), a.hp1 + s1 * hps, W, Hh, X + 4 * k, Y, pk_mx(mine[1]), pk_my(mine[1]));
        pw[k] = (r0 >= 0 && r1 >= 0) ? wavg4b(p0, p1, w1t ? static_cast<int>(w1t[r0 & 3]) : a.w1[r0 & 3])
                                     : (r0 >= 0 ? p0 : p1);
      }
      const uint32_t sw[2] = {src.x, src.y};
#pragma unroll
      for (int k = 0; k < 8; ++k)
        res[r * 16 + c0 + k] = static_cast<int>((sw[k >> 2] >> (8 * (k & 3))) & 255u) -
                               static_cast<int>((pw[k >> 2] >> (8 * (k & 3))) & 255u);
      wave_sync();
      int satd = 0;
      if (hl < 16) {  // block hl of this half's MB; rows of 16 lanes sum below
        const int bx = (hl & 3) * 4, by = (hl >> 2) * 4;
        int rr[16];
#pragma unroll
        for (int yy = 0; yy < 4; ++yy)
#pragma unroll
          for (int xx = 0; xx < 4; ++xx) rr[yy * 4 + xx] = res[(by + yy) * 16 + bx + xx];
        satd = h264::satd4x4(rr);
      }
      const int ssum = sum16(satd);
      const int su = __builtin_amdgcn_readlane(ssum, 0), sl = __builtin_amdgcn_readlane(ssum, 32);
      const int cost_d = (half ? sl : su) + lambda;
      const bool take = act && (forced || cost_d <= cost_e + a.bias * lambda);
      const int final_cost = take ? cost_d : cost_e;
      const bool intra = ic < final_cost;  // encode_inter's rule
      if (take) *reinterpret_cast<uint2*>(a.pred_out + o * 256 + r * 16 + c0) = make_uint2(pw[0], pw[1]);
      if (hl == 0 && act) {
        // this MB's final motion: the direct one, else the explicit record b_decide wrote
        int fin[4][2];
        if (take) {
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            fin[qq][0] = pk[qq][0];
            fin[qq][1] = pk[qq][1];
          }
        } else {
          const uint32_t hm[2][4] = {{hmv0.x, hmv0.y, hmv0.z, hmv0.w}, {hmv1.x, hmv1.y, hmv1.z, hmv1.w}};
          const uint32_t hr[2] = {href.x, href.y};
#pragma unroll
          for (int qq = 0; qq < 4; ++qq)
#pragma unroll
            for (int l = 0; l < 2; ++l) {
              const int mx = static_cast<int16_t>(hm[l][qq] & 0xFFFFu), my = static_cast<int16_t>(hm[l][qq] >> 16);
              fin[qq][l] = static_cast<int>((hr[l] >> (8 * qq)) & 255u) | ((mx & 4095) << 8) | (my << 20);
            }
        }
        int* e = cur_row + x * 5;
        e[0] = intra;
        e[1] = fin[2][0];
        e[2] = fin[3][0];
        e[3] = fin[2][1];
        e[4] = fin[3][1];
        left_intra = intra;
        left_q1[0] = fin[1][0];
        left_q1[1] = fin[1][1];
        if (take) {
          MbHeader& h = H[mb];
          h.kind = h264::MBK_BDIRECT;
          h.sub_direct = 0;
#pragma unroll
          for (int qq = 0; qq < 4; ++qq)
#pragma unroll
            for (int l = 0; l < 2; ++l) {
              h.ref[l][qq] = static_cast<int8_t>(pk_ref(pk[qq][l]));
              h.mv[l][qq][0] = static_cast<int16_t>(pk_mx(pk[qq][l]));
              h.mv[l][qq][1] = static_cast<int16_t>(pk_my(pk[qq][l]));
            }
          CB[mb] = cost_d;
        }
      }
      // publish: the lower half's own next step reads the upper half's LDS entries in program
      // order; the next wave's upper row waits on this wave's lower row (prog)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
      wave_sync();
      if (hl == 0 && act) __hip_atomic_store(prog + y, x + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
}

// ---------------------------------------------------------------- spatial direct, fast path
// b_decide (spatial = 2) prices direct in parallel with an estimate of the spatial motion and
// decides every MB; what it cannot know is the neighbours' *final* motion, which 8.4.1.2.2
// derives the direct motion from.  b_spatial_exact walks each slot's MBs in decoding order --
// integer work only, one lane per MB row (row y two MBs behind row y - 1, all rows of a slot in
// one workgroup in lock step, a barrier per step) -- and writes the exact motion of every
// direct MB / B_Direct_8x8 quadrant into its record, flagging the MBs whose motion changed;
// b_spatial_fixup then re-predicts those (fully parallel).  The decisions and costs stay as
// b_decide made them (encode_inter's intra-vs-inter rule, which the derivation must agree on,
// reads the same costs), so the bitstream is exact while the serial chain costs microseconds
// instead of b_spatial_decide's SATD per MB on the chain.
struct BSpatialExactArgs {
  Geom g;
  MbHeader* hdr;          // [B, nmb] in / out
  const int* intra_cost;  // [B, nmb]: an MB turns intra when intra_cost < cost (encode_inter)
  const int* cost;        // [B, nmb]
  const uint8_t* czero;   // [B, nmb] colZeroFlag bits (b_direct_mv)
  uint8_t* fix;           // [B, nmb] out: 1 = the direct motion changed, re-predict; 2 = made explicit
  const SlotRoute* rt;
  int slice_rows;         // MB rows per slice (0: one slice): no neighbours above a slice's first row
  // quarter-sample tolerance: a direct quadrant whose exact motion is further than this from
  // the estimate b_decide priced keeps the estimate as explicit motion; -1 = never (the direct
  // MB is always re-predicted with the exact motion)
  int tol;
};

constexpr int kExactWaves = 5;  // one lane per MB row: 320 >= 8K's 270 rows

__global__ __launch_bounds__(64 * kExactWaves) void b_spatial_exact(BSpatialExactArgs a) {
  const Geom& g = a.g;
  const int slot = blockIdx.x, nmb = g.nmb(), wmb = g.wmb, hmb = g.hmb;
  if (!route_active(a.rt, slot, SK_B)) return;  // uniform per workgroup
  __shared__ int nbq[2][kSpatialMaxCols][5];      // [row parity][column]: intra, L0 q2, L0 q3, L1 q2, L1 q3
  const int y = threadIdx.x;
  const bool row_ok = y < hmb;
  MbHeader* H = a.hdr + static_cast<size_t>(slot) * nmb;
  const int* IC = a.intra_cost + static_cast<size_t>(slot) * nmb;
  const int* CB = a.cost + static_cast<size_t>(slot) * nmb;
  const uint8_t* CZ = a.czero + static_cast<size_t>(slot) * nmb;
  uint8_t* FX = a.fix + static_cast<size_t>(slot) * nmb;
  int* cur_row = &nbq[y & 1][0][0];
  const int* up_row = &nbq[(y & 1) ^ 1][0][0];
  int left_intra = 0, left_q1[2] = {0, 0};
  const int nsteps = wmb + 2 * (hmb - 1);
  for (int step = 0; step < nsteps; ++step) {
    const int x = step - 2 * y;
    if (row_ok && x >= 0 && x < wmb) {
      const int mb = y * wmb + x;
      MbHeader& h = H[mb];
      const int kind = h.kind;
      const bool intra = IC[mb] < CB[mb];
      const int sdir = kind == h264::MBK_BDIRECT ? 15 : (kind == h264::MBK_B8x8 ? h.sub_direct : 0);
      int fin[4][2];
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
#pragma unroll
        for (int l = 0; l < 2; ++l)
          fin[qq][l] = (h.ref[l][qq] & 255) | ((h.mv[l][qq][0] & 4095) << 8) | (h.mv[l][qq][1] << 20);
      bool changed = false, converted = false;
      if (!intra && sdir) {
        const bool top = y > 0 && (a.slice_rows <= 0 || y % a.slice_rows != 0);
        const bool aA = x > 0, aB = top, aC = top && x + 1 < wmb, aD = x > 0 && top;
        int refs[2], pmv[2][2];
#pragma unroll
        for (int l = 0; l < 2; ++l) {
          const NbMv16 A = nb_packed(aA, left_intra, left_q1[l]);
          const NbMv16 Bn = aB ? nb_packed(true, up_row[x * 5], up_row[x * 5 + 1 + 2 * l]) : NbMv16{false, -1, {0, 0}};
          const NbMv16 C = aC ? nb_packed(true, up_row[(x + 1) * 5], up_row[(x + 1) * 5 + 1 + 2 * l])
                              : (aD ? nb_packed(true, up_row[(x - 1) * 5], up_row[(x - 1) * 5 + 2 + 2 * l])
                                    : NbMv16{false, -1, {0, 0}});
          spatial_pmv(A, Bn, C, refs[l], pmv[l][0], pmv[l][1]);
        }
        const bool zero = refs[0] < 0 && refs[1] < 0;
        const int cz = CZ[mb];
        int ex[4][2][3];    // exact motion of the direct quadrants: ref, mvx, mvy per list
        int conv = 0;       // quadrants whose exact motion is off the estimate by more than tol
        int moved = 0;      // quadrants whose exact motion differs at all
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          if (!((sdir >> qq) & 1)) continue;
#pragma unroll
          for (int l = 0; l < 2; ++l) {
            int rf = refs[l], vx = pmv[l][0], vy = pmv[l][1];
            if (zero) {
              rf = 0;
              vx = vy = 0;
            } else if (rf < 0 || (rf == 0 && ((cz >> qq) & 1))) {
              vx = vy = 0;
            }
            ex[qq][l][0] = rf;
            ex[qq][l][1] = vx;
            ex[qq][l][2] = vy;
            const int er = h.ref[l][qq], evx = h.mv[l][qq][0], evy = h.mv[l][qq][1];
            if (((rf & 255) | ((vx & 4095) << 8) | (vy << 20)) != fin[qq][l]) moved |= 1 << qq;
            if (rf != er || (rf >= 0 && (abs(vx - evx) > a.tol || abs(vy - evy) > a.tol))) conv |= 1 << qq;
          }
        }
        if (conv && a.tol >= 0) {
          converted = true;
          // The prediction b_decide priced (and encode_inter will subtract) is the estimate's:
          // instead of re-predicting with motion nobody priced, the MB keeps the estimated
          // motion and codes it explicitly -- B_L0 / L1 / Bi partitions of the shape the
          // quadrant motion allows (B_Direct_16x16) or explicit 8x8 sub-blocks (B_8x8).  Its
          // final motion (what later MBs derive from) is then the estimate, already in `fin`.
          if (kind == h264::MBK_BDIRECT) {
            auto same = [&](int p, int q) { return fin[p][0] == fin[q][0] && fin[p][1] == fin[q][1]; };
            h.kind = (same(0, 1) && same(2, 3)) ? (same(0, 2) ? h264::MBK_B16x16 : h264::MBK_B16x8)
                                                : ((same(0, 2) && same(1, 3)) ? h264::MBK_B8x16 : h264::MBK_B8x8);
            h.sub_direct = 0;
            moved = 0;  // no quadrant keeps direct
          } else {
            h.sub_direct = static_cast<uint8_t>(h.sub_direct & ~conv);
            moved &= ~conv;
          }
        }
        // the remaining direct quadrants take the exact motion (re-predicted by b_spatial_fixup)
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          if (!((moved >> qq) & 1)) continue;
          changed = true;
#pragma unroll
          for (int l = 0; l < 2; ++l) {
            const int rf = ex[qq][l][0], vx = ex[qq][l][1], vy = ex[qq][l][2];
            fin[qq][l] = (rf & 255) | ((vx & 4095) << 8) | (vy << 20);
            h.ref[l][qq] = static_cast<int8_t>(rf);
            h.mv[l][qq][0] = static_cast<int16_t>(vx);
            h.mv[l][qq][1] = static_cast<int16_t>(vy);
          }
        }
      }
      FX[mb] = changed ? 1 : (converted ? 2 : 0);  // 2: explicit now, prediction unchanged
      int* e = cur_row + x * 5;
      e[0] = intra;
      e[1] = fin[2][0];
      e[2] = fin[3][0];
      e[3] = fin[2][1];
      e[4] = fin[3][1];
      left_intra = intra;
      left_q1[0] = fin[1][0];
      left_q1[1] = fin[1][1];
    }
    __syncthreads();
  }
}

// Re-prediction of the direct quadrants whose exact motion differs from b_decide's estimate.
struct BSpatialFixArgs {
  Geom g;
  const MbHeader* hdr;
  const uint8_t* fix;
  const uint8_t *ref0, *hp0;  // pools [B, nbuf, plane] (every list-0 entry, by route)
  const uint8_t *ref1, *hp1;
  uint8_t* pred_out;
  const SlotRoute* rt;
  int nbuf;
};

__global__ __launch_bounds__(64) void b_spatial_fixup(BSpatialFixArgs a) {
  const Geom& g = a.g;
  const int nmb = g.nmb();
  int mb, slot;
  xcd_unit_slot(mb, slot);
  if (!route_active(a.rt, slot, SK_B)) return;
  const size_t o = static_cast<size_t>(slot) * nmb + mb;
  if (a.fix[o] != 1) return;  // wave-uniform
  const int lane = threadIdx.x;
  const int mx = mb % g.wmb, my = mb / g.wmb;
  const int W = g.W, H = g.H;
  const int r = lane >> 2, c0 = (lane & 3) * 4;
  const int X = mx * 16 + c0, Y = my * 16 + r;
  const int q = (r >> 3) * 2 + (c0 >> 3);
  const MbHeader& h = a.hdr[o];
  const bool dq = h.kind == h264::MBK_BDIRECT || (h.kind == h264::MBK_B8x8 && ((h.sub_direct >> q) & 1));
  if (!dq) return;  // (lane-divergent exit after the last wave-wide step)
  const size_t hps = hp_plane_bytes(W, H);
  const int r0 = h.ref[0][q], r1 = h.ref[1][q];
  uint32_t p0 = 0, p1 = 0;
  if (r0 >= 0) {
    const size_t s0 = route_index(a.rt, a.nbuf, slot, RO_L0 + (r0 & 3));
    p0 = mc4(a.ref0 + s0 * g.ysize(), a.hp0 + s0 * hps, W, H, X, Y, h.mv[0][q][0], h.mv[0][q][1]);
  }
  if (r1 >= 0) {
    const size_t s1 = route_index(a.rt, a.nbuf, slot, RO_L1);
    p1 = mc4(a.ref1 + s1 * g.ysize(), a.hp1 + s1 * hps, W, H, X, Y, h.mv[1][q][0], h.mv[1][q][1]);
  }
  const int w1 = a.rt ? a.rt[slot].w1[r0 & 3] : 32;
  *reinterpret_cast<uint32_t*>(a.pred_out + o * 256 + r * 16 + c0) =
      (r0 >= 0 && r1 >= 0) ? wavg4b(p0, p1, w1) : (r0 >= 0 ? p0 : p1);
}

// ---------------------------------------------------------------- P_Skip-aware vector choice
// ME prices vectors against a temporal predictor, so on noisy content neighbouring MBs of
// one uniform motion pick slightly different quarter-sample vectors and none of them can
// be coded as P_Skip (mv == the skip predictor, no residual) -- every MB pays mb_type +
// mvd bins even where the residual quantises to zero.  This pass (Jacobi, over the whole
// picture in parallel) offers each MB the P_Skip predictor computed from its neighbours'
// current vectors (clause 8.4.1.1: 0 if A or B is unavailable or a zero vector, else the
// median of A, B, C/D) and takes it when SATD(skip prediction) <= SATD(own vector) +
// lambda * mvd bits.  Two passes let a uniform field settle; the writer still derives
// skip exactly from the final records.
struct PRefineArgs {
  Geom g;
  const uint8_t* src_y;
  const uint8_t* ref;       // G plane of the reference
  const uint8_t* hp;        // its half-sample planes
  const int16_t* mv_in;     // [B, nmb, 2]
  int16_t* mv_out;          // [B, nmb, 2]
  int* cost;                // [B, nmb] ME cost (SATD + lambda * bits vs pm), updated in place
  const int16_t* pm;        // [B, nmb, 2] the ME's predictor (to recover the SATD part of cost)
  uint8_t* pred;            // [B, nmb, 256] luma prediction, rewritten for MBs that switch
  const int* qp;
  const int8_t* aq;
  const SlotRoute* rt;      // routed (route.h): ref / hp are pools, P slots' RefPicList0[0]
  int nbuf;
  // Jacobi passes after the first (p_mv_refine): which MBs changed their vector in the previous
  // pass (nullable: every MB is evaluated).  An MB whose own and whose neighbours' (A, B, C,
  // D) vectors stayed put would derive the same skip predictor at the same cost -- it only
  // copies its vector through.  chg_out: this pass's changes
  const uint8_t* chg_in;
  uint8_t* chg_out;
};

__device__ __forceinline__ int median3(int a, int b, int c) { return max(min(a, b), min(max(a, b), c)); }

// Four MBs per wave, one 16-lane row each: a lane prices one 4x4 block of its MB straight
// from registers (no LDS) and the row sums them with DPP.  The kernel is a short chain of
// dependent loads (neighbour vectors -> prediction -> cost) per MB, so it is bound by how
// many MBs are in flight; one MB per wave left it at ~1.5 ms per launch at the headline.
constexpr int kRefineMbsPerWave = 4;

__global__ __launch_bounds__(64) void p_mv_refine(PRefineArgs a) {
  const Geom& g = a.g;
  const int nmb = g.nmb();
  int unit, slot;
  xcd_unit_slot(unit, slot);
  if (!route_active(a.rt, slot, SK_P)) return;
  const int lane = threadIdx.x & 15;
  const int mb = unit * kRefineMbsPerWave + (threadIdx.x >> 4);
  if (mb >= nmb) return;   // whole 16-lane rows only: the DPP sums below stay row-local
  const size_t o = static_cast<size_t>(slot) * nmb + mb;
  const int mx = mb % g.wmb, my = mb / g.wmb;
  const int16_t* mv = a.mv_in + static_cast<size_t>(slot) * nmb * 2;
  const int cx = mv[mb * 2], cy = mv[mb * 2 + 1];
  if (a.chg_in) {  // row-uniform
    const uint8_t* c = a.chg_in + static_cast<size_t>(slot) * nmb;
    bool any = c[mb];
    if (mx > 0) any = any || c[mb - 1];
    if (my > 0) any = any || c[mb - g.wmb] || (mx + 1 < g.wmb && c[mb - g.wmb + 1]) || (mx > 0 && c[mb - g.wmb - 1]);
    if (!any) {
      if (lane == 0) {
        a.mv_out[o * 2] = static_cast<int16_t>(cx);
        a.mv_out[o * 2 + 1] = static_cast<int16_t>(cy);
        if (a.chg_out) a.chg_out[o] = 0;
      }
      return;
    }
  }
  // P_Skip predictor from the neighbours' current vectors (all list 0, ref 0)
  const bool hasA = mx > 0, hasB = my > 0, hasC = my > 0 && mx < g.wmb - 1, hasD = mx > 0 && my > 0;
  int sx = 0, sy = 0;
  if (hasA && hasB) {
    const int ax = mv[(mb - 1) * 2], ay = mv[(mb - 1) * 2 + 1];
    const int bx = mv[(mb - g.wmb) * 2], by = mv[(mb - g.wmb) * 2 + 1];
    if (!((ax == 0 && ay == 0) || (bx == 0 && by == 0))) {
      const int cn = hasC ? mb - g.wmb + 1 : (hasD ? mb - g.wmb - 1 : -1);
      const int ccx = cn >= 0 ? mv[cn * 2] : 0, ccy = cn >= 0 ? mv[cn * 2 + 1] : 0;
      sx = median3(ax, bx, ccx);
      sy = median3(ay, by, ccy);
    }
  }
  if (sx == cx && sy == cy) {
    if (lane == 0) {
      a.mv_out[o * 2] = static_cast<int16_t>(cx);
      a.mv_out[o * 2 + 1] = static_cast<int16_t>(cy);
      if (a.chg_out) a.chg_out[o] = 0;
    }
    return;
  }
  const int W = g.W, H = g.H;
  const int bx4 = (lane & 3) * 4, by4 = (lane >> 2) * 4;
  const int X = mx * 16 + bx4, Y = my * 16 + by4;
  const size_t yo = static_cast<size_t>(slot) * g.ysize();
  const size_t s0 = route_index(a.rt, a.nbuf, slot, RO_L0);
  const uint8_t* G0 = a.ref + s0 * g.ysize();
  const uint8_t* H0 = a.hp + s0 * hp_plane_bytes(W, H);
  uint32_t ps[4], sw[4];
#pragma unroll
  for (int y = 0; y < 4; ++y) {
    sw[y] = *reinterpret_cast<const uint32_t*>(a.src_y + yo + static_cast<size_t>(Y + y) * W + X);
    ps[y] = mc4(G0, H0, W, H, X, Y + y, sx, sy);
  }
  const int satd = sum16(satd4x4_u8(sw, ps));
  const int qp = clampi(a.qp[slot] + (a.aq ? a.aq[o] : 0), 0, 51);
  const int lambda = h264::kLambda[qp];
  const int pmx = a.pm ? a.pm[o * 2] : 0, pmy = a.pm ? a.pm[o * 2 + 1] : 0;
  const int satd_me = a.cost[o] - lambda * (mvbits_se(cx - pmx) + mvbits_se(cy - pmy));
  const int c_me = satd_me + lambda * (mvbits_se(cx - sx) + mvbits_se(cy - sy) + 1);
  const bool take = satd <= c_me;
  if (take) {
#pragma unroll
    for (int y = 0; y < 4; ++y) *reinterpret_cast<uint32_t*>(a.pred + o * 256 + (by4 + y) * 16 + bx4) = ps[y];
  }
  if (lane == 0) {
    a.mv_out[o * 2] = static_cast<int16_t>(take ? sx : cx);
    a.mv_out[o * 2 + 1] = static_cast<int16_t>(take ? sy : cy);
    if (take) a.cost[o] = satd + lambda * (mvbits_se(sx - pmx) + mvbits_se(sy - pmy));
    if (a.chg_out) a.chg_out[o] = take;  // (take moves the vector: sx, sy != cx, cy here)
  }
}


// 16-lane-row form (four blocks per wave): this lane's 4x4 block = rows by4..by4+3 of src / pw,
// summed over the row with DPP (every lane of a row holds the same block's total)
__device__ __forceinline__ int satd16_rows(const uint32_t* src, const uint32_t* pw) {
  const uint32_t s4[4] = {src[0], src[1], src[2], src[3]}, p4[4] = {pw[0], pw[1], pw[2], pw[3]};
  return sum16(satd4x4_u8(s4, p4));
}

// ---- HEVC merge-aware vector choice (the H.265 analogue of p_mv_refine): after the 16x16
// search each block is offered the current vectors of its spatial merge neighbours (A1 left,
// B1 above, B0 above-right, A0 below-left, B2 above-left; 8.5.3.2.3) and the zero vector;
// the cheapest by SATD + lambda * (merge_idx bits) replaces the searched vector when it beats
// the search's SATD + lambda * mvd bits, so the CABAC writer can code the CU as merge / skip.
// Jacobi pass: reads mv_in, writes mv_out.  (The candidates approximate the normative merge
// list on the 16x16 grid; the writer codes AMVP whenever the vector is not in the real list.)
__global__ __launch_bounds__(64) void hevc_merge_refine(PRefineArgs a) {
  const Geom& g = a.g;
  const int nmb = g.nmb();
  int unit, slot;
  xcd_unit_slot(unit, slot);
  const int lane = threadIdx.x & 15;   // four blocks per wave, as p_mv_refine
  const int mb = unit * kRefineMbsPerWave + (threadIdx.x >> 4);
  if (mb >= nmb) return;
  const size_t o = static_cast<size_t>(slot) * nmb + mb;
  const int mx = mb % g.wmb, my = mb / g.wmb;
  const int16_t* mv = a.mv_in + static_cast<size_t>(slot) * nmb * 2;
  const int cx = mv[mb * 2], cy = mv[mb * 2 + 1];
  int kx[6], ky[6], nk = 0;
  auto add = [&](bool ok, int n) {
    if (!ok) return;
    const int vx = mv[n * 2], vy = mv[n * 2 + 1];
    for (int j = 0; j < nk; ++j)
      if (kx[j] == vx && ky[j] == vy) return;
    kx[nk] = vx;
    ky[nk] = vy;
    ++nk;
  };
  add(mx > 0, mb - 1);                              // A1
  add(my > 0, mb - g.wmb);                          // B1
  add(my > 0 && mx < g.wmb - 1, mb - g.wmb + 1);    // B0
  add(mx > 0 && my < g.hmb - 1, mb + g.wmb - 1);    // A0
  add(mx > 0 && my > 0, mb - g.wmb - 1);            // B2
  {
    bool z = false;
    for (int j = 0; j < nk; ++j) z |= kx[j] == 0 && ky[j] == 0;
    if (!z) {
      kx[nk] = 0;
      ky[nk] = 0;
      ++nk;
    }
  }
  const int qp = clampi(a.qp[slot] + (a.aq ? a.aq[o] : 0), 0, 51);
  const int lambda = h264::kLambda[qp];
  const int pmx = a.pm ? a.pm[o * 2] : 0, pmy = a.pm ? a.pm[o * 2 + 1] : 0;
  const int c_me = a.cost[o];  // SATD + lambda * mvd bits against the search predictor
  const int W = g.W, H = g.H;
  const int X = mx * 16 + (lane & 3) * 4, Y = my * 16 + (lane >> 2) * 4;
  const size_t yo = static_cast<size_t>(slot) * g.ysize();
  const uint8_t* G0 = a.ref + yo;
  const uint8_t* H0 = a.hp + static_cast<size_t>(slot) * 3 * (W + 2 * kHpMargin) * (H + 2 * kHpMargin);
  uint32_t src[4];
#pragma unroll
  for (int y = 0; y < 4; ++y) src[y] = *reinterpret_cast<const uint32_t*>(a.src_y + yo + static_cast<size_t>(Y + y) * W + X);
  int best = c_me, bx_ = cx, by_ = cy;
  for (int j = 0; j < nk; ++j) {
    if (kx[j] == cx && ky[j] == cy) {  // the searched vector is itself a merge candidate
      best = min(best, c_me - lambda * (mvbits_se(cx - pmx) + mvbits_se(cy - pmy)) + lambda * (1 + j));
      continue;
    }
    uint32_t ps[4];
#pragma unroll
    for (int y = 0; y < 4; ++y) ps[y] = mc4(G0, H0, W, H, X, Y + y, kx[j], ky[j]);
    const int satd = satd16_rows(src, ps);
    const int cst = satd + lambda * (1 + j);  // merge_flag + truncated-unary merge_idx
    if (cst < best) {
      best = cst;
      bx_ = kx[j];
      by_ = ky[j];
    }
  }
  if (lane == 0) {
    a.mv_out[o * 2] = static_cast<int16_t>(bx_);
    a.mv_out[o * 2 + 1] = static_cast<int16_t>(by_);
    a.cost[o] = best;
  }
}

// ---- HEVC B pictures (x265 --bframes): the two searches (list 0 against the previous
// anchor, list 1 against the next) become one motion per 16x16 block -- L0, L1 or bi --
// and then merge-aware passes like hevc_merge_refine, over B motion (direction + two
// vectors).  Motion per block: mvb [B, nmb, 4] = (L0 x, y, L1 x, y), dir [B, nmb] (CuDir),
// cost = SATD + lambda * bits and bits (so a pass can recover the SATD part).
struct HevcBArgs {
  Geom g;
  const uint8_t* src_y;
  const uint8_t *ref0, *ref1;   // 8-bit proxies of RefPicList0[0] / RefPicList1[0]
  const uint8_t *hp0, *hp1;     // their half-sample planes
  const int16_t *mv0, *mv1;     // [B, nmb, 2] searched vectors
  const int *cost0, *cost1;     // their costs against pm0 / pm1
  const int16_t *pm0, *pm1;     // search predictors
  const int16_t* tmv;           // [B, nmb, 4] temporal merge candidate (both lists)
  const uint8_t* tdir;          // [B, nmb] its direction (0: none)
  const int16_t* mvb_in;        // [B, nmb, 4]
  const uint8_t* dir_in;        // [B, nmb]
  int16_t* mvb_out;
  uint8_t* dir_out;
  int* cost;                    // [B, nmb]
  int* bits;                    // [B, nmb]
  const int* qp;
  const int8_t* aq;
  int bslice;                   // 0: P picture (list 0 only)
  int max_merge;                // MaxNumMergeCand
  int ctu_shift;                // log2(CTU size / 16): 1 for 32x32 CTBs, 2 for 64x64 CTUs
  // merge passes: blocks whose motion the previous pass changed (nullable: every block is
  // re-evaluated); a block whose own and whose neighbours' motion stayed put would rebuild the
  // same list at the same costs, so it only copies its motion through
  const uint8_t* chg_in;
  uint8_t* chg_out;
  // x265 --ref: P pictures with nref0 > 1 active list-0 pictures.  A motion's direction byte
  // carries its list-0 refIdx in bits 2-3 (CuDir in bits 0-1); xref / xhp are the proxies and
  // half-sample planes of RefPicList0[1 ..], and the P init pass picks per block among the
  // list-0[0] search (mv0 / cost0 / pm0) and the farther searches xmv / xcost / xpm
  // ([nref0 - 1, B, nmb, ...]; xcost kNoCost = not searched) at cost + lambda * ref_idx bins
  int nref0;
  const uint8_t* xref[3];
  const uint8_t* xhp[3];
  const int16_t* xmv;
  const int* xcost;
  const int16_t* xpm;
};

// RefPicList0[r]'s 8-bit proxy / half-sample planes (constant indices only: no scratch)
__device__ __forceinline__ const uint8_t* l0_ref(const HevcBArgs& a, int r) {
  return r == 0 ? a.ref0 : (r == 1 ? a.xref[0] : (r == 2 ? a.xref[1] : a.xref[2]));
}
__device__ __forceinline__ const uint8_t* l0_hp(const HevcBArgs& a, int r) {
  return r == 0 ? a.hp0 : (r == 1 ? a.xhp[0] : (r == 2 ? a.xhp[1] : a.xhp[2]));
}
// ref_idx_l0 bins (TR, cMax nref - 1)
__device__ __forceinline__ int ref_bins(int r, int nref) { return nref <= 1 ? 0 : min(r + 1, nref - 1); }

// z-scan availability (6.4.1) of the 16x16 block (nx, ny) for the block (mx, my) on the 16x16
// grid: CTUs in raster order, blocks inside a CTU in z-order
__device__ __forceinline__ bool avail16(const Geom& g, int sh, int nx, int ny, int mx, int my) {
  if (nx < 0 || ny < 0 || nx >= g.wmb || ny >= g.hmb) return false;
  const int ux = nx >> sh, uy = ny >> sh, cx = mx >> sh, cy = my >> sh;
  if (ux != cx || uy != cy) return uy < cy || (uy == cy && ux < cx);
  const int m = (1 << sh) - 1;
  auto z = [](int x, int y) { return (x & 1) | ((y & 1) << 1) | ((x & 2) << 1) | ((y & 2) << 2); };
  return z(nx & m, ny & m) < z(mx & m, my & m);
}

// luma prediction (4 samples of row Y, columns X..X+3) of a B motion
__device__ __forceinline__ uint32_t mc4_b(const HevcBArgs& a, const uint8_t* G0, const uint8_t* H0, const uint8_t* G1,
                                          const uint8_t* H1, int X, int Y, int dir, int x0, int y0, int x1, int y1) {
  const int W = a.g.W, H = a.g.H;
  if (dir == 1) return mc4(G0, H0, W, H, X, Y, x0, y0);
  if (dir == 2) return mc4(G1, H1, W, H, X, Y, x1, y1);
  return avg4b(mc4(G0, H0, W, H, X, Y, x0, y0), mc4(G1, H1, W, H, X, Y, x1, y1));
}

// four blocks per wave (16-lane rows, a 4x4 sub-block per lane), as hevc_b_merge
__global__ __launch_bounds__(64) void hevc_b_choose(HevcBArgs a) {
  const Geom& g = a.g;
  const int nmb = g.nmb();
  int unit, slot;
  xcd_unit_slot(unit, slot);
  const int lane = threadIdx.x & 15;
  const int mb = unit * 4 + (threadIdx.x >> 4);
  if (mb >= nmb) return;
  const size_t o = static_cast<size_t>(slot) * nmb + mb;
  const int mx = mb % g.wmb, my = mb / g.wmb;
  const int X = mx * 16 + (lane & 3) * 4, Y = my * 16 + (lane >> 2) * 4;
  const size_t yo = static_cast<size_t>(slot) * g.ysize();
  const size_t ho = static_cast<size_t>(slot) * 3 * (g.W + 2 * kHpMargin) * (g.H + 2 * kHpMargin);
  const uint8_t *G0 = a.ref0 + yo, *G1 = a.ref1 + yo, *H0 = a.hp0 + ho, *H1 = a.hp1 + ho;
  const int x0 = a.mv0[o * 2], y0 = a.mv0[o * 2 + 1], x1 = a.mv1[o * 2], y1 = a.mv1[o * 2 + 1];
  uint32_t src[4], pw[4];
#pragma unroll
  for (int y = 0; y < 4; ++y) {
    src[y] = *reinterpret_cast<const uint32_t*>(a.src_y + yo + static_cast<size_t>(Y + y) * g.W + X);
    pw[y] = mc4_b(a, G0, H0, G1, H1, X, Y + y, 3, x0, y0, x1, y1);
  }
  const int satd_bi = satd16_rows(src, pw);
  const int qp = clampi(a.qp[slot] + (a.aq ? a.aq[o] : 0), 0, 51);
  const int lam = h264::kLambda[qp];
  const int b0 = mvbits_se(x0 - a.pm0[o * 2]) + mvbits_se(y0 - a.pm0[o * 2 + 1]);
  const int b1 = mvbits_se(x1 - a.pm1[o * 2]) + mvbits_se(y1 - a.pm1[o * 2 + 1]);
  // inter_pred_idc: "1" bi, "00" / "01" single list
  const int c_l0 = a.cost0[o] + 2 * lam, c_l1 = a.cost1[o] + 2 * lam;
  const int c_bi = satd_bi + lam * (b0 + b1 + 1);
  int dir = 1, best = c_l0, bits = b0 + 2;
  if (c_l1 < best) { dir = 2; best = c_l1; bits = b1 + 2; }
  if (c_bi < best) { dir = 3; best = c_bi; bits = b0 + b1 + 1; }
  if (lane == 0) {
    int16_t* m = a.mvb_out + o * 4;
    m[0] = static_cast<int16_t>(dir & 1 ? x0 : 0);
    m[1] = static_cast<int16_t>(dir & 1 ? y0 : 0);
    m[2] = static_cast<int16_t>(dir & 2 ? x1 : 0);
    m[3] = static_cast<int16_t>(dir & 2 ? y1 : 0);
    a.dir_out[o] = static_cast<uint8_t>(dir);
    a.cost[o] = best;
    a.bits[o] = bits;
  }
}

// P pictures enter the merge passes in the same form: the list-0 search, bits = its mvd bits;
// with several list-0 pictures the cheapest search at cost + lambda * ref_idx bins
__global__ __launch_bounds__(256) void hevc_b_init_p(HevcBArgs a) {
  const int nmb = a.g.nmb();
  const int i = blockIdx.x * 256 + threadIdx.x, slot = blockIdx.y;
  if (i >= nmb) return;
  const size_t o = static_cast<size_t>(slot) * nmb + i;
  int x0 = a.mv0[o * 2], y0 = a.mv0[o * 2 + 1];
  int best = a.cost0[o], bits = mvbits_se(x0 - a.pm0[o * 2]) + mvbits_se(y0 - a.pm0[o * 2 + 1]), br = 0;
  if (a.nref0 > 1) {
    const int qp = clampi(a.qp[slot] + (a.aq ? a.aq[o] : 0), 0, 51);
    const int lam = h264::kLambda[qp];
    best += lam * ref_bins(0, a.nref0);
    bits += ref_bins(0, a.nref0);
    const size_t plane = static_cast<size_t>(a.g.B) * nmb;
    for (int r = 1; r < a.nref0; ++r) {
      const size_t xo = (r - 1) * plane + o;
      const int c = a.xcost[xo];
      if (c >= kNoCostB) continue;
      const int rb = ref_bins(r, a.nref0);
      if (c + lam * rb < best) {
        best = c + lam * rb;
        br = r;
        x0 = a.xmv[xo * 2];
        y0 = a.xmv[xo * 2 + 1];
        bits = mvbits_se(x0 - a.xpm[xo * 2]) + mvbits_se(y0 - a.xpm[xo * 2 + 1]) + rb;
      }
    }
  }
  int16_t* m = a.mvb_out + o * 4;
  m[0] = static_cast<int16_t>(x0);
  m[1] = static_cast<int16_t>(y0);
  m[2] = m[3] = 0;
  a.dir_out[o] = static_cast<uint8_t>(1 | (br << 2));
  a.cost[o] = best;
  a.bits[o] = bits;
}

// Jacobi pass.  Each block is offered the merge list the CABAC writer would build for it as a
// 16x16 CU (8.5.3.2.2-8.5.3.2.5 on the 16x16 grid of current motions, z-scan availability in
// a 32x32 CTB: the below-left neighbour exists only for quadrant 0, the above-right one not for
// quadrant 3; pruning A1-B1, B1-B0, A1-A0, A1/B1-B2; the temporal candidate, combined
// bi-predictive and zero candidates; MaxNumMergeCand entries); the cheapest by SATD + lambda *
// (merge_flag + merge_idx bins) replaces the block's motion when it beats its cost.
//
// Four blocks per wave (one 16-lane row each, a 4x4 sub-block per lane, SATD in registers), as
// p_mv_refine: the pass is a chain of dependent loads per block, bound by blocks in flight.
constexpr int kMergeMbsPerWave = 4;

__global__ __launch_bounds__(64) void hevc_b_merge(HevcBArgs a) {
  const Geom& g = a.g;
  const int nmb = g.nmb();
  int unit, slot;
  xcd_unit_slot(unit, slot);
  const int lane = threadIdx.x & 15;
  const int mb = unit * kMergeMbsPerWave + (threadIdx.x >> 4);
  if (mb >= nmb) return;   // whole rows only: the DPP sums stay row-local
  const size_t o = static_cast<size_t>(slot) * nmb + mb;
  const size_t sb = static_cast<size_t>(slot) * nmb;
  const int mx = mb % g.wmb, my = mb / g.wmb;
  const int q = (mx & 1) | ((my & 1) << 1);
  const int maxc = a.max_merge;
  if (a.chg_in) {  // row-uniform (one MB per 16-lane row)
    const uint8_t* c = a.chg_in + sb;
    bool any = c[mb];
    if (mx > 0) any = any || c[mb - 1] || (my + 1 < g.hmb && c[mb + g.wmb - 1]);
    if (my > 0) any = any || c[mb - g.wmb] || (mx > 0 && c[mb - g.wmb - 1]) || (mx + 1 < g.wmb && c[mb - g.wmb + 1]);
    if (!any) {
      if (lane == 0) {
        *reinterpret_cast<uint2*>(a.mvb_out + o * 4) = *reinterpret_cast<const uint2*>(a.mvb_in + o * 4);
        a.dir_out[o] = a.dir_in[o];
        if (a.chg_out) a.chg_out[o] = 0;
      }
      return;
    }
  }
  int kd[6], kv[6][4], nk = 0;
  auto load = [&](int n, int* d, int* w) {
    const int dd = a.dir_in[sb + n];
    const int16_t* v = a.mvb_in + (sb + n) * 4;
    *d = dd;
    w[0] = dd & 1 ? v[0] : 0;
    w[1] = dd & 1 ? v[1] : 0;
    w[2] = dd & 2 ? v[2] : 0;
    w[3] = dd & 2 ? v[3] : 0;
  };
  auto same = [](int da, const int* wa, int db, const int* wb) {
    return da == db && wa[0] == wb[0] && wa[1] == wb[1] && wa[2] == wb[2] && wa[3] == wb[3];
  };
  int dA1 = 0, dB1 = 0, dB0 = 0, dA0 = 0, dB2 = 0, wA1[4], wB1[4], wB0[4], wA0[4], wB2[4];
  const bool a1 = mx > 0, av_b1 = my > 0;
  // above-right / below-left: z-scan order inside the CTU (32x32: B0 unavailable for quadrant 3,
  // A0 available for quadrant 0 only)
  bool b0 = avail16(g, a.ctu_shift, mx + 1, my - 1, mx, my), a0 = avail16(g, a.ctu_shift, mx - 1, my + 1, mx, my);
  bool b2 = mx > 0 && my > 0;
  (void)q;
  if (a1) load(mb - 1, &dA1, wA1);
  if (av_b1) load(mb - g.wmb, &dB1, wB1);
  if (b0) load(mb - g.wmb + 1, &dB0, wB0);
  if (a0) load(mb + g.wmb - 1, &dA0, wA0);
  if (b2) load(mb - g.wmb - 1, &dB2, wB2);
  const bool b1 = av_b1 && !(a1 && same(dA1, wA1, dB1, wB1));
  if (b0 && av_b1 && same(dB1, wB1, dB0, wB0)) b0 = false;
  if (a0 && a1 && same(dA1, wA1, dA0, wA0)) a0 = false;
  if (b2 && ((a1 && same(dA1, wA1, dB2, wB2)) || (av_b1 && same(dB1, wB1, dB2, wB2)))) b2 = false;
  if (static_cast<int>(a0) + a1 + b0 + b1 == 4) b2 = false;
  // the list lives in registers: every index below is a compile-time one (selects over the
  // six entries), so no scratch memory
  auto push = [&](int d, const int* w) {
#pragma unroll
    for (int t = 0; t < 6; ++t) {
      if (t == nk) {
        kd[t] = d;
#pragma unroll
        for (int c = 0; c < 4; ++c) kv[t][c] = w[c];
      }
    }
    nk += nk < 6;
  };
  if (a1) push(dA1, wA1);
  if (b1) push(dB1, wB1);
  if (b0) push(dB0, wB0);
  if (a0) push(dA0, wA0);
  if (b2) push(dB2, wB2);
  if (nk < maxc && a.tdir && a.tdir[o]) {
    const int td = a.bslice ? 3 : 1;
    const int16_t* t = a.tmv + o * 4;
    const int w[4] = {t[0], t[1], a.bslice ? t[2] : 0, a.bslice ? t[3] : 0};
    push(td, w);
  }
  const int orig = nk;
  if (a.bslice && orig > 1 && orig < maxc) {
    const int l0i[12] = {0, 1, 0, 2, 1, 2, 0, 3, 1, 3, 2, 3};
    const int l1i[12] = {1, 0, 2, 0, 2, 1, 3, 0, 3, 1, 3, 2};
#pragma unroll
    for (int c = 0; c < 12; ++c) {
      if (c >= orig * (orig - 1) || nk >= maxc) break;
      const int i0 = l0i[c], i1 = l1i[c];  // compile-time after unrolling
      if ((kd[i0] & 1) && (kd[i1] & 2)) {
        const int w[4] = {kv[i0][0], kv[i0][1], kv[i1][2], kv[i1][3]};
        push(3, w);
      }
    }
  }
  {
    // zero candidates: refIdx 0, 1, .. through the active list-0 size (P), then 0
    const int z[4] = {0, 0, 0, 0};
    for (int zi = 0; nk < maxc; ++zi) push(a.bslice ? 3 : (1 | ((zi < a.nref0 ? zi : 0) << 2)), z);
  }
  if (nk > maxc) nk = maxc;
  const int cd = a.dir_in[o];
  const int16_t* cvp = a.mvb_in + o * 4;
  const int cw[4] = {cd & 1 ? cvp[0] : 0, cd & 1 ? cvp[1] : 0, cd & 2 ? cvp[2] : 0, cd & 2 ? cvp[3] : 0};
  const int qp = clampi(a.qp[slot] + (a.aq ? a.aq[o] : 0), 0, 51);
  const int lam = h264::kLambda[qp];
  const int c_cur = a.cost[o];
  const int satd_cur = c_cur - lam * a.bits[o];
  const int X = mx * 16 + (lane & 3) * 4, Y = my * 16 + (lane >> 2) * 4;
  const size_t yo = static_cast<size_t>(slot) * g.ysize();
  const size_t ho = static_cast<size_t>(slot) * 3 * (g.W + 2 * kHpMargin) * (g.H + 2 * kHpMargin);
  const uint8_t *G1 = a.bslice ? a.ref1 + yo : a.ref0 + yo, *H1 = a.bslice ? a.hp1 + ho : a.hp0 + ho;
  uint32_t src[4];
#pragma unroll
  for (int y = 0; y < 4; ++y)
    src[y] = *reinterpret_cast<const uint32_t*>(a.src_y + yo + static_cast<size_t>(Y + y) * g.W + X);
  int best = c_cur, bbits = a.bits[o], bj = -1;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    if (j >= nk) break;
    bool dup = false;  // the same motion earlier in the list: never cheaper
#pragma unroll
    for (int i = 0; i < j; ++i) dup = dup || same(kd[i], kv[i], kd[j], kv[j]);
    if (dup) continue;
    int sat = satd_cur;
    if (!same(kd[j], kv[j], cd, cw)) {
      uint32_t pw[4];
      const int r0 = (kd[j] >> 2) & 3;  // list-0 refIdx (P pictures with several list-0 pictures)
      const uint8_t *G0 = l0_ref(a, r0) + yo, *H0 = l0_hp(a, r0) + ho;
#pragma unroll
      for (int y = 0; y < 4; ++y)
        pw[y] = mc4_b(a, G0, H0, G1, H1, X, Y + y, kd[j] & 3, kv[j][0], kv[j][1], kv[j][2], kv[j][3]);
      sat = satd16_rows(src, pw);
    }
    const int nb = 1 + (maxc > 1 ? min(j + 1, maxc - 1) : 0);  // merge_flag + truncated-unary merge_idx
    const int cst = sat + lam * nb;
    if (cst < best) {
      best = cst;
      bbits = nb;
      bj = j;
    }
  }
  if (lane == 0) {
    int16_t* m = a.mvb_out + o * 4;
    if (a.chg_out) {  // the motion (not just its cost) differs from the pass's input
      bool moved = false;
#pragma unroll
      for (int t = 0; t < 6; ++t)
        if (t == bj) moved = !same(kd[t], kv[t], cd, cw);
      a.chg_out[o] = moved;
    }
    if (bj >= 0) {
      int bd = 0, bw[4] = {0, 0, 0, 0};
#pragma unroll
      for (int t = 0; t < 6; ++t) {
        if (t == bj) {
          bd = kd[t];
#pragma unroll
          for (int c = 0; c < 4; ++c) bw[c] = kv[t][c];
        }
      }
      for (int c = 0; c < 4; ++c) m[c] = static_cast<int16_t>(bw[c]);
      a.dir_out[o] = static_cast<uint8_t>(bd);
    } else {
      for (int c = 0; c < 4; ++c) m[c] = cvp[c];
      a.dir_out[o] = static_cast<uint8_t>(cd);
    }
    a.cost[o] = best;
    a.bits[o] = bbits;
  }
}

// ---- P_8x8 / P_16x8 / P_8x16 partitions (x264 --partitions p8x8, its default).  After the
// 16x16 search and the skip-aware refinement, each 8x8 quadrant of a P macroblock searches
// its own vector: predictor candidates (the MB's vector, the left / top / top-right /
// right / bottom MBs' vectors, zero, the temporal predictor), then a half-sample and a
// quarter-sample ring around the best, SATD on the frame-level G/b/h/j planes.  The split
// wins when sum(SATD_q) + lambda * (mvd bits against the partition predictors of clause
// 8.4.1.3 + sub_mb_type overhead) beats the 16x16 cost; encode_inter then codes the four
// vectors (as P_16x8 / P_8x16 when they pair up).
//
// One wave per MB: lane = quadrant (2 bits) x 4x4 block of the quadrant (2 bits) x
// candidate slot (2 bits); block SATDs sum over lane bits 2-3, the best candidate of a
// quadrant is a min over bits 0-1.
struct PPartArgs {
  Geom g;
  const uint8_t* src_y;
  const uint8_t* ref;
  const uint8_t* hp;
  const int16_t* mv;    // [B, nmb, 2] final 16x16 vectors
  const int16_t* pm;    // [B, nmb, 2] the ME's predictor (its cost is priced against it)
  int* cost;            // [B, nmb] in: 16x16 cost; out: the chosen mode's cost
  uint8_t* pred;        // [B, nmb, 256] luma prediction, rewritten when the split wins
  int16_t* mv8;         // [B, nmb, 4, 2] out: per-quadrant vectors (all equal: 16x16)
  const int* qp;
  const int8_t* aq;
  int overhead;         // bits charged to the split beyond the mvds
  int min_satd;         // 16x16 SATD at or below this: no split search
  const SlotRoute* rt;  // routed (route.h): ref / hp are pools, P slots' RefPicList0[0]
  int nbuf;
  // HEVC 8x8 inter CUs (x265's minimum CU): the 16x16 cost is the merge passes' (SATD +
  // lambda * bits16, merge-aware), so it is compared as it stands; only blocks whose motion is
  // RefPicList0[0] list-0 (dir16 == 1) may split; pred is not rewritten (may be null)
  const int* bits16;
  const uint8_t* dir16;
};

__device__ __forceinline__ void med_pred(int ax, int ay, bool ha, int bx, int by, bool hb, int cx, int cy, bool hc,
                                         int* px, int* py) {
  // clause 8.4.1.3.1 with every neighbour at ref 0: B and C unavailable, A available -> A
  if (ha && !hb && !hc) {
    *px = ax;
    *py = ay;
    return;
  }
  if (!ha) ax = ay = 0;
  if (!hb) bx = by = 0;
  if (!hc) cx = cy = 0;
  *px = median3(ax, bx, cx);
  *py = median3(ay, by, cy);
}

// 8 waves per SIMD (64 VGPRs, a 60-byte spill; 6 at the compiler's 80 without spill): 18.9 -> 16.6 ms per
// step, +0.3 % headline (round-5 same-box A/B, profiles/r5_scratch_ab.md)
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8, 8))) void p_part8x8(PPartArgs a) {
  const Geom& g = a.g;
  const int nmb = g.nmb();
  int mb, slot;
  xcd_unit_slot(mb, slot);
  if (!route_active(a.rt, slot, SK_P)) return;
  const int lane = threadIdx.x;
  const size_t o = static_cast<size_t>(slot) * nmb + mb;
  const int mx = mb % g.wmb, my = mb / g.wmb;
  const int16_t* mv = a.mv + static_cast<size_t>(slot) * nmb * 2;
  const int vx = mv[mb * 2], vy = mv[mb * 2 + 1];
  const int qp = clampi(a.qp[slot] + (a.aq ? a.aq[o] : 0), 0, 51);
  const int lambda = h264::kLambda[qp];
  const int pmx = a.pm ? a.pm[o * 2] : 0, pmy = a.pm ? a.pm[o * 2 + 1] : 0;
  const int cost_in = a.cost[o];
  const int satd16 = a.bits16 ? cost_in - lambda * a.bits16[o] : cost_in - lambda * (mvbits_se(vx - pmx) + mvbits_se(vy - pmy));
  int16_t* m8 = a.mv8 + o * 8;
  const uint32_t vw = (static_cast<uint32_t>(vx) & 0xFFFFu) | (static_cast<uint32_t>(vy) << 16);
  if (satd16 <= a.min_satd || (a.dir16 && a.dir16[o] != 1)) {
    if (lane == 0) *reinterpret_cast<uint4*>(m8) = make_uint4(vw, vw, vw, vw);
    return;
  }
  // neighbouring MBs' 16x16 vectors (current picture)
  const bool hA = mx > 0, hB = my > 0, hC = my > 0 && mx < g.wmb - 1, hD = mx > 0 && my > 0;
  const bool hR = mx < g.wmb - 1, hU = my < g.hmb - 1;
  auto nv = [&](bool h, int n, int c) { return h ? static_cast<int>(mv[n * 2 + c]) : 0; };
  const int Ax = nv(hA, mb - 1, 0), Ay = nv(hA, mb - 1, 1);
  const int Bx = nv(hB, mb - g.wmb, 0), By = nv(hB, mb - g.wmb, 1);
  const int Cx = hC ? nv(true, mb - g.wmb + 1, 0) : nv(hD, mb - g.wmb - 1, 0);
  const int Cy = hC ? nv(true, mb - g.wmb + 1, 1) : nv(hD, mb - g.wmb - 1, 1);
  const bool hCD = hC || hD;
  // candidate predictors of every quadrant
  int cvx[8], cvy[8];
  cvx[0] = vx; cvy[0] = vy;
  cvx[1] = hA ? Ax : vx; cvy[1] = hA ? Ay : vy;
  cvx[2] = hB ? Bx : vx; cvy[2] = hB ? By : vy;
  cvx[3] = hCD ? Cx : vx; cvy[3] = hCD ? Cy : vy;
  cvx[4] = hR ? nv(true, mb + 1, 0) : vx; cvy[4] = hR ? nv(true, mb + 1, 1) : vy;
  cvx[5] = hU ? nv(true, mb + g.wmb, 0) : vx; cvy[5] = hU ? nv(true, mb + g.wmb, 1) : vy;
  cvx[6] = 0; cvy[6] = 0;
  cvx[7] = pmx; cvy[7] = pmy;
  const int q = lane >> 4, blk = (lane >> 2) & 3, c = lane & 3;
  // search-time partition predictor (the MB's own vector stands in for its other quadrants)
  int spx, spy;
  if (q == 0) med_pred(Ax, Ay, hA, Bx, By, hB, Bx, By, hB, &spx, &spy);
  else if (q == 1) med_pred(vx, vy, true, Bx, By, hB, Cx, Cy, hCD, &spx, &spy);
  else if (q == 2) med_pred(Ax, Ay, hA, vx, vy, true, vx, vy, true, &spx, &spy);
  else { spx = vx; spy = vy; }
  const int W = g.W, H = g.H;
  const int X = mx * 16 + (q & 1) * 8 + (blk & 1) * 4, Y = my * 16 + (q >> 1) * 8 + (blk >> 1) * 4;
  const size_t yo = static_cast<size_t>(slot) * g.ysize();
  const size_t s0 = route_index(a.rt, a.nbuf, slot, RO_L0);
  const uint8_t* G0 = a.ref + s0 * g.ysize();
  const uint8_t* H0 = a.hp + s0 * hp_plane_bytes(W, H);
  uint32_t srow[4];
#pragma unroll
  for (int y = 0; y < 4; ++y) srow[y] = *reinterpret_cast<const uint32_t*>(a.src_y + yo + static_cast<size_t>(Y + y) * W + X);
  // SATD of this quadrant at vector (x, y), summed over its four blocks
  auto qsatd = [&](int x, int y) -> int {
    uint32_t p4[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) p4[k] = mc4(G0, H0, W, H, X, Y + k, x, y);
    int s = satd4x4_u8(srow, p4);
    s += __shfl_xor(s, 4, 64);
    s += __shfl_xor(s, 8, 64);
    return s;
  };
  auto qmin = [](int k) {
    k = min(k, __shfl_xor(k, 1, 64));
    return min(k, __shfl_xor(k, 2, 64));
  };
  // stage 1: predictor candidates
  int bvx = vx, bvy = vy, bcost = 0x7FFFFFFF;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int i = it * 4 + c;
    // candidate i by selects (an index by lane would put cvx / cvy in scratch memory)
    int ix = 0, iy = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      ix = c == t ? cvx[it * 4 + t] : ix;
      iy = c == t ? cvy[it * 4 + t] : iy;
    }
    const int x = clampi(ix, -2048, 2047), y = clampi(iy, -512, 511);
    const int cst = qsatd(x, y) + lambda * (mvbits_se(x - spx) + mvbits_se(y - spy));
    const int key = qmin((cst << 3) | i);
    // the winner's vector from the lane of the quad that priced it
    const int wl = (lane & ~3) | (key & 3);
    const int wx = __shfl(x, wl, 64), wy = __shfl(y, wl, 64);
    if ((key >> 3) < bcost) {
      bcost = key >> 3;
      bvx = wx;
      bvy = wy;
    }
  }
  // stages 2-3: half- then quarter-sample rings around the best
#pragma unroll
  for (int step = 2; step >= 1; --step) {
    const int ox = bvx, oy = bvy;
    int kbest = 0x7FFFFFFF;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int i = it * 4 + c;                 // 0..7: the ring without its centre
      const int idx = i < 4 ? i : i + 1;
      const int x = ox + (idx % 3 - 1) * step, y = oy + (idx / 3 - 1) * step;
      const int cst = qsatd(x, y) + lambda * (mvbits_se(x - spx) + mvbits_se(y - spy));
      kbest = min(kbest, qmin((cst << 3) | i));
    }
    if ((kbest >> 3) < bcost) {
      bcost = kbest >> 3;
      const int i = kbest & 7, idx = i < 4 ? i : i + 1;
      bvx = ox + (idx % 3 - 1) * step;
      bvy = oy + (idx / 3 - 1) * step;
    }
  }
  const int bsatd = bcost - lambda * (mvbits_se(bvx - spx) + mvbits_se(bvy - spy));
  // every lane: all four quadrants' results (uniform per 16 lanes -> readlane)
  int qx[4], qy[4], qs[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    qx[k] = __builtin_amdgcn_readlane(bvx, 16 * k);
    qy[k] = __builtin_amdgcn_readlane(bvy, 16 * k);
    qs[k] = __builtin_amdgcn_readlane(bsatd, 16 * k);
  }
  // exact-form partition predictors (neighbouring MBs still as their 16x16 vectors)
  int p0x, p0y, p1x, p1y, p2x, p2y, p3x, p3y, p16x, p16y;
  med_pred(Ax, Ay, hA, Bx, By, hB, Bx, By, hB, &p0x, &p0y);
  med_pred(qx[0], qy[0], true, Bx, By, hB, Cx, Cy, hCD, &p1x, &p1y);
  med_pred(Ax, Ay, hA, qx[0], qy[0], true, qx[1], qy[1], true, &p2x, &p2y);
  med_pred(qx[2], qy[2], true, qx[1], qy[1], true, qx[0], qy[0], true, &p3x, &p3y);
  med_pred(Ax, Ay, hA, Bx, By, hB, Cx, Cy, hCD, &p16x, &p16y);
  const int bits8 = mvbits_se(qx[0] - p0x) + mvbits_se(qy[0] - p0y) + mvbits_se(qx[1] - p1x) + mvbits_se(qy[1] - p1y) +
                    mvbits_se(qx[2] - p2x) + mvbits_se(qy[2] - p2y) + mvbits_se(qx[3] - p3x) + mvbits_se(qy[3] - p3y);
  const int cost8 = qs[0] + qs[1] + qs[2] + qs[3] + lambda * (bits8 + a.overhead);
  const int cost16 = a.bits16 ? cost_in : satd16 + lambda * (mvbits_se(vx - p16x) + mvbits_se(vy - p16y));
  const bool uniform = qx[0] == qx[1] && qx[0] == qx[2] && qx[0] == qx[3] && qy[0] == qy[1] && qy[0] == qy[2] &&
                       qy[0] == qy[3];
  const bool split = !uniform && cost8 < cost16;
  if (split && a.pred) {
    // lane (q, blk, c) rewrites row c of its block
    const uint32_t p = mc4(G0, H0, W, H, X, Y + c, bvx, bvy);
    const int lx = (q & 1) * 8 + (blk & 1) * 4, ly = (q >> 1) * 8 + (blk >> 1) * 4 + c;
    *reinterpret_cast<uint32_t*>(a.pred + o * 256 + ly * 16 + lx) = p;
  }
  if (lane == 0) {
    if (split) {
      auto w = [](int x, int y) { return (static_cast<uint32_t>(x) & 0xFFFFu) | (static_cast<uint32_t>(y) << 16); };
      *reinterpret_cast<uint4*>(m8) = make_uint4(w(qx[0], qy[0]), w(qx[1], qy[1]), w(qx[2], qy[2]), w(qx[3], qy[3]));
      a.cost[o] = cost8 - cost16 + cost_in;     // the 16x16 cost's convention, shifted by the gain
    } else {
      *reinterpret_cast<uint4*>(m8) = make_uint4(vw, vw, vw, vw);
    }
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

extern "C" void mivc_launch_b_direct(int B, int wmb, int hmb, const void* col, const int* dsf, const int* direct_copy,
                                     int nref, int16_t* dmv, int8_t* dref, int16_t* pm0, int16_t* pm1, void* stream,
                                     const void* route, int nbuf, uint8_t* czero) {
  BDirectArgs a;
  a.czero = czero;
  a.rt = static_cast<const SlotRoute*>(route);
  a.nbuf = nbuf;
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.col = static_cast<const MbHeader*>(col);
  for (int r = 0; r < kMaxRefs; ++r) {  // refIdxCol beyond the list: the last entry (never produced)
    const int rr = r < nref ? r : nref - 1;
    a.dsf[r] = dsf[rr];
    a.direct_copy[r] = direct_copy[rr];
  }
  a.dmv = dmv;
  a.dref = dref;
  a.pm0 = pm0;
  a.pm1 = pm1;
  hipLaunchKernelGGL(b_direct_mv, dim3((wmb * hmb + 255) / 256, B), dim3(256), 0, static_cast<hipStream_t>(stream), a);
}

extern "C" void mivc_launch_b_decide(int B, int wmb, int hmb, const uint8_t* src_y, const uint8_t* ref0,
                                     const uint8_t* ref1, const uint8_t* hp0, const uint8_t* hp1, const int16_t* mv0,
                                     const int16_t* mv1, const int* cost0, const int* cost1, const uint8_t* pred0,
                                     const uint8_t* pred1, const int16_t* pm0, const int16_t* pm1, const int16_t* dmv,
                                     const int* qp, const int8_t* aq, void* hdr, uint8_t* pred_out, int* cost_out,
                                     void* stream, const int* w1, int nref, const int8_t* dref,
                                     const uint8_t* const* ref0k, const uint8_t* const* hp0k, int direct_only, int bparts, int have_direct,
                                     int spatial, int dbias, const void* route, int nbuf, const uint8_t* czero) {
  BDecideArgs a;
  a.czero = czero;
  a.rt = static_cast<const SlotRoute*>(route);
  a.nbuf = nbuf;
  a.spatial = spatial;
  a.dbias = dbias;
  a.direct_only = direct_only;
  a.have_direct = have_direct;
  a.bparts = bparts;
  for (int r = 0; r < kMaxRefs; ++r) {
    const int rr = r < nref ? r : nref - 1;
    a.w1[r] = w1[rr];
    a.ref0k[r] = rr == 0 ? ref0 : ref0k[rr];
    a.hp0k[r] = rr == 0 ? hp0 : hp0k[rr];
  }
  a.dref = dref;
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.src_y = src_y;
  a.ref0 = ref0;
  a.ref1 = ref1;
  a.hp0 = hp0;
  a.hp1 = hp1;
  a.mv0 = mv0;
  a.mv1 = mv1;
  a.cost0 = cost0;
  a.cost1 = cost1;
  a.pred0 = pred0;
  a.pred1 = pred1;
  a.pm0 = pm0;
  a.pm1 = pm1;
  a.dmv = dmv;
  a.qp = qp;
  a.aq = aq;
  a.hdr = static_cast<MbHeader*>(hdr);
  a.pred_out = pred_out;
  a.cost_out = cost_out;
  const dim3 grid((wmb * hmb + kDecideMbsPerWave - 1) / kDecideMbsPerWave, B);
  const hipStream_t st = static_cast<hipStream_t>(stream);
  if (direct_only && spatial == 0)
    hipLaunchKernelGGL(b_decide<3>, grid, dim3(64), 0, st, a);
  else if (direct_only)
    hipLaunchKernelGGL(b_decide<1>, grid, dim3(64), 0, st, a);
  else if (have_direct)
    hipLaunchKernelGGL(b_decide<2>, grid, dim3(64), 0, st, a);
  else
    hipLaunchKernelGGL(b_decide<0>, grid, dim3(64), 0, st, a);
}

extern "C" void mivc_launch_p_refine(int B, int wmb, int hmb, const uint8_t* src_y, const uint8_t* ref,
                                     const uint8_t* hp, const int16_t* mv_in, int16_t* mv_out, int* cost,
                                     const int16_t* pm, uint8_t* pred, const int* qp, const int8_t* aq,
                                     void* stream, const void* route, int nbuf, const uint8_t* chg_in,
                                     uint8_t* chg_out) {
  PRefineArgs a;
  a.chg_in = chg_in;
  a.chg_out = chg_out;
  a.rt = static_cast<const SlotRoute*>(route);
  a.nbuf = nbuf;
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.src_y = src_y;
  a.ref = ref;
  a.hp = hp;
  a.mv_in = mv_in;
  a.mv_out = mv_out;
  a.cost = cost;
  a.pm = pm;
  a.pred = pred;
  a.qp = qp;
  a.aq = aq;
  hipLaunchKernelGGL(p_mv_refine, dim3((wmb * hmb + kRefineMbsPerWave - 1) / kRefineMbsPerWave, B), dim3(64), 0,
                     static_cast<hipStream_t>(stream), a);
}

extern "C" void mivc_launch_p_part8(int B, int wmb, int hmb, const uint8_t* src_y, const uint8_t* ref,
                                    const uint8_t* hp, const int16_t* mv, const int16_t* pm, int* cost, uint8_t* pred,
                                    int16_t* mv8, const int* qp, const int8_t* aq, int overhead, int min_satd,
                                    void* stream, const void* route, int nbuf, const int* bits16,
                                    const uint8_t* dir16) {
  PPartArgs a;
  a.bits16 = bits16;
  a.dir16 = dir16;
  a.rt = static_cast<const SlotRoute*>(route);
  a.nbuf = nbuf;
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.src_y = src_y;
  a.ref = ref;
  a.hp = hp;
  a.mv = mv;
  a.pm = pm;
  a.cost = cost;
  a.pred = pred;
  a.mv8 = mv8;
  a.qp = qp;
  a.aq = aq;
  a.overhead = overhead;
  a.min_satd = min_satd;
  hipLaunchKernelGGL(p_part8x8, dim3(wmb * hmb, B), dim3(64), 0, static_cast<hipStream_t>(stream), a);
}

extern "C" void mivc_launch_hevc_merge_refine(int B, int wmb, int hmb, const uint8_t* src_y, const uint8_t* ref,
                                              const uint8_t* hp, const int16_t* mv_in, int16_t* mv_out, int* cost,
                                              const int16_t* pm, const int* qp, const int8_t* aq, void* stream) {
  PRefineArgs a;
  a.chg_in = nullptr;
  a.chg_out = nullptr;
  a.rt = nullptr;
  a.nbuf = 0;
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.src_y = src_y;
  a.ref = ref;
  a.hp = hp;
  a.mv_in = mv_in;
  a.mv_out = mv_out;
  a.cost = cost;
  a.pm = pm;
  a.pred = nullptr;
  a.qp = qp;
  a.aq = aq;
  hipLaunchKernelGGL(hevc_merge_refine, dim3((wmb * hmb + kRefineMbsPerWave - 1) / kRefineMbsPerWave, B), dim3(64), 0,
                     static_cast<hipStream_t>(stream), a);
}

extern "C" void mivc_launch_hevc_b(int mode, int B, int wmb, int hmb, const uint8_t* src_y, const uint8_t* ref0,
                                   const uint8_t* ref1, const uint8_t* hp0, const uint8_t* hp1, const int16_t* mv0,
                                   const int16_t* mv1, const int* cost0, const int* cost1, const int16_t* pm0,
                                   const int16_t* pm1, const int16_t* tmv, const uint8_t* tdir, const int16_t* mvb_in,
                                   const uint8_t* dir_in, int16_t* mvb_out, uint8_t* dir_out, int* cost, int* bits,
                                   const int* qp, const int8_t* aq, void* stream, int bslice, int max_merge,
                                   int ctu64, const uint8_t* chg_in, uint8_t* chg_out, int nref0,
                                   const uint8_t* const* xref, const uint8_t* const* xhp, const int16_t* xmv,
                                   const int* xcost, const int16_t* xpm) {
  HevcBArgs a;
  a.nref0 = nref0 < 1 ? 1 : nref0;
  for (int r = 0; r < 3; ++r) {
    a.xref[r] = r + 1 < a.nref0 ? xref[r] : ref0;
    a.xhp[r] = r + 1 < a.nref0 ? xhp[r] : hp0;
  }
  a.xmv = xmv;
  a.xcost = xcost;
  a.xpm = xpm;
  a.chg_in = chg_in;
  a.chg_out = chg_out;
  a.ctu_shift = ctu64 ? 2 : 1;
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.src_y = src_y;
  a.ref0 = ref0;
  a.ref1 = ref1;
  a.hp0 = hp0;
  a.hp1 = hp1;
  a.mv0 = mv0;
  a.mv1 = mv1;
  a.cost0 = cost0;
  a.cost1 = cost1;
  a.pm0 = pm0;
  a.pm1 = pm1;
  a.tmv = tmv;
  a.tdir = tdir;
  a.mvb_in = mvb_in;
  a.dir_in = dir_in;
  a.mvb_out = mvb_out;
  a.dir_out = dir_out;
  a.cost = cost;
  a.bits = bits;
  a.qp = qp;
  a.aq = aq;
  a.bslice = bslice;
  a.max_merge = max_merge;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (mode == 0) hipLaunchKernelGGL(hevc_b_choose, dim3((wmb * hmb + 3) / 4, B), dim3(64), 0, st, a);
  else if (mode == 1)
    hipLaunchKernelGGL(hevc_b_merge, dim3((wmb * hmb + kMergeMbsPerWave - 1) / kMergeMbsPerWave, B), dim3(64), 0, st, a);
  else hipLaunchKernelGGL(hevc_b_init_p, dim3((wmb * hmb + 255) / 256, B), dim3(256), 0, st, a);
}

extern "C" void mivc_launch_b_spatial(int B, int wmb, int hmb, void* hdr, const void* col, const uint8_t* src_y,
                                      const uint8_t* ref1, const uint8_t* hp1, const uint8_t* const* ref0k,
                                      const uint8_t* const* hp0k, const int* w1, int nref, uint8_t* pred_out, int* err,
                                      void* stream, const int* intra_cost, int* cost, const int* qp, const int8_t* aq,
                                      int bias, const void* route, int nbuf) {
  BSpatialArgs a;
  a.rt = static_cast<const SlotRoute*>(route);
  a.nbuf = nbuf;
  a.bias = bias;
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.hdr = static_cast<MbHeader*>(hdr);
  a.col = static_cast<const MbHeader*>(col);
  a.err = err;
  a.intra_cost = intra_cost;
  a.cost = cost;
  a.src_y = src_y;
  a.ref1 = ref1;
  a.hp1 = hp1;
  for (int r = 0; r < kMaxRefs; ++r) {
    const int rr = r < nref ? r : nref - 1;
    a.ref0k[r] = ref0k[rr];
    a.hp0k[r] = hp0k[rr];
    a.w1[r] = w1[rr];
  }
  a.pred_out = pred_out;
  a.qp = qp;
  a.aq = aq;
  hipLaunchKernelGGL(b_spatial_decide, dim3(B), dim3(64 * kSpatialWaves), 0, static_cast<hipStream_t>(stream), a);
}

extern "C" void mivc_launch_b_spatial_exact(int B, int wmb, int hmb, void* hdr, const int* intra_cost, const int* cost,
                                            const uint8_t* czero, uint8_t* fix, void* stream, const void* route,
                                            int slice_rows, int tol) {
  BSpatialExactArgs a;
  a.slice_rows = slice_rows;
  a.tol = tol;
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.hdr = static_cast<MbHeader*>(hdr);
  a.intra_cost = intra_cost;
  a.cost = cost;
  a.czero = czero;
  a.fix = fix;
  a.rt = static_cast<const SlotRoute*>(route);
  const int waves = (hmb + 63) / 64;
  hipLaunchKernelGGL(b_spatial_exact, dim3(B), dim3(64 * waves), 0, static_cast<hipStream_t>(stream), a);
}

extern "C" void mivc_launch_b_spatial_fixup(int B, int wmb, int hmb, const void* hdr, const uint8_t* fix,
                                            const uint8_t* ref0, const uint8_t* hp0, const uint8_t* ref1,
                                            const uint8_t* hp1, uint8_t* pred_out, void* stream, const void* route,
                                            int nbuf) {
  BSpatialFixArgs a;
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.hdr = static_cast<const MbHeader*>(hdr);
  a.fix = fix;
  a.ref0 = ref0;
  a.hp0 = hp0;
  a.ref1 = ref1;
  a.hp1 = hp1;
  a.pred_out = pred_out;
  a.rt = static_cast<const SlotRoute*>(route);
  a.nbuf = nbuf;
  hipLaunchKernelGGL(b_spatial_fixup, dim3(wmb * hmb, B), dim3(64), 0, static_cast<hipStream_t>(stream), a);
}
