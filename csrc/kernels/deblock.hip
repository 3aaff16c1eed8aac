// In-loop deblocking filter (clause 8.7), SURVEY.md K-C9.
//
// The normative result depends on macroblock raster order: MB n+1's left edge
// filter reads samples MB n's horizontal edges already modified, and MB (x, y)'s
// top edge reads samples MB (x+1, y-1)'s left edge modified.  So MB (x, y) runs
// after (x-1, y) and (x+1, y-1): the same row wavefront as intra coding (one
// workgroup of kDeblockWaves wave64s per frame, wave w owns rows w, w+kDeblockWaves,
// ..., LDS row-progress counters at workgroup scope).  Inside an
// MB the 16 lines of an edge are filtered in parallel (lanes 0-15 luma, 16-31
// chroma), edges in the normative order (vertical left->right, then horizontal
// top->bottom).  Boundary strengths are derived per MB from the decision
// records (intra, non-zero coefficients, motion vectors).
#include "kcommon.h"

namespace mivc {
namespace gpu {

using h264::MbHeader;

struct DeblockArgs {
  Geom g;
  uint8_t *rec_y, *rec_u, *rec_v;
  const MbHeader* hdr;
  const uint8_t* nz;   // [B, nmb, 16] raster
  int chroma_qp_offset;
  int alpha_off, beta_off;  // slice_alpha_c0_offset_div2*2, slice_beta_offset_div2*2
  int* err;
};

constexpr int kDeblockWaves = 16;

constexpr int LT = 20;  // luma tile stride: 4 halo + 16
constexpr int CT = 12;  // chroma tile stride: 4 halo (2 used) + 8 -- rows stay 4-byte aligned

struct DeblockShared {
  alignas(16) uint8_t ty[LT * LT];
  alignas(16) uint8_t tc[2][CT * 10];
  alignas(16) uint32_t hdrw[3][12];  // MbHeader of the current, left and top MB
  uint8_t nzb[3][16];                // their non-zero flags
  int bs[2][4][4];                   // [dir][edge][segment]
  uint32_t left_y[16];               // previous MB's columns 12..15 after filtering (one word per row)
  uint32_t left_c[2][8];             // previous MB's chroma columns 4..7
  int saved_x;
};

__device__ __forceinline__ void filter_line(uint8_t* q0p, int step, int bs, int alpha, int beta, int tc0, bool chroma) {
  int p0 = q0p[-step], p1 = q0p[-2 * step], q0 = q0p[0], q1 = q0p[step];
  int d0 = p0 - q0, d1 = p1 - p0, d2 = q1 - q0;
  if (!((d0 < 0 ? -d0 : d0) < alpha && (d1 < 0 ? -d1 : d1) < beta && (d2 < 0 ? -d2 : d2) < beta)) return;
  if (chroma) {
    if (bs < 4) {
      int tc = tc0 + 1;
      int delta = clampi((((q0 - p0) << 2) + (p1 - q1) + 4) >> 3, -tc, tc);
      q0p[-step] = static_cast<uint8_t>(h264::clip1(p0 + delta));
      q0p[0] = static_cast<uint8_t>(h264::clip1(q0 - delta));
    } else {
      q0p[-step] = static_cast<uint8_t>((2 * p1 + p0 + q1 + 2) >> 2);
      q0p[0] = static_cast<uint8_t>((2 * q1 + q0 + p1 + 2) >> 2);
    }
    return;
  }
  int p2 = q0p[-3 * step], q2 = q0p[2 * step];
  int ap = p2 - p0, aq = q2 - q0;
  ap = ap < 0 ? -ap : ap;
  aq = aq < 0 ? -aq : aq;
  if (bs < 4) {
    int tc = tc0 + (ap < beta) + (aq < beta);
    int delta = clampi((((q0 - p0) << 2) + (p1 - q1) + 4) >> 3, -tc, tc);
    q0p[-step] = static_cast<uint8_t>(h264::clip1(p0 + delta));
    q0p[0] = static_cast<uint8_t>(h264::clip1(q0 - delta));
    if (ap < beta) q0p[-2 * step] = static_cast<uint8_t>(p1 + clampi((p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1, -tc0, tc0));
    if (aq < beta) q0p[step] = static_cast<uint8_t>(q1 + clampi((q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1, -tc0, tc0));
  } else {
    int ad = d0 < 0 ? -d0 : d0;
    bool strong = ad < ((alpha >> 2) + 2);
    if (ap < beta && strong) {
      int p3 = q0p[-4 * step];
      q0p[-step] = static_cast<uint8_t>((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
      q0p[-2 * step] = static_cast<uint8_t>((p2 + p1 + p0 + q0 + 2) >> 2);
      q0p[-3 * step] = static_cast<uint8_t>((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
    } else {
      q0p[-step] = static_cast<uint8_t>((2 * p1 + p0 + q1 + 2) >> 2);
    }
    if (aq < beta && strong) {
      int q3 = q0p[3 * step];
      q0p[0] = static_cast<uint8_t>((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
      q0p[step] = static_cast<uint8_t>((p0 + q0 + q1 + q2 + 2) >> 2);
      q0p[2 * step] = static_cast<uint8_t>((2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3);
    } else {
      q0p[0] = static_cast<uint8_t>((2 * q1 + q0 + p1 + 2) >> 2);
    }
  }
}

// mv of the 4x4 block at raster r of an MB (from the per-quadrant MbHeader vectors)
__device__ __forceinline__ void blk_mv(const MbHeader& h, int r, int* mv) {
  int q = ((r >> 3) & 1) * 2 + ((r & 3) >> 1);
  mv[0] = h.mv[q][0];
  mv[1] = h.mv[q][1];
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ void deblock_mb(const DeblockArgs& a, DeblockShared& S, int slot, int mx, int my) {
  const Geom& g = a.g;
  const int lane = lane_id();
  const int W = g.W, cw = g.cw();
  const size_t o = static_cast<size_t>(slot) * g.nmb() + my * g.wmb + mx;
  uint8_t* recy = a.rec_y + slot * g.ysize();
  uint8_t* recc[2] = {a.rec_u + slot * g.csize(), a.rec_v + slot * g.csize()};
  const int X0 = mx * 16, Y0 = my * 16, XC = mx * 8, YC = my * 8;
  const bool has_left = mx > 0, has_top = my > 0;
  const bool left_saved = S.saved_x == mx - 1;

  // ---- phase 1: every global read of this MB in one batch (dwords), then the LDS stores
  const uint32_t* hdr32 = reinterpret_cast<const uint32_t*>(a.hdr);
  uint32_t la, lb = 0, lc = 0, ld = 0;
  {
    const int r = lane >> 2, c4 = (lane & 3) * 4;
    la = *reinterpret_cast<const uint32_t*>(recy + static_cast<size_t>(Y0 + r) * W + X0 + c4);
  }
  if (lane < 16) {
    if (has_top) lb = *reinterpret_cast<const uint32_t*>(recy + static_cast<size_t>(Y0 - 4 + (lane >> 2)) * W + X0 + (lane & 3) * 4);
  } else if (lane < 32) {
    if (has_left && !left_saved) lb = *reinterpret_cast<const uint32_t*>(recy + static_cast<size_t>(Y0 + lane - 16) * W + X0 - 4);
  } else {
    const int comp = (lane - 32) >> 4, i = lane & 15;
    lb = *reinterpret_cast<const uint32_t*>(recc[comp] + static_cast<size_t>(YC + (i >> 1)) * cw + XC + (i & 1) * 4);
  }
  if (lane < 8) {
    const int comp = lane >> 2, r = (lane >> 1) & 1, h = lane & 1;
    if (has_top) lc = *reinterpret_cast<const uint32_t*>(recc[comp] + static_cast<size_t>(YC - 2 + r) * cw + XC + h * 4);
  } else if (lane < 24) {
    const int comp = (lane - 8) >> 3, r = (lane - 8) & 7;
    if (has_left && !left_saved) lc = *reinterpret_cast<const uint32_t*>(recc[comp] + static_cast<size_t>(YC + r) * cw + XC - 4);
  } else if (lane < 60) {
    const int which = (lane - 24) / 12, k = (lane - 24) % 12;
    const bool ok = which == 0 || (which == 1 ? has_left : has_top);
    const size_t mbo = which == 0 ? o : (which == 1 ? o - 1 : o - g.wmb);
    if (ok) lc = hdr32[mbo * 12 + k];
  }
  if (lane < 12) {
    const int which = lane >> 2, k = lane & 3;
    const bool ok = which == 0 || (which == 1 ? has_left : has_top);
    const size_t mbo = which == 0 ? o : (which == 1 ? o - 1 : o - g.wmb);
    if (ok) ld = reinterpret_cast<const uint32_t*>(a.nz)[mbo * 4 + k];
  }
  {
    const int r = lane >> 2, c4 = (lane & 3) * 4;
    *reinterpret_cast<uint32_t*>(&S.ty[(r + 4) * LT + 4 + c4]) = la;
  }
  if (lane < 16) {
    if (has_top) *reinterpret_cast<uint32_t*>(&S.ty[(lane >> 2) * LT + 4 + (lane & 3) * 4]) = lb;
  } else if (lane < 32) {
    if (has_left) *reinterpret_cast<uint32_t*>(&S.ty[(lane - 16 + 4) * LT]) = left_saved ? S.left_y[lane - 16] : lb;
  } else {
    const int comp = (lane - 32) >> 4, i = lane & 15;
    *reinterpret_cast<uint32_t*>(&S.tc[comp][((i >> 1) + 2) * CT + 4 + (i & 1) * 4]) = lb;
  }
  if (lane < 8) {
    const int comp = lane >> 2, r = (lane >> 1) & 1, h = lane & 1;
    if (has_top) *reinterpret_cast<uint32_t*>(&S.tc[comp][r * CT + 4 + h * 4]) = lc;
  } else if (lane < 24) {
    const int comp = (lane - 8) >> 3, r = (lane - 8) & 7;
    if (has_left) *reinterpret_cast<uint32_t*>(&S.tc[comp][(r + 2) * CT]) = left_saved ? S.left_c[comp][r] : lc;
  } else if (lane < 60) {
    S.hdrw[(lane - 24) / 12][(lane - 24) % 12] = lc;
  }
  if (lane < 12) reinterpret_cast<uint32_t*>(S.nzb[lane >> 2])[lane & 3] = ld;
  wave_sync();

  // ---- boundary strengths: lane = dir*16 + edge*4 + seg
  const MbHeader* HQ = reinterpret_cast<const MbHeader*>(S.hdrw[0]);
  if (lane < 32) {
    int dir = lane >> 4, e = (lane >> 2) & 3, k = lane & 3;
    int bs = 0;
    bool mbedge = e == 0;
    bool avail = !mbedge || (dir == 0 ? has_left : has_top);
    if (avail) {
      const int pw = mbedge ? (dir == 0 ? 1 : 2) : 0;
      const MbHeader* HP = reinterpret_cast<const MbHeader*>(S.hdrw[pw]);
      int rq = dir == 0 ? (e + 4 * k) : (k + 4 * e);
      int rp = dir == 0 ? (mbedge ? 3 + 4 * k : e - 1 + 4 * k) : (mbedge ? k + 12 : k + 4 * (e - 1));
      bool iq = h264::mbk_is_intra(HQ->kind), ip = h264::mbk_is_intra(HP->kind);
      if (mbedge && (iq || ip)) bs = 4;
      else if (iq || ip) bs = 3;
      else if (S.nzb[pw][rp] || S.nzb[0][rq]) bs = 2;
      else {
        int mp[2], mq[2];
        blk_mv(*HP, rp, mp);
        blk_mv(*HQ, rq, mq);
        int dx = mp[0] - mq[0], dy = mp[1] - mq[1];
        bs = (dx >= 4 || dx <= -4 || dy >= 4 || dy <= -4) ? 1 : 0;
      }
    }
    S.bs[dir][e][k] = bs;
  }
  wave_sync();

  // QPs are uniform: read them into SGPRs so the alpha/beta/tc0 lookups are scalar loads
  const int qpq = uni(HQ->qp);
  const int qpl = uni(reinterpret_cast<const MbHeader*>(S.hdrw[1])->qp);
  const int qpt = uni(reinterpret_cast<const MbHeader*>(S.hdrw[2])->qp);
  // ---- vertical edges, then horizontal edges
  for (int dir = 0; dir < 2; ++dir) {
    for (int e = 0; e < 4; ++e) {
      if (e == 0 && !(dir == 0 ? has_left : has_top)) continue;
      const int qpp = e == 0 ? (dir == 0 ? qpl : qpt) : qpq;
      if (lane < 16) {
        int bs = S.bs[dir][e][lane >> 2];
        const int qpav = (qpp + qpq + 1) >> 1;
        const int ia = clampi(qpav + a.alpha_off, 0, 51), ib = clampi(qpav + a.beta_off, 0, 51);
        const int t1 = h264::kTc0[ia][0], t2 = h264::kTc0[ia][1], t3 = h264::kTc0[ia][2];
        const int alpha = h264::kAlpha[ia], beta = h264::kBeta[ib];
        if (bs) {
          int tc0 = bs == 1 ? t1 : (bs == 2 ? t2 : (bs == 3 ? t3 : 0));
          uint8_t* q0 = dir == 0 ? &S.ty[(lane + 4) * LT + 4 + 4 * e] : &S.ty[(4 + 4 * e) * LT + 4 + lane];
          filter_line(q0, dir == 0 ? 1 : LT, bs, alpha, beta, tc0, false);
        }
      } else if (lane < 32 && (e == 0 || e == 2)) {
        int comp = (lane - 16) >> 3, i = (lane - 16) & 7;
        int bs = S.bs[dir][e][i >> 1];
        const int cp = h264::chroma_qp(qpp, a.chroma_qp_offset), cq = h264::chroma_qp(qpq, a.chroma_qp_offset);
        const int qpav = (cp + cq + 1) >> 1;
        const int ia = clampi(qpav + a.alpha_off, 0, 51), ib = clampi(qpav + a.beta_off, 0, 51);
        const int t1 = h264::kTc0[ia][0], t2 = h264::kTc0[ia][1], t3 = h264::kTc0[ia][2];
        const int alpha = h264::kAlpha[ia], beta = h264::kBeta[ib];
        if (bs) {
          int tc0 = bs == 1 ? t1 : (bs == 2 ? t2 : (bs == 3 ? t3 : 0));
          int ce = e >> 1;
          uint8_t* t = S.tc[comp];
          uint8_t* q0 = dir == 0 ? &t[(i + 2) * CT + 4 + 4 * ce] : &t[(2 + 4 * ce) * CT + 4 + i];
          filter_line(q0, dir == 0 ? 1 : CT, bs, alpha, beta, tc0, true);
        }
      }
      wave_sync();
    }
  }
  // ---- write back (dwords): MB interior + the modified halo (3 luma / 1 chroma lines; the
  // 4th luma / 2nd chroma column of the left halo is rewritten unchanged -- its MB is final)
  {
    const int r = lane >> 2, c4 = (lane & 3) * 4;
    *reinterpret_cast<uint32_t*>(recy + static_cast<size_t>(Y0 + r) * W + X0 + c4) =
        *reinterpret_cast<const uint32_t*>(&S.ty[(r + 4) * LT + 4 + c4]);
  }
  if (lane < 12) {
    if (has_top) {
      const int r = 1 + (lane >> 2), c4 = (lane & 3) * 4;  // rows -3..-1
      *reinterpret_cast<uint32_t*>(recy + static_cast<size_t>(Y0 - 4 + r) * W + X0 + c4) =
          *reinterpret_cast<const uint32_t*>(&S.ty[r * LT + 4 + c4]);
    }
  } else if (lane < 28) {
    if (has_left) {
      const int r = lane - 12;
      *reinterpret_cast<uint32_t*>(recy + static_cast<size_t>(Y0 + r) * W + X0 - 4) =
          *reinterpret_cast<const uint32_t*>(&S.ty[(r + 4) * LT]);
    }
  } else if (lane < 60) {
    const int comp = (lane - 28) >> 4, i = (lane - 28) & 15;
    *reinterpret_cast<uint32_t*>(recc[comp] + static_cast<size_t>(YC + (i >> 1)) * cw + XC + (i & 1) * 4) =
        *reinterpret_cast<const uint32_t*>(&S.tc[comp][((i >> 1) + 2) * CT + 4 + (i & 1) * 4]);
  }
  if (lane < 4) {
    if (has_top) {
      const int comp = lane >> 1, h = lane & 1;  // chroma row -1
      *reinterpret_cast<uint32_t*>(recc[comp] + static_cast<size_t>(YC - 1) * cw + XC + h * 4) =
          *reinterpret_cast<const uint32_t*>(&S.tc[comp][1 * CT + 4 + h * 4]);
    }
  } else if (lane < 20) {
    if (has_left) {
      const int comp = (lane - 4) >> 3, r = (lane - 4) & 7;  // chroma column -1 (word -4..-1)
      *reinterpret_cast<uint32_t*>(recc[comp] + static_cast<size_t>(YC + r) * cw + XC - 4) =
          *reinterpret_cast<const uint32_t*>(&S.tc[comp][(r + 2) * CT]);
    }
  }
  // ---- keep this MB's right edge for the next iteration (final values)
  if (lane < 16) S.left_y[lane] = *reinterpret_cast<const uint32_t*>(&S.ty[(lane + 4) * LT + 16]);
  else if (lane < 32) {
    const int comp = (lane - 16) >> 3, r = (lane - 16) & 7;
    S.left_c[comp][r] = *reinterpret_cast<const uint32_t*>(&S.tc[comp][(r + 2) * CT + 8]);
  }
  if (lane == 0) S.saved_x = mx;
  wave_sync();
}

__global__ __launch_bounds__(64 * kDeblockWaves) void deblock_wavefront(DeblockArgs a) {
  __shared__ DeblockShared SS[kDeblockWaves];
  __shared__ int prog[kMaxRows];
  const Geom& g = a.g;
  const int slot = blockIdx.x;
  for (int i = threadIdx.x; i < g.hmb; i += blockDim.x) prog[i] = 0;
  const int w = wave_id();
  if (lane_id() == 0) SS[w].saved_x = -2;
  __syncthreads();
  DeblockShared& S = SS[w];
  for (int y = w; y < g.hmb; y += kDeblockWaves) {
    for (int x = 0; x < g.wmb; ++x) {
      if (y > 0) row_wait(prog, y - 1, min(x + 2, g.wmb), a.err);
      deblock_mb(a, S, slot, x, y);
      row_publish(prog, y, x + 1);
    }
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

extern "C" void mivc_launch_deblock(int B, int wmb, int hmb, uint8_t* rec_y, uint8_t* rec_u, uint8_t* rec_v,
                                    const void* hdr, const uint8_t* nz, int chroma_qp_offset, int alpha_off,
                                    int beta_off, int* err, void* stream) {
  DeblockArgs a;
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.rec_y = rec_y;
  a.rec_u = rec_u;
  a.rec_v = rec_v;
  a.hdr = static_cast<const mivc::h264::MbHeader*>(hdr);
  a.nz = nz;
  a.chroma_qp_offset = chroma_qp_offset;
  a.alpha_off = alpha_off;
  a.beta_off = beta_off;
  a.err = err;
  hipLaunchKernelGGL(deblock_wavefront, dim3(B), dim3(64 * kDeblockWaves), 0, static_cast<hipStream_t>(stream), a);
}
