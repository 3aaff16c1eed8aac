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
constexpr int CT = 10;  // chroma tile stride: 2 halo + 8

struct DeblockShared {
  uint8_t ty[LT * LT];
  uint8_t tc[2][CT * CT];
  int bs[2][4][4];         // [dir][edge][segment]
  uint8_t left_y[16][4];   // previous MB's columns 12..15 after filtering
  uint8_t left_c[2][8][2]; // previous MB's chroma columns 6..7
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

__device__ __forceinline__ void deblock_mb(const DeblockArgs& a, DeblockShared& S, int slot, int mx, int my) {
  const Geom& g = a.g;
  const int lane = lane_id();
  const int W = g.W, cw = g.cw();
  const size_t o = static_cast<size_t>(slot) * g.nmb() + my * g.wmb + mx;
  uint8_t* recy = a.rec_y + slot * g.ysize();
  const int X0 = mx * 16, Y0 = my * 16;
  const bool has_left = mx > 0, has_top = my > 0;

  // ---- load tiles
  for (int i = lane; i < 16 * 16; i += 64) {
    int r = i >> 4, c = i & 15;
    S.ty[(r + 4) * LT + c + 4] = recy[static_cast<size_t>(Y0 + r) * W + X0 + c];
  }
  if (has_top)
    for (int i = lane; i < 4 * 16; i += 64) {
      int r = i >> 4, c = i & 15;
      S.ty[r * LT + c + 4] = recy[static_cast<size_t>(Y0 - 4 + r) * W + X0 + c];
    }
  if (has_left && lane < 16) {
    for (int c = 0; c < 4; ++c) {
      S.ty[(lane + 4) * LT + c] =
          S.saved_x == mx - 1 ? S.left_y[lane][c] : recy[static_cast<size_t>(Y0 + lane) * W + X0 - 4 + c];
    }
  }
  for (int comp = 0; comp < 2; ++comp) {
    uint8_t* rc = (comp == 0 ? a.rec_u : a.rec_v) + slot * g.csize();
    uint8_t* t = S.tc[comp];
    {
      int r = lane >> 3, c = lane & 7;
      t[(r + 2) * CT + c + 2] = rc[static_cast<size_t>(my * 8 + r) * cw + mx * 8 + c];
    }
    if (has_top && lane < 16) {
      int r = lane >> 3, c = lane & 7;
      t[r * CT + c + 2] = rc[static_cast<size_t>(my * 8 - 2 + r) * cw + mx * 8 + c];
    }
    if (has_left && lane < 16) {
      int r = lane >> 1, c = lane & 1;
      t[(r + 2) * CT + c] =
          S.saved_x == mx - 1 ? S.left_c[comp][r][c] : rc[static_cast<size_t>(my * 8 + r) * cw + mx * 8 - 2 + c];
    }
  }
  // ---- boundary strengths: lane = dir*16 + edge*4 + seg
  if (lane < 32) {
    int dir = lane >> 4, e = (lane >> 2) & 3, k = lane & 3;
    const MbHeader& Q = a.hdr[o];
    int bs = 0;
    bool mbedge = e == 0;
    bool avail = !mbedge || (dir == 0 ? has_left : has_top);
    if (avail) {
      size_t op = mbedge ? (dir == 0 ? o - 1 : o - g.wmb) : o;
      const MbHeader& P = a.hdr[op];
      int rq = dir == 0 ? (e + 4 * k) : (k + 4 * e);
      int rp = dir == 0 ? (mbedge ? 3 + 4 * k : e - 1 + 4 * k) : (mbedge ? k + 12 : k + 4 * (e - 1));
      bool iq = h264::mbk_is_intra(Q.kind), ip = h264::mbk_is_intra(P.kind);
      if (mbedge && (iq || ip)) bs = 4;
      else if (iq || ip) bs = 3;
      else if (a.nz[op * 16 + rp] || a.nz[o * 16 + rq]) bs = 2;
      else {
        int mp[2], mq[2];
        blk_mv(P, rp, mp);
        blk_mv(Q, rq, mq);
        int dx = mp[0] - mq[0], dy = mp[1] - mq[1];
        bs = (dx >= 4 || dx <= -4 || dy >= 4 || dy <= -4) ? 1 : 0;
      }
    }
    S.bs[dir][e][k] = bs;
  }
  wave_sync();

  const int qpq = a.hdr[o].qp;
  // ---- vertical edges, then horizontal edges
  for (int dir = 0; dir < 2; ++dir) {
    for (int e = 0; e < 4; ++e) {
      if (e == 0 && !(dir == 0 ? has_left : has_top)) continue;
      int qpp = e == 0 ? a.hdr[dir == 0 ? o - 1 : o - g.wmb].qp : qpq;
      if (lane < 16) {
        int bs = S.bs[dir][e][lane >> 2];
        if (bs) {
          int qpav = (qpp + qpq + 1) >> 1;
          int ia = clampi(qpav + a.alpha_off, 0, 51), ib = clampi(qpav + a.beta_off, 0, 51);
          int tc0 = bs < 4 ? h264::kTc0[ia][bs - 1] : 0;
          uint8_t* q0 = dir == 0 ? &S.ty[(lane + 4) * LT + 4 + 4 * e] : &S.ty[(4 + 4 * e) * LT + 4 + lane];
          filter_line(q0, dir == 0 ? 1 : LT, bs, h264::kAlpha[ia], h264::kBeta[ib], tc0, false);
        }
      } else if (lane < 32 && (e == 0 || e == 2)) {
        int comp = (lane - 16) >> 3, i = (lane - 16) & 7;
        int bs = S.bs[dir][e][i >> 1];
        if (bs) {
          int cp = h264::chroma_qp(qpp, a.chroma_qp_offset), cq = h264::chroma_qp(qpq, a.chroma_qp_offset);
          int qpav = (cp + cq + 1) >> 1;
          int ia = clampi(qpav + a.alpha_off, 0, 51), ib = clampi(qpav + a.beta_off, 0, 51);
          int tc0 = bs < 4 ? h264::kTc0[ia][bs - 1] : 0;
          int ce = e >> 1;
          uint8_t* t = S.tc[comp];
          uint8_t* q0 = dir == 0 ? &t[(i + 2) * CT + 2 + 4 * ce] : &t[(2 + 4 * ce) * CT + 2 + i];
          filter_line(q0, dir == 0 ? 1 : CT, bs, h264::kAlpha[ia], h264::kBeta[ib], tc0, true);
        }
      }
      wave_sync();
    }
  }
  // ---- write back: MB interior + modified halo (3 luma / 1 chroma lines)
  for (int i = lane; i < 16 * 16; i += 64) {
    int r = i >> 4, c = i & 15;
    recy[static_cast<size_t>(Y0 + r) * W + X0 + c] = S.ty[(r + 4) * LT + c + 4];
  }
  if (has_top && lane < 48) {
    int r = lane >> 4, c = lane & 15;  // rows -3..-1
    recy[static_cast<size_t>(Y0 - 3 + r) * W + X0 + c] = S.ty[(r + 1) * LT + c + 4];
  }
  if (has_left && lane < 48) {
    int r = lane / 3, c = lane % 3;  // cols -3..-1
    recy[static_cast<size_t>(Y0 + r) * W + X0 - 3 + c] = S.ty[(r + 4) * LT + c + 1];
  }
  for (int comp = 0; comp < 2; ++comp) {
    uint8_t* rc = (comp == 0 ? a.rec_u : a.rec_v) + slot * g.csize();
    const uint8_t* t = S.tc[comp];
    {
      int r = lane >> 3, c = lane & 7;
      rc[static_cast<size_t>(my * 8 + r) * cw + mx * 8 + c] = t[(r + 2) * CT + c + 2];
    }
    if (has_top && lane < 8) rc[static_cast<size_t>(my * 8 - 1) * cw + mx * 8 + lane] = t[1 * CT + lane + 2];
    if (has_left && lane >= 8 && lane < 16) {
      int r = lane - 8;
      rc[static_cast<size_t>(my * 8 + r) * cw + mx * 8 - 1] = t[(r + 2) * CT + 1];
    }
  }
  wave_sync();
  // ---- keep this MB's right edge for the next iteration (final values)
  if (lane < 16)
    for (int c = 0; c < 4; ++c) S.left_y[lane][c] = S.ty[(lane + 4) * LT + 16 + c];
  if (lane >= 16 && lane < 48) {
    int comp = (lane - 16) >> 4, r = ((lane - 16) >> 1) & 7, c = lane & 1;
    S.left_c[comp][r][c] = S.tc[comp][(r + 2) * CT + 8 + c];
  }
  if (lane == 0) S.saved_x = mx;
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
