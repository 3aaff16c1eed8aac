// Motion estimation for P macroblocks:
//   1. integer full search in a (2R+1)^2 window around a temporal predictor,
//      SAD with v_sad_u8 on a reference window staged in LDS (unaligned rows
//      re-aligned with v_alignbyte_b32);
//   2. half-sample then quarter-sample refinement around the best integer
//      vector, on half-pel planes (b, h, j of clause 8.4.2.2.1) computed once per
//      MB into LDS; cost = SATD (4x4 Hadamard) + lambda * |mvd| bits.
// One wave64 per macroblock; grid = (nmb, B).
#include "kcommon.h"

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
};

constexpr int kMaxR = 16;
constexpr int kWinRows = 16 + 2 * kMaxR;      // 48
constexpr int kWinWords = (16 + 2 * kMaxR + 4) / 4;  // 13 words (52 bytes) per row

__device__ __forceinline__ int wave_min_key(int key) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    int o = __shfl_xor(key, off, 64);
    key = o < key ? o : key;
  }
  return key;
}

__global__ __launch_bounds__(64) void me_p16x16(MeArgs a) {
  const Geom& g = a.g;
  const int mb = blockIdx.x, slot = blockIdx.y;
  const int mx = mb % g.wmb, my = mb / g.wmb;
  const int lane = threadIdx.x;
  const int X0 = mx * 16, Y0 = my * 16;
  const uint8_t* src = a.src_y + slot * g.ysize();
  const uint8_t* ref = a.ref_y + slot * g.ysize();
  const int W = g.W, H = g.H;
  const int qp = a.qp[slot];
  const int lambda = h264::kLambda[qp];
  const int R = a.range < kMaxR ? a.range : kMaxR;

  __shared__ uint32_t s_win[kWinRows * kWinWords];
  __shared__ uint8_t s_src[256];
  __shared__ uint8_t s_G[26 * 26];
  __shared__ int16_t s_B1[25 * 20];
  __shared__ uint8_t s_b[20 * 20], s_h[20 * 20], s_j[20 * 20];

  // ---- stage the source MB first (needed to rank the search-centre candidates)
  for (int i = lane; i < 256; i += 64) s_src[i] = src[static_cast<size_t>(Y0 + (i >> 4)) * W + X0 + (i & 15)];
  __syncthreads();
  // ---- search centre: best (SAD + mv cost) of the temporal predictors at this MB and its
  // left/top/right neighbours in the previous frame, and the zero vector
  int pmx = 0, pmy = 0;
  int cx = 0, cy = 0;
  if (a.pred_mv) {
    const int16_t* pm = a.pred_mv + static_cast<size_t>(slot) * g.nmb() * 2;
    pmx = pm[mb * 2];
    pmy = pm[mb * 2 + 1];
    int cand[5][2];
    int nc = 0;
    cand[nc][0] = (pmx + 2) >> 2; cand[nc][1] = (pmy + 2) >> 2; ++nc;
    if (mx > 0) { cand[nc][0] = (pm[(mb - 1) * 2] + 2) >> 2; cand[nc][1] = (pm[(mb - 1) * 2 + 1] + 2) >> 2; ++nc; }
    if (my > 0) { cand[nc][0] = (pm[(mb - g.wmb) * 2] + 2) >> 2; cand[nc][1] = (pm[(mb - g.wmb) * 2 + 1] + 2) >> 2; ++nc; }
    if (mx < g.wmb - 1) { cand[nc][0] = (pm[(mb + 1) * 2] + 2) >> 2; cand[nc][1] = (pm[(mb + 1) * 2 + 1] + 2) >> 2; ++nc; }
    cand[nc][0] = 0; cand[nc][1] = 0; ++nc;
    int best = 0x7FFFFFFF;
    const int r = lane >> 2, c4 = (lane & 3) * 4;
    for (int k = 0; k < nc; ++k) {
      int dx = clampi(cand[k][0], -128, 128), dy = clampi(cand[k][1], -128, 128);
      int yy = clampi(Y0 + r + dy, 0, H - 1);
      const uint8_t* rp = ref + static_cast<size_t>(yy) * W;
      int sad = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        int d = static_cast<int>(s_src[r * 16 + c4 + q]) - rp[clampi(X0 + c4 + q + dx, 0, W - 1)];
        sad += d < 0 ? -d : d;
      }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) sad += __shfl_xor(sad, off, 64);
      int cost = sad + lambda * (h264::se_bits(dx * 4 - pmx) + h264::se_bits(dy * 4 - pmy));
      if (cost < best) {
        best = cost;
        cx = dx;
        cy = dy;
      }
    }
  }

  // ---- stage the reference window
  const int wx0 = X0 + cx - R, wy0 = Y0 + cy - R;
  const int wrows = 16 + 2 * R, wbytes = (16 + 2 * R + 4);
  for (int i = lane; i < wrows * kWinWords; i += 64) {
    int r = i / kWinWords, w = i % kWinWords;
    uint32_t word = 0;
    int yy = clampi(wy0 + r, 0, H - 1);
    const uint8_t* row = ref + static_cast<size_t>(yy) * W;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      int xx = wx0 + w * 4 + k;
      uint32_t px = (w * 4 + k < wbytes) ? row[clampi(xx, 0, W - 1)] : 0u;
      word |= px << (8 * k);
    }
    s_win[r * kWinWords + w] = word;
  }
  __syncthreads();
  uint32_t srcw[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) srcw[i] = reinterpret_cast<const uint32_t*>(s_src)[i];

  // ---- integer full search
  const int side = 2 * R + 1, ncand = side * side;
  int best_key = 0x7FFFFFFF;
  for (int p = lane; p < ncand; p += 64) {
    int dy = p / side, dx = p % side;
    int w0 = dx >> 2, sh = dx & 3;
    uint32_t sad = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint32_t* rowp = s_win + (dy + r) * kWinWords + w0;
      uint32_t a0 = rowp[0], a1 = rowp[1], a2 = rowp[2], a3 = rowp[3], a4 = rowp[4];
      uint32_t b0 = __builtin_amdgcn_alignbyte(a1, a0, sh);
      uint32_t b1 = __builtin_amdgcn_alignbyte(a2, a1, sh);
      uint32_t b2 = __builtin_amdgcn_alignbyte(a3, a2, sh);
      uint32_t b3 = __builtin_amdgcn_alignbyte(a4, a3, sh);
      sad = sad4(srcw[r * 4 + 0], b0, sad);
      sad = sad4(srcw[r * 4 + 1], b1, sad);
      sad = sad4(srcw[r * 4 + 2], b2, sad);
      sad = sad4(srcw[r * 4 + 3], b3, sad);
    }
    int mvx = (cx + dx - R) * 4, mvy = (cy + dy - R) * 4;
    int cost = static_cast<int>(sad) + lambda * (h264::se_bits(mvx - pmx) + h264::se_bits(mvy - pmy));
    int key = (cost << 12) | p;
    best_key = key < best_key ? key : best_key;
  }
  // zero vector (may lie outside the window)
  {
    uint32_t sad = 0;
    int r = lane >> 2, c4 = (lane & 3) * 4;
    const uint8_t* rp = ref + static_cast<size_t>(Y0 + r) * W + X0 + c4;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      int d = static_cast<int>(s_src[r * 16 + c4 + k]) - rp[k];
      sad += d < 0 ? -d : d;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) sad += __shfl_xor(static_cast<int>(sad), off, 64);
    int cost = static_cast<int>(sad) + lambda * (h264::se_bits(-pmx) + h264::se_bits(-pmy));
    int key = (cost << 12) | 4095;
    best_key = key < best_key ? key : best_key;
  }
  best_key = wave_min_key(best_key);
  int bp = best_key & 4095;
  int bx, by;  // integer displacement
  if (bp == 4095) {
    bx = 0;
    by = 0;
  } else {
    bx = cx + (bp % side) - R;
    by = cy + (bp / side) - R;
  }
  int best_mvx = bx * 4, best_mvy = by * 4;

  // ---- sub-pel refinement
  // planes origin: integer (bx-2, by-2) relative to the MB; G origin (bx-4, by-4)
  for (int i = lane; i < 26 * 26; i += 64) {
    int r = i / 26, c = i % 26;
    int yy = clampi(Y0 + by - 4 + r, 0, H - 1), xx = clampi(X0 + bx - 4 + c, 0, W - 1);
    s_G[i] = ref[static_cast<size_t>(yy) * W + xx];
  }
  __syncthreads();
  for (int i = lane; i < 25 * 20; i += 64) {
    int r = i / 20, u = i % 20;
    const uint8_t* gr = s_G + r * 26 + u;
    s_B1[i] = static_cast<int16_t>(h264::tap6(gr[0], gr[1], gr[2], gr[3], gr[4], gr[5]));
  }
  __syncthreads();
  for (int i = lane; i < 400; i += 64) {
    int v = i / 20, u = i % 20;
    s_b[i] = static_cast<uint8_t>(h264::clip1((s_B1[(v + 2) * 20 + u] + 16) >> 5));
    const uint8_t* gc = s_G + v * 26 + u + 2;
    s_h[i] = static_cast<uint8_t>(h264::clip1((h264::tap6(gc[0], gc[26], gc[52], gc[78], gc[104], gc[130]) + 16) >> 5));
    const int16_t* bc = s_B1 + v * 20 + u;
    int j1 = h264::tap6(bc[0], bc[20], bc[40], bc[60], bc[80], bc[100]);
    s_j[i] = static_cast<uint8_t>(h264::clip1((j1 + 512) >> 10));
  }
  __syncthreads();

  auto G = [&](int u, int v) -> int { return s_G[(v + 2) * 26 + u + 2]; };
  auto qpel = [&](int u, int v, int xf, int yf) -> int {
    if (xf == 0 && yf == 0) return G(u, v);
    if (yf == 0) {
      int b = s_b[v * 20 + u];
      if (xf == 2) return b;
      return ((xf == 1 ? G(u, v) : G(u + 1, v)) + b + 1) >> 1;
    }
    if (xf == 0) {
      int h = s_h[v * 20 + u];
      if (yf == 2) return h;
      return ((yf == 1 ? G(u, v) : G(u, v + 1)) + h + 1) >> 1;
    }
    if (xf == 2 && yf == 2) return s_j[v * 20 + u];
    if (xf == 2) return (s_j[v * 20 + u] + (yf == 1 ? s_b[v * 20 + u] : s_b[(v + 1) * 20 + u]) + 1) >> 1;
    if (yf == 2) return (s_j[v * 20 + u] + (xf == 1 ? s_h[v * 20 + u] : s_h[v * 20 + u + 1]) + 1) >> 1;
    int b = yf == 1 ? s_b[v * 20 + u] : s_b[(v + 1) * 20 + u];
    int h = xf == 1 ? s_h[v * 20 + u] : s_h[v * 20 + u + 1];
    return (b + h + 1) >> 1;
  };
  // SATD of candidate (dqx, dqy) quarter offsets relative to (4bx, 4by): this lane does 4x4 block (lane&15)
  auto satd_cand = [&](int dqx, int dqy) -> int {
    int blk = lane & 15;
    int px0 = (blk & 3) * 4, py0 = (blk >> 2) * 4;
    int xf = dqx & 3, yf = dqy & 3, ox = dqx >> 2, oy = dqy >> 2;
    int r[16];
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        int u = px0 + x + ox + 2, v = py0 + y + oy + 2;
        r[y * 4 + x] = static_cast<int>(s_src[(py0 + y) * 16 + px0 + x]) - qpel(u, v, xf, yf);
      }
    int s = h264::satd4x4(r);
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
    return s;
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
    // centre + 8 half-pel neighbours (3 passes of 4 candidates, 16 lanes each)
    int bkey = 0x7FFFFFFF;
    const int ncand_h = a.subpel >= 1 ? 9 : 1;
    for (int base = 0; base < ncand_h; base += 4) {
      int ci = base + (lane >> 4);
      int c = ci < ncand_h ? ci : 0;
      int ox, oy;
      ring(c, 2, &ox, &oy);
      int s = satd_cand(ox, oy);
      int mvx = best_mvx + ox, mvy = best_mvy + oy;
      int cost = s + lambda * (h264::se_bits(mvx - pmx) + h264::se_bits(mvy - pmy));
      int key = ci < ncand_h ? ((cost << 4) | c) : 0x7FFFFFFF;
      bkey = key < bkey ? key : bkey;
    }
    bkey = wave_min_key(bkey);
    best_cost = bkey >> 4;
    ring(bkey & 15, 2, &hx, &hy);
    if (a.subpel >= 2) {
      int qkey = (best_cost << 4) | 0;
      for (int base = 1; base < 9; base += 4) {
        int ci = base + (lane >> 4);
        int ox, oy;
        ring(ci, 1, &ox, &oy);
        int s = satd_cand(hx + ox, hy + oy);
        int mvx = best_mvx + hx + ox, mvy = best_mvy + hy + oy;
        int cost = s + lambda * (h264::se_bits(mvx - pmx) + h264::se_bits(mvy - pmy));
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
    best_mvx += hx;
    best_mvy += hy;
  }
  const size_t o = static_cast<size_t>(slot) * g.nmb() + mb;
  // ---- final luma prediction for the chosen vector
  {
    int dqx = best_mvx - 4 * bx, dqy = best_mvy - 4 * by;
    int xf = dqx & 3, yf = dqy & 3, ox = dqx >> 2, oy = dqy >> 2;
    uint32_t word = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      int i = lane * 4 + k;
      int px = i & 15, py = i >> 4;
      word |= static_cast<uint32_t>(qpel(px + ox + 2, py + oy + 2, xf, yf)) << (8 * k);
    }
    reinterpret_cast<uint32_t*>(a.out_pred + o * 256)[lane] = word;
  }
  // ---- open-loop Intra16x16 estimate on source pixels: lane = mode * 16 + block
  {
    int mode = lane >> 4, blk = lane & 15;
    bool has_top = my > 0, has_left = mx > 0;
    bool ok = (mode == 0 && has_top) || (mode == 1 && has_left) || mode == 2 || (mode == 3 && has_top && has_left);
    int top[16], left[16], tl = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      top[i] = has_top ? src[static_cast<size_t>(Y0 - 1) * W + X0 + i] : 0;
      left[i] = has_left ? src[static_cast<size_t>(Y0 + i) * W + X0 - 1] : 0;
    }
    if (has_top && has_left) tl = src[static_cast<size_t>(Y0 - 1) * W + X0 - 1];
    int pa = 0, pb = 0, pc = 0, dc = 0;
    if (mode == 3 && ok) h264::i16_plane_params(top, left, tl, &pa, &pb, &pc);
    if (mode == 2) dc = h264::i16_dc(top, left, (has_top ? h264::AV_TOP : 0) | (has_left ? h264::AV_LEFT : 0));
    int bx4 = (blk & 3) * 4, by4 = (blk >> 2) * 4;
    int r[16];
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        int X = bx4 + x, Y = by4 + y, pv;
        if (mode == 0) pv = top[X];
        else if (mode == 1) pv = left[Y];
        else if (mode == 2) pv = dc;
        else pv = h264::clip1((pa + pb * (X - 7) + pc * (Y - 7) + 16) >> 5);
        r[y * 4 + x] = static_cast<int>(s_src[Y * 16 + X]) - pv;
      }
    int s = h264::satd4x4(r);
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
    int key = ok ? s : 0x3FFFFFFF;
    key = min(key, __shfl_xor(key, 16, 64));
    key = min(key, __shfl_xor(key, 32, 64));
    if (lane == 0) {
      a.out_mv[o * 2] = static_cast<int16_t>(best_mvx);
      a.out_mv[o * 2 + 1] = static_cast<int16_t>(best_mvy);
      a.out_cost[o] = best_cost;
      a.out_intra_cost[o] = key + lambda * 4;
    }
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

extern "C" void mivc_launch_me(int B, int wmb, int hmb, const uint8_t* src_y, const uint8_t* ref_y,
                               const int16_t* pred_mv, int16_t* out_mv, int* out_cost, uint8_t* out_pred,
                               int* out_intra_cost, const int* qp, int range, int subpel, void* stream) {
  MeArgs a;
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.src_y = src_y;
  a.ref_y = ref_y;
  a.pred_mv = pred_mv;
  a.out_mv = out_mv;
  a.out_cost = out_cost;
  a.out_pred = out_pred;
  a.out_intra_cost = out_intra_cost;
  a.qp = qp;
  a.range = range;
  a.subpel = subpel;
  hipLaunchKernelGGL(me_p16x16, dim3(wmb * hmb, B), dim3(64), 0, static_cast<hipStream_t>(stream), a);
}
