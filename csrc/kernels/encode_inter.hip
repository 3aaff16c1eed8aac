// P-macroblock mode decision + transform/quant/reconstruction, fully parallel
// over macroblocks (inter prediction depends only on the previous frame's
// deblocked reconstruction, never on neighbours in the current frame):
//   * intra-vs-inter decision from the ME cost and the open-loop Intra16x16
//     estimate (MBs that go intra are flagged for the wavefront kernel);
//   * chroma motion compensation (eighth-sample bilinear, clause 8.4.2.2.2);
//   * 4x4 forward core transform, dead-zone quantisation, x264-style coefficient
//     decimation, dequantisation and the normative inverse transform, so the
//     reconstruction written here is exactly what a decoder produces.
// SURVEY.md K-C8.  One wave64 per macroblock: lanes 0-15 luma 4x4 blocks,
// lanes 16-23 chroma 4x4 blocks; grid = (nmb, B).
#include "kcommon.h"

namespace mivc {
namespace gpu {

using h264::MbHeader;

struct InterArgs {
  Geom g;
  const uint8_t *src_y, *src_u, *src_v;
  const uint8_t *ref_y, *ref_u, *ref_v;
  uint8_t *rec_y, *rec_u, *rec_v;
  const uint8_t* pred_y;   // [B, nmb, 256] from ME
  const int16_t* mv;       // [B, nmb, 2]
  const int* me_cost;      // [B, nmb]
  const int* intra_cost;   // [B, nmb]
  const int* qp;           // [B]
  int chroma_qp_offset;
  MbHeader* hdr;           // [B, nmb]
  int16_t* coef;           // [B, nmb, 408]
  uint8_t* nz;             // [B, nmb, 16] luma nonzero flags (raster 4x4)
  uint8_t* intra_flag;     // [B, nmb]
  int* intra_count;        // [B]
};

// x264 decimate_score for a 4x4 block in scan order (start..15)
__device__ __forceinline__ int decimate_score(const int* scan, int start) {
  const int tab[16] = {3, 2, 2, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  int idx = 15;
  while (idx >= start && scan[idx] == 0) --idx;
  int score = 0;
  while (idx >= start) {
    int v = scan[idx--];
    if (v > 1 || v < -1) return 9;
    int run = 0;
    while (idx >= start && scan[idx] == 0) {
      --idx;
      ++run;
    }
    score += tab[run];
  }
  return score;
}

__global__ __launch_bounds__(64) void encode_inter_mb(InterArgs a) {
  const Geom& g = a.g;
  const int mb = blockIdx.x, slot = blockIdx.y;
  const int mx = mb % g.wmb, my = mb / g.wmb;
  const int lane = threadIdx.x;
  const size_t o = static_cast<size_t>(slot) * g.nmb() + mb;
  const int W = g.W, cw = g.cw();
  const int qp = a.qp[slot];
  const int qpc = h264::chroma_qp(qp, a.chroma_qp_offset);

  __shared__ int s_score[24];
  __shared__ int s_cdc[2][4];
  __shared__ int s_clev[2][4];
  __shared__ int s_flags[4];  // [0] luma 8x8 keep mask, [1] chroma AC keep mask (bit per comp), [2] cbp

  const int mvx = a.mv[o * 2], mvy = a.mv[o * 2 + 1];
  const bool go_intra = a.intra_cost[o] < a.me_cost[o];
  MbHeader* h = a.hdr + o;
  int16_t* coef = a.coef + o * h264::kCoefPerMb;
  if (go_intra) {
    // the wavefront kernel encodes this MB closed-loop; leave a consistent placeholder
    if (lane == 0) {
      a.intra_flag[o] = 1;
      atomicAdd(a.intra_count + slot, 1);
      h->kind = h264::MBK_I16x16;
    }
    return;
  }

  const uint8_t* srcy = a.src_y + slot * g.ysize();
  const uint8_t* pred = a.pred_y + o * 256;
  int lv[16];     // raster levels of this lane's block
  int res[16];    // residual / reconstruction scratch
  int pr[16];     // prediction
  int comp = 0, cb = 0;
  const int X0 = mx * 16, Y0 = my * 16;

  if (lane < 16) {
    // ---- luma block (blkIdx order)
    int bx = h264::kBlkX[lane] * 4, by = h264::kBlkY[lane] * 4;
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        pr[y * 4 + x] = pred[(by + y) * 16 + bx + x];
        res[y * 4 + x] = static_cast<int>(srcy[static_cast<size_t>(Y0 + by + y) * W + X0 + bx + x]) - pr[y * 4 + x];
      }
    h264::forward_core4x4(res);
    int qbits = 15 + qp / 6;
#pragma unroll
    for (int r = 0; r < 16; ++r) lv[r] = h264::quant_coef(res[r], h264::kQuantMF[qp % 6][h264::kPosClass[r]], qbits, 11);
    int scan[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) scan[i] = lv[h264::kZigzag4x4[i]];
    s_score[lane] = decimate_score(scan, 0);
  } else if (lane < 24) {
    // ---- chroma block: MC + residual + forward + AC quant; DC handled after exchange
    comp = (lane - 16) >> 2;
    cb = (lane - 16) & 3;
    const uint8_t* srcc = (comp == 0 ? a.src_u : a.src_v) + slot * g.csize();
    const uint8_t* refc = (comp == 0 ? a.ref_u : a.ref_v) + slot * g.csize();
    int CH = g.ch();
    int bx = (cb & 1) * 4, by = (cb >> 1) * 4;
    int xf = mvx & 7, yf = mvy & 7;
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        int px = mx * 8 + bx + x, py = my * 8 + by + y;
        int xi = px + (mvx >> 3), yi = py + (mvy >> 3);
        int x0 = clampi(xi, 0, cw - 1), x1 = clampi(xi + 1, 0, cw - 1);
        int y0 = clampi(yi, 0, CH - 1), y1 = clampi(yi + 1, 0, CH - 1);
        int A = refc[static_cast<size_t>(y0) * cw + x0], B = refc[static_cast<size_t>(y0) * cw + x1];
        int C = refc[static_cast<size_t>(y1) * cw + x0], D = refc[static_cast<size_t>(y1) * cw + x1];
        pr[y * 4 + x] = ((8 - xf) * (8 - yf) * A + xf * (8 - yf) * B + (8 - xf) * yf * C + xf * yf * D + 32) >> 6;
        res[y * 4 + x] = static_cast<int>(srcc[static_cast<size_t>(py) * cw + px]) - pr[y * 4 + x];
      }
    h264::forward_core4x4(res);
    s_cdc[comp][cb] = res[0];
    int qbits = 15 + qpc / 6;
#pragma unroll
    for (int r = 0; r < 16; ++r) lv[r] = r == 0 ? 0 : h264::quant_coef(res[r], h264::kQuantMF[qpc % 6][h264::kPosClass[r]], qbits, 11);
    int scan[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) scan[i] = lv[h264::kZigzag4x4[i]];
    s_score[lane] = decimate_score(scan, 1);
  }
  __syncthreads();
  if (lane == 16 || lane == 20) {
    // chroma DC: 2x2 Hadamard + quantisation with qbits+1
    int c = lane == 16 ? 0 : 1;
    int d0 = s_cdc[c][0], d1 = s_cdc[c][1], d2 = s_cdc[c][2], d3 = s_cdc[c][3];
    int f[4] = {d0 + d1 + d2 + d3, d0 - d1 + d2 - d3, d0 + d1 - d2 - d3, d0 - d1 - d2 + d3};
    int qbits = 15 + qpc / 6;
#pragma unroll
    for (int i = 0; i < 4; ++i) s_clev[c][i] = h264::quant_coef(f[i], h264::kQuantMF[qpc % 6][0], qbits + 1, 11);
  }
  if (lane == 0) {
    int keep = 0, total = 0;
    for (int b8 = 0; b8 < 4; ++b8) {
      int s = s_score[b8 * 4] + s_score[b8 * 4 + 1] + s_score[b8 * 4 + 2] + s_score[b8 * 4 + 3];
      if (s >= 4) keep |= 1 << b8;
      total += s;
    }
    if (total < 6) keep = 0;
    int ckeep = 0;
    for (int c = 0; c < 2; ++c) {
      int s = s_score[16 + 4 * c] + s_score[17 + 4 * c] + s_score[18 + 4 * c] + s_score[19 + 4 * c];
      if (s >= 7) ckeep |= 1 << c;
    }
    s_flags[0] = keep;
    s_flags[1] = ckeep;
  }
  __syncthreads();
  if (lane < 16) {
    int b8 = lane >> 2;
    bool keep = (s_flags[0] >> b8) & 1;
    bool any = false;
    int16_t* dst = coef + h264::COEF_LUMA + lane * 16;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      int v = keep ? lv[h264::kZigzag4x4[i]] : 0;
      dst[i] = static_cast<int16_t>(v);
      any |= v != 0;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) res[r] = keep ? h264::dequant_coef(lv[r], qp, r) : 0;
    if (any) h264::inverse_core4x4(res);
    int bx = h264::kBlkX[lane] * 4, by = h264::kBlkY[lane] * 4;
    uint8_t* recy = a.rec_y + slot * g.ysize();
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      uint32_t word = 0;
#pragma unroll
      for (int x = 0; x < 4; ++x) word |= static_cast<uint32_t>(h264::clip1(pr[y * 4 + x] + (any ? res[y * 4 + x] : 0))) << (8 * x);
      *reinterpret_cast<uint32_t*>(recy + static_cast<size_t>(Y0 + by + y) * W + X0 + bx) = word;
    }
    a.nz[o * 16 + h264::kBlkX[lane] + 4 * h264::kBlkY[lane]] = any;
  } else if (lane < 24) {
    bool keep_ac = (s_flags[1] >> comp) & 1;
    int16_t* dst = coef + h264::COEF_CHROMA_AC + (comp * 4 + cb) * 16;
    bool any_ac = false;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      int v = (keep_ac && i > 0) ? lv[h264::kZigzag4x4[i]] : 0;
      dst[i] = static_cast<int16_t>(v);
      any_ac |= v != 0;
    }
    const int* cl = s_clev[comp];
    if (cb == 0)
      for (int i = 0; i < 4; ++i) coef[h264::COEF_CHROMA_DC + comp * 4 + i] = static_cast<int16_t>(cl[i]);
    int f[4] = {cl[0] + cl[1] + cl[2] + cl[3], cl[0] - cl[1] + cl[2] - cl[3], cl[0] + cl[1] - cl[2] - cl[3],
                cl[0] - cl[1] - cl[2] + cl[3]};
    int ls = 16 * h264::kDequantV[qpc % 6][0];
#pragma unroll
    for (int r = 0; r < 16; ++r) res[r] = (keep_ac && r > 0) ? h264::dequant_coef(lv[r], qpc, r) : 0;
    res[0] = ((f[cb] * ls) << (qpc / 6)) >> 5;
    bool any = any_ac || cl[0] || cl[1] || cl[2] || cl[3];
    if (any) h264::inverse_core4x4(res);
    uint8_t* recc = (comp == 0 ? a.rec_u : a.rec_v) + slot * g.csize();
    int bx = (cb & 1) * 4, by = (cb >> 1) * 4;
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      uint32_t word = 0;
#pragma unroll
      for (int x = 0; x < 4; ++x) word |= static_cast<uint32_t>(h264::clip1(pr[y * 4 + x] + (any ? res[y * 4 + x] : 0))) << (8 * x);
      *reinterpret_cast<uint32_t*>(recc + static_cast<size_t>(my * 8 + by + y) * cw + mx * 8 + bx) = word;
    }
  } else if (lane < 40) {
    coef[h264::COEF_LUMA_DC + (lane - 24)] = 0;
  } else if (lane == 40) {
    h->kind = h264::MBK_P16x16;
    h->qp = static_cast<int8_t>(qp);
    h->i16_mode = 0;
    h->chroma_mode = 0;
    h->flags = 0;
    for (int q = 0; q < 4; ++q) {
      h->mv[q][0] = static_cast<int16_t>(mvx);
      h->mv[q][1] = static_cast<int16_t>(mvy);
    }
    a.intra_flag[o] = 0;
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

extern "C" void mivc_launch_encode_inter(int B, int wmb, int hmb, const uint8_t* src_y, const uint8_t* src_u,
                                         const uint8_t* src_v, const uint8_t* ref_y, const uint8_t* ref_u,
                                         const uint8_t* ref_v, uint8_t* rec_y, uint8_t* rec_u, uint8_t* rec_v,
                                         const uint8_t* pred_y, const int16_t* mv, const int* me_cost,
                                         const int* intra_cost, const int* qp, int chroma_qp_offset, void* hdr,
                                         int16_t* coef, uint8_t* nz, uint8_t* intra_flag, int* intra_count,
                                         void* stream) {
  InterArgs a;
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.src_y = src_y;
  a.src_u = src_u;
  a.src_v = src_v;
  a.ref_y = ref_y;
  a.ref_u = ref_u;
  a.ref_v = ref_v;
  a.rec_y = rec_y;
  a.rec_u = rec_u;
  a.rec_v = rec_v;
  a.pred_y = pred_y;
  a.mv = mv;
  a.me_cost = me_cost;
  a.intra_cost = intra_cost;
  a.qp = qp;
  a.chroma_qp_offset = chroma_qp_offset;
  a.hdr = static_cast<MbHeader*>(hdr);
  a.coef = coef;
  a.nz = nz;
  a.intra_flag = intra_flag;
  a.intra_count = intra_count;
  hipLaunchKernelGGL(encode_inter_mb, dim3(wmb * hmb, B), dim3(64), 0, static_cast<hipStream_t>(stream), a);
}
