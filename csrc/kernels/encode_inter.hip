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
// lanes 16-23 chroma 4x4 blocks (two MBs per wave, see encode_inter_mb).
#include "h264_trellis.h"

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
  const int16_t* mv8;      // [B, nmb, 4, 2] per-quadrant vectors of P partitions (nullable: 16x16)
  const int* me_cost;      // [B, nmb]
  const int* intra_cost;   // [B, nmb]
  const int* qp;           // [B]
  const int8_t* aq;        // [B, nmb] adaptive-quantisation QP offsets (nullable)
  int chroma_qp_offset;
  MbHeader* hdr;           // [B, nmb]
  int16_t* coef;           // [B, nmb, 408]
  uint8_t* nz;             // [B, nmb, 16] luma nonzero flags (raster 4x4)
  uint8_t* intra_flag;     // [B, nmb]
  int* intra_count;        // [B]
  // B pictures (bmode): the motion of every MB is already in hdr (kind / ref / mv per
  // quadrant, written by b_decide); chroma predicts from ref (list 0) and / or ref1
  // (list 1), averaged for bi-prediction; pred_y is b_decide's luma prediction
  const uint8_t *ref1_u, *ref1_v;
  int bmode;
  int w1[4];               // B pictures: implicit bi-prediction weight of list 1 per refIdxL0 (32: average)
  int t8;                  // High profile: choose the 8x8 transform per MB (sa8d < satd, as x264)
  // several list-0 pictures (x264 --ref): chroma of RefPicList0[r] (entry 0 = ref_u / ref_v);
  // P pictures take r from mref (the reference selection, nullable: 0), B pictures from the
  // records b_decide wrote
  const uint8_t* refs_u[4];
  const uint8_t* refs_v[4];
  const int8_t* mref;      // [B, nmb] (P pictures)
  // explicit weighted prediction of RefPicList0[0] in P pictures (nullable): [B, 8] = luma
  // weight, offset, log2 denominator, Cb weight, offset, Cr weight, offset, chroma denominator
  const int* wp;
  // x264 --trellis 1 (its default: on the final encode of each MB): levels by a rate-distortion
  // choice instead of the dead-zone rounding (trellis_lite below); 0 = off, 1 = 4x4 luma only
  // (round 3), 2 = also the 8x8 luma blocks and the chroma AC blocks
  int trellis;
  float trellis_lambda;    // multiplier of the SSD lambda 0.85 * 2^((QP - 12) / 3)
  // routed (route.h): ref_* / refs_* / ref1_* / rec_* are pools [B, nbuf, plane]; slots coding a
  // P (bmode 0) or B (bmode 1) picture take their roles and implicit weights from SlotRoute
  const SlotRoute* rt;
  int nbuf;
};

// trellis_lite4x4 / trellis_lite8_chunk: h264_trellis.h

// clause 8.4.2.3.2 for one sample: ((p * w + 2^(d-1)) >> d) + o, clipped
__device__ __forceinline__ int wp_sample(int p, int w, int o, int d) {
  return h264::clip1((d >= 1 ? ((p * w + (1 << (d - 1))) >> d) : p * w) + o);
}


// Eighth-sample chroma prediction (clause 8.4.2.2.2) of a 4x4 block at (px0, py0) of a
// cw x ch plane with vector (mvx, mvy) (quarter-luma = eighth-chroma units).
__device__ __forceinline__ void chroma_mc4x4(const uint8_t* refc, int cw, int CH, int px0, int py0, int mvx, int mvy,
                                             int (&pv)[4][4]) {
  const int xf = mvx & 7, yf = mvy & 7;
  const int xi = px0 + (mvx >> 3), yi = py0 + (mvy >> 3);
  int rw[5][5];  // reference samples (rows yi..yi+4, cols xi..xi+4), edge-clamped
  if (xi >= 0 && xi + 8 <= cw && yi >= 0 && yi + 5 <= CH) {
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const uint8_t* row = refc + static_cast<size_t>(yi + r) * cw;
      const int a = xi & ~3;
      const uint32_t w0 = *reinterpret_cast<const uint32_t*>(row + a), w1 = *reinterpret_cast<const uint32_t*>(row + a + 4);
      const uint32_t w4 = __builtin_amdgcn_alignbyte(w1, w0, xi & 3), w5 = row[xi + 4];
#pragma unroll
      for (int c = 0; c < 4; ++c) rw[r][c] = __builtin_amdgcn_ubfe(w4, 8 * c, 8);
      rw[r][4] = w5;
    }
  } else {
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const uint8_t* row = refc + static_cast<size_t>(clampi(yi + r, 0, CH - 1)) * cw;
#pragma unroll
      for (int c = 0; c < 5; ++c) rw[r][c] = row[clampi(xi + c, 0, cw - 1)];
    }
  }
  const int wA = (8 - xf) * (8 - yf), wB = xf * (8 - yf), wC = (8 - xf) * yf, wD = xf * yf;
#pragma unroll
  for (int y = 0; y < 4; ++y)
#pragma unroll
    for (int x = 0; x < 4; ++x)
      pv[y][x] = (wA * rw[y][x] + wB * rw[y][x + 1] + wC * rw[y + 1][x] + wD * rw[y + 1][x + 1] + 32) >> 6;
}

// x264 decimate_score of a 4x4 block in scan order (start..15), branch-free: 9 if any
// |level| > 1, else the sum over non-zero levels of kTab[zeros between it and the
// previous non-zero level (or `start`)], kTab = {3, 2, 2, 1, 1, 1, 0, ...}.
__device__ __forceinline__ int decimate_score(const int* scan, int start) {
  int score = 0, last = start - 1;
  bool big = false;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (i < start) continue;
    const int v = scan[i];
    const bool nzv = v != 0;
    big |= v > 1 || v < -1;
    const int run = i - last - 1;
    const int t = run == 0 ? 3 : (run <= 2 ? 2 : (run <= 5 ? 1 : 0));
    score += nzv ? t : 0;
    last = nzv ? i : last;
  }
  return big ? 9 : score;
}

// 4 bytes of a reference row starting at byte x (any alignment), from an aligned dword pair
__device__ __forceinline__ uint32_t ld4(const uint8_t* row, int x) {
  const int a = x & ~3;
  const uint32_t w0 = *reinterpret_cast<const uint32_t*>(row + a), w1 = *reinterpret_cast<const uint32_t*>(row + a + 4);
  return __builtin_amdgcn_alignbyte(w1, w0, x & 3);
}

// Two macroblocks per wave64 (lanes 0-31 MB 2i, 32-63 MB 2i+1); in each half lanes 0-15
// code the luma 4x4 blocks (blkIdx order), 16-23 the chroma 4x4 blocks, 24-31 records.
// Rows move as dwords (prediction, source, reference, reconstruction), levels as
// 16-byte stores, and the decimation score is branch-free.
// 4 waves per SIMD (128 VGPRs, a 16-byte spill) instead of the compiler's 3 at 140: inter
// 316 -> 274 ms per headline step, bytes unchanged (profiles/r5_occupancy_ab.md); at 5 waves
// the 132-byte spill made it slower (380 ms)
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 8))) void encode_inter_mb(InterArgs a) {
  const Geom& g = a.g;
  const int lane = threadIdx.x, half = lane >> 5, hl = lane & 31;
  const int nmb = g.nmb();
  int ux, slot;
  xcd_unit_slot(ux, slot);
  if (!route_active(a.rt, slot, a.bmode ? SK_B : SK_P)) return;  // wave-uniform
  const size_t rcur = route_index(a.rt, a.nbuf, slot, RO_CUR);
  const int mb = ux * 2 + half;
  const bool live = mb < nmb;
  const int mbc = live ? mb : nmb - 1;
  const int mx = mbc % g.wmb, my = mbc / g.wmb;
  const size_t o = static_cast<size_t>(slot) * nmb + mbc;
  const int W = g.W, cw = g.cw(), CH = g.ch();
  // QP is uniform within each half-wave (one MB) but, with adaptive quantisation, not
  // across the wave: fetch both halves' QPs into SGPRs so every table row below is a
  // scalar load, then select per lane
  const int qp_l = clampi(a.qp[slot] + (a.aq ? a.aq[o] : 0), 0, 51);
  const int qp0 = __builtin_amdgcn_readlane(qp_l, 0), qp1 = __builtin_amdgcn_readlane(qp_l, 32);
  const int qpc0 = h264::chroma_qp(qp0, a.chroma_qp_offset), qpc1 = h264::chroma_qp(qp1, a.chroma_qp_offset);
  const int qp = half ? qp1 : qp0, qpc = half ? qpc1 : qpc0;
  int mf[3], mfc[3], dv[3], dvc[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    mf[c] = half ? h264::kQuantMF[qp1 % 6][c] : h264::kQuantMF[qp0 % 6][c];
    mfc[c] = half ? h264::kQuantMF[qpc1 % 6][c] : h264::kQuantMF[qpc0 % 6][c];
    dv[c] = half ? h264::kDequantV[qp1 % 6][c] : h264::kDequantV[qp0 % 6][c];
    dvc[c] = half ? h264::kDequantV[qpc1 % 6][c] : h264::kDequantV[qpc0 % 6][c];
  }

  __shared__ int s_score[2][24];
  __shared__ int s_cdc[2][2][4];
  __shared__ int s_clev[2][2][4];
  __shared__ int s_flags[2][2];  // [half][0] luma 8x8 keep mask, [1] chroma AC keep mask (bit per comp)
  // 8x8 transform path (a.t8): residual copies for the sa8d Hadamard and the transform,
  // the 8x8 levels in scan order, per-block cost terms
  __shared__ int s_h8[2][4][64];
  __shared__ int s_d8[2][4][64];
  __shared__ int16_t s_l8[2][4][64];
  __shared__ int s_cost[2][2][16];   // [half][0: satd per 4x4 lane, 1: sa8d partial per (b8, k)]
  __shared__ int s_t8[2][3];         // [half][0] use 8x8, [1] keep mask of the 8x8 blocks, [2] 8x8 tried
  __shared__ int s_nz8[2][4][4];     // trellis: [half][b8][chunk] the dead-zone levels are non-zero
  __shared__ uint32_t s_px[2][2][16][4];  // a.t8: [half][source / prediction][row][dword] luma samples

  const int mvx = a.bmode ? 0 : a.mv[o * 2], mvy = a.bmode ? 0 : a.mv[o * 2 + 1];
  const bool go_intra = a.intra_cost[o] < a.me_cost[o];
  MbHeader* h = a.hdr + o;
  int16_t* coef = a.coef + o * h264::kCoefPerMb;
  if (live && go_intra && hl == 0) {
    // the wavefront kernel encodes this MB closed-loop; leave a consistent placeholder
    a.intra_flag[o] = 1;
    atomicAdd(a.intra_count + slot, 1);
    h->kind = h264::MBK_I16x16;
  }
  const bool work = live && !go_intra;

  int lv[16];     // raster levels of this lane's block
  int res[16];    // residual / reconstruction scratch
  uint32_t prw[4];  // prediction rows (4 bytes each)
  const int comp = (hl - 16) >> 2, cb = (hl - 16) & 3;
  const int X0 = mx * 16, Y0 = my * 16;
  const int lbx = (((hl >> 2) & 1) * 2 + (hl & 1)) * 4, lby = (((hl >> 3) & 1) * 2 + ((hl >> 1) & 1)) * 4;
  const int cbx = (cb & 1) * 4, cby = (cb >> 1) * 4;

  if (work && hl < 16) {
    // ---- luma block: residual against the ME prediction, forward transform, quantisation
    const uint8_t* srcy = a.src_y + slot * g.ysize() + static_cast<size_t>(Y0 + lby) * W + X0 + lbx;
    const uint8_t* pred = a.pred_y + o * 256 + lby * 16 + lbx;
    uint32_t sw[4];
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      prw[y] = *reinterpret_cast<const uint32_t*>(pred + y * 16);
      sw[y] = *reinterpret_cast<const uint32_t*>(srcy + static_cast<size_t>(y) * W);
    }
    if (a.wp && !a.bmode && !(a.mref && a.mref[o])) {  // weighted RefPicList0[0] prediction
      const int* wt = a.wp + slot * 8;
      const int w = wt[0], wo = wt[1], d = wt[2];
      if (w != (1 << d) || wo != 0) {
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          int v4[4];
#pragma unroll
          for (int x = 0; x < 4; ++x) v4[x] = wp_sample(static_cast<int>(__builtin_amdgcn_ubfe(prw[y], 8 * x, 8)), w, wo, d);
          prw[y] = pack4_u8(v4);
        }
      }
    }
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int x = 0; x < 4; ++x)
        res[y * 4 + x] = static_cast<int>(__builtin_amdgcn_ubfe(sw[y], 8 * x, 8)) -
                         static_cast<int>(__builtin_amdgcn_ubfe(prw[y], 8 * x, 8));
    // 4x4 transform, quantisation and decimation score (always: most MBs end here)
    h264::forward_core4x4(res);
    {
      const int qbits = 15 + qp / 6;
      if (a.trellis) {
        trellis_lite4x4(res, lv, mf, qbits, trellis_lambda4(a.trellis_lambda, qp));
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) lv[r] = h264::quant_coef(res[r], mf[h264::kPosClass[r]], qbits, 11);
      }
      int scan[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) scan[i] = lv[h264::kZigzag4x4[i]];
      s_score[half][hl] = decimate_score(scan, 0);
    }
    if (a.t8) {
      // stage this block's source and prediction rows for the 8x8 trial (s_px[half][0 / 1])
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        s_px[half][0][lby + y][lbx >> 2] = sw[y];
        s_px[half][1][lby + y][lbx >> 2] = prw[y];
      }
    }
  } else if (work && hl < 24) {
    // ---- chroma block: eighth-sample MC (clause 8.4.2.2.2) + residual + forward + AC quant
    const uint8_t* srcc = (comp == 0 ? a.src_u : a.src_v) + slot * g.csize();
    const int px0 = mx * 8 + cbx, py0 = my * 8 + cby;
    int pv[4][4];
    if (!a.bmode) {
      // the 4x4 chroma block cb covers luma quadrant cb (its partition's vector)
      const int cmx = a.mv8 ? a.mv8[o * 8 + cb * 2] : mvx, cmy = a.mv8 ? a.mv8[o * 8 + cb * 2 + 1] : mvy;
      const int r = a.mref ? a.mref[o] : 0;
      chroma_mc4x4((comp == 0 ? a.refs_u[r] : a.refs_v[r]) + route_index(a.rt, a.nbuf, slot, RO_L0 + r) * g.csize(), cw,
                   CH, px0, py0, cmx, cmy, pv);
      if (a.wp && r == 0) {
        const int* wt = a.wp + slot * 8;
        const int w = wt[3 + 2 * comp], wo = wt[4 + 2 * comp], d = wt[7];
        if (w != (1 << d) || wo != 0) {
#pragma unroll
          for (int y = 0; y < 4; ++y)
#pragma unroll
            for (int x = 0; x < 4; ++x) pv[y][x] = wp_sample(pv[y][x], w, wo, d);
        }
      }
    } else {
      // the 4x4 chroma block cb covers luma quadrant cb: its lists and vectors
      const int r0 = h->ref[0][cb];
      const bool u0 = r0 >= 0, u1 = h->ref[1][cb] >= 0;
      const int w1 = a.rt ? a.rt[slot].w1[r0 & 3] : a.w1[r0 & 3];
      int p1[4][4];
      if (u0) chroma_mc4x4((comp == 0 ? a.refs_u[r0 & 3] : a.refs_v[r0 & 3]) +
                               route_index(a.rt, a.nbuf, slot, RO_L0 + (r0 & 3)) * g.csize(), cw, CH, px0, py0,
                           h->mv[0][cb][0], h->mv[0][cb][1], pv);
      if (u1) chroma_mc4x4((comp == 0 ? a.ref1_u : a.ref1_v) + route_index(a.rt, a.nbuf, slot, RO_L1) * g.csize(), cw,
                           CH, px0, py0,
                           h->mv[1][cb][0], h->mv[1][cb][1], p1);
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int x = 0; x < 4; ++x)  // implicit weights (a.w1 = 32: the plain average)
          pv[y][x] = u0 ? (u1 ? h264::clip1((pv[y][x] * (64 - w1) + p1[y][x] * w1 + 32) >> 6) : pv[y][x]) : p1[y][x];
    }
    uint32_t sw[4];
#pragma unroll
    for (int y = 0; y < 4; ++y) sw[y] = *reinterpret_cast<const uint32_t*>(srcc + static_cast<size_t>(py0 + y) * cw + px0);
#pragma unroll
    for (int y = 0; y < 4; ++y) {
#pragma unroll
      for (int x = 0; x < 4; ++x) res[y * 4 + x] = static_cast<int>(__builtin_amdgcn_ubfe(sw[y], 8 * x, 8)) - pv[y][x];
      prw[y] = pack4_u8(pv[y]);
    }
    h264::forward_core4x4(res);
    s_cdc[half][comp][cb] = res[0];
    const int qbits = 15 + qpc / 6;
    if (a.trellis >= 2) {  // chroma AC by the same rate-distortion choice, at the chroma QP's lambda
      trellis_lite4x4(res, lv, mfc, qbits, trellis_lambda4(a.trellis_lambda, qpc), 1);
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        lv[r] = r == 0 ? 0 : h264::quant_coef(res[r], mfc[h264::kPosClass[r]], qbits, 11);
    }
    int scan[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) scan[i] = lv[h264::kZigzag4x4[i]];
    s_score[half][hl] = decimate_score(scan, 1);
  }
  if (a.t8) {
    // High profile: an MB whose 4x4 luma levels survive decimation also tries the 8x8
    // transform -- sa8d of the residual < its satd picks it (x264 analyse), and only then is it
    // transformed and quantised; MBs without luma residual keep the 4x4 flag-free coding
    // (transform_size_8x8_flag is not even coded for them).  The whole wave meets here (the
    // sa8d runs on the matrix cores for both MBs at once).
    wave_sync();
    if (hl == 0) {
      int total = 0, any = 0;
#pragma unroll
      for (int b8 = 0; b8 < 4; ++b8) {
        const int sc = s_score[half][b8 * 4] + s_score[half][b8 * 4 + 1] + s_score[half][b8 * 4 + 2] +
                       s_score[half][b8 * 4 + 3];
        any |= sc >= 4;
        total += sc;
      }
      s_t8[half][2] = work && any && total >= 6;
      s_t8[half][0] = 0;
      s_t8[half][1] = 0;
    }
    wave_sync();
    const bool try0 = s_t8[0][2], try1 = s_t8[1][2];
    if (try0 || try1) {  // wave-uniform
      const bool mine = half ? try1 : try0;
      if (mine && hl < 16) {
        // this 4x4 block's residual: the 8x8 transform input (s_d8) and its 4x4 satd
        const int b8 = (lby >> 3) * 2 + (lbx >> 3), ox = lbx & 4, oy = lby & 4;
        int r2[16];
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const uint32_t sv = s_px[half][0][lby + y][lbx >> 2], pv = s_px[half][1][lby + y][lbx >> 2];
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            r2[y * 4 + x] = static_cast<int>(__builtin_amdgcn_ubfe(sv, 8 * x, 8)) -
                            static_cast<int>(__builtin_amdgcn_ubfe(pv, 8 * x, 8));
            s_d8[half][b8][(oy + y) * 8 + ox + x] = r2[y * 4 + x];
          }
        }
        s_cost[half][0][hl] = h264::satd4x4(r2);
      }
      // sa8d of the 8 8x8 blocks (columns 4 * half + b8; columns 8..15 idle) on the int8 matrix
      // cores: vec(H8 X H8^T) = H64 vec(X) with H64 = H8 (x) H8 (Sylvester: (-1)^popcount(i & k)),
      // X = S - P split as (S - 128) - (P - 128) so both operands fit int8 (exact)
      const int col = lane & 15, grp = lane >> 4;
      mfma_i32x4 sop = {0, 0, 0, 0}, pop = {0, 0, 0, 0};
      if (col < 8) {
        const int ch = col >> 2, b8 = col & 3, r0 = (b8 >> 1) * 8 + 2 * grp, c0 = (b8 & 1) * 2;
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          mfma_i32x4& op = sp ? pop : sop;
          op[0] = static_cast<int>(s_px[ch][sp][r0][c0] ^ 0x80808080u);
          op[1] = static_cast<int>(s_px[ch][sp][r0][c0 + 1] ^ 0x80808080u);
          op[2] = static_cast<int>(s_px[ch][sp][r0 + 1][c0] ^ 0x80808080u);
          op[3] = static_cast<int>(s_px[ch][sp][r0 + 1][c0 + 1] ^ 0x80808080u);
        }
      }
      // this lane's A rows: H64[16 t + col][16 grp + j] = (-1)^popcount(t & grp) H16[col][j]
      mfma_i32x4 hp, hn;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t w = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) w |= ((__builtin_popcount(col & (4 * q + b)) & 1) ? 0xFFu : 0x01u) << (8 * b);
        hp[q] = static_cast<int>(w);
        hn[q] = static_cast<int>(w ^ 0xFEFEFEFEu);  // 0x01 <-> 0xFF: the negation
      }
      int sa = 0;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bool neg = __builtin_popcount(t & grp) & 1;
        mfma_i32x4 d = __builtin_amdgcn_mfma_i32_16x16x64_i8(neg ? hn : hp, sop, mfma_i32x4{0, 0, 0, 0}, 0, 0, 0);
        d = __builtin_amdgcn_mfma_i32_16x16x64_i8(neg ? hp : hn, pop, d, 0, 0, 0);
        sa += abs(d[0]) + abs(d[1]) + abs(d[2]) + abs(d[3]);
      }
      sa = sum_row_groups(sa);  // |coefficients| of column col, summed over its 4 lane groups
      int sa8d = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) sa8d += (__shfl(sa, 4 * half + b, 64) + 2) >> 2;
      wave_sync();
      if (mine && hl == 0) {
        int satd = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) satd += s_cost[half][0][i];
        s_t8[half][0] = sa8d < satd;
      }
      wave_sync();
      if (work && hl < 16 && s_t8[half][0]) {
      // ---- 8x8 transform: forward passes, quantisation of scan positions 16k .. 16k + 15
      // with this chunk's share of x264's decimate_score64 (zero runs priced 3 / 2 / 1 / 0;
      // 9 once any |level| > 1): runs inside the chunk here, the run into its first
      // non-zero level from the previous chunks' last
      const int tb = hl >> 2, k = hl & 3;
      int* dd = s_d8[half][tb];
      dct8_pass(dd + (2 * k) * 8, 1);
      dct8_pass(dd + (2 * k + 1) * 8, 1);
      wave_sync();
      dct8_pass(dd + 2 * k, 8);
      dct8_pass(dd + 2 * k + 1, 8);
      wave_sync();
      const int qbits8 = 16 + qp / 6;
      const int m = qp % 6;
      int lastnz = -1, firstnz = -1, inner = 0;
      bool big = false;
      int q8[16];
      if (a.trellis >= 2) {
        // x264 --trellis on the 8x8 blocks too: the dead-zone levels say which later chunks
        // keep a non-zero level, then each chunk runs the greedy choice back to front
        float z[16];
        bool nzc = false;
        const float inv = exp2f(-static_cast<float>(qbits8));
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int pos = kZz8[k * 16 + i];
          const int mf8 = kQuant8MF[m][pos8(pos & 7, pos >> 3)];
          z[i] = static_cast<float>(dd[pos]) * static_cast<float>(mf8) * inv;
          nzc |= h264::quant_coef(dd[pos], mf8, qbits8, 11) != 0;
        }
        s_nz8[half][tb][k] = nzc;
        wave_sync();
        bool later = false;
#pragma unroll
        for (int j = 1; j < 4; ++j) later |= (j > k) && s_nz8[half][tb][j];
        trellis_lite8_chunk(z, q8, a.trellis_lambda * 0.136f, later);
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int pos = kZz8[k * 16 + i];
          q8[i] = h264::quant_coef(dd[pos], kQuant8MF[m][pos8(pos & 7, pos >> 3)], qbits8, 11);
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int idx = k * 16 + i;
        const int v = q8[i];
        s_l8[half][tb][idx] = static_cast<int16_t>(v);
        const bool nzv = v != 0;
        big |= v > 1 || v < -1;
        const int run = idx - lastnz - 1;
        inner += (nzv && firstnz >= 0) ? (run <= 3 ? 3 : (run <= 11 ? 2 : (run <= 23 ? 1 : 0))) : 0;
        firstnz = (nzv && firstnz < 0) ? idx : firstnz;
        lastnz = nzv ? idx : lastnz;
      }
      int* stat = &s_h8[half][tb][16 * k];  // the Hadamard copy is spent: reuse it
      wave_sync();
      stat[0] = lastnz;
      wave_sync();
      int prev = -1;
#pragma unroll
      for (int j = 0; j < 3; ++j) prev = (j < k) ? max(prev, s_h8[half][tb][16 * j]) : prev;
      const int run0 = firstnz - prev - 1;
      const int sc = inner + (firstnz >= 0 ? (run0 <= 3 ? 3 : (run0 <= 11 ? 2 : (run0 <= 23 ? 1 : 0))) : 0);
      wave_sync();
      stat[1] = sc;
      stat[2] = big;
      wave_sync();
      if (hl == 0) {
        int keep = 0, total = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int* st0 = s_h8[half][b];
          const int scb = (st0[2] | st0[18] | st0[34] | st0[50]) ? 9 : (st0[1] + st0[17] + st0[33] + st0[49]);
          if (scb >= 4) keep |= 1 << b;
          total += scb;
        }
        if (total < 6) keep = 0;
        s_t8[half][1] = keep;
      }
      }
    }
  }
  wave_sync();
  if (work && (hl == 16 || hl == 20)) {
    // chroma DC: 2x2 Hadamard + quantisation with qbits+1
    const int c = hl == 16 ? 0 : 1;
    const int d0 = s_cdc[half][c][0], d1 = s_cdc[half][c][1], d2 = s_cdc[half][c][2], d3 = s_cdc[half][c][3];
    const int f[4] = {d0 + d1 + d2 + d3, d0 - d1 + d2 - d3, d0 + d1 - d2 - d3, d0 - d1 - d2 + d3};
    const int qbits = 15 + qpc / 6;
#pragma unroll
    for (int i = 0; i < 4; ++i) s_clev[half][c][i] = h264::quant_coef(f[i], mfc[0], qbits + 1, 11);
  }
  if (work && hl == 0) {
    int keep = 0, total = 0;
#pragma unroll
    for (int b8 = 0; b8 < 4; ++b8) {
      const int sc = s_score[half][b8 * 4] + s_score[half][b8 * 4 + 1] + s_score[half][b8 * 4 + 2] +
                     s_score[half][b8 * 4 + 3];
      if (sc >= 4) keep |= 1 << b8;
      total += sc;
    }
    if (total < 6) keep = 0;
    int ckeep = 0;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int sc = s_score[half][16 + 4 * c] + s_score[half][17 + 4 * c] + s_score[half][18 + 4 * c] +
                     s_score[half][19 + 4 * c];
      if (sc >= 7) ckeep |= 1 << c;
    }
    s_flags[half][0] = keep;
    s_flags[half][1] = ckeep;
  }
  wave_sync();
  if (!work) return;
  auto store_levels = [](int16_t* dst, const int* v) {  // 16 levels, 16-byte aligned
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = (static_cast<uint32_t>(v[2 * i]) & 0xFFFFu) | (static_cast<uint32_t>(v[2 * i + 1]) << 16);
    reinterpret_cast<uint4*>(dst)[0] = make_uint4(w[0], w[1], w[2], w[3]);
    reinterpret_cast<uint4*>(dst)[1] = make_uint4(w[4], w[5], w[6], w[7]);
  };
  const bool use8 = a.t8 && s_t8[half][0];
  if (hl < 16 && use8) {
    // ---- 8x8 transform: levels in 8x8 scan order (chunk k of block b8), dequantise into
    // the transform buffer, inverse 8x8 (lanes on rows / columns 2k, 2k + 1), then every 4x4
    // lane adds its part of the residual to the prediction
    const int b8 = hl >> 2, k = hl & 3;
    const bool keep = (s_t8[half][1] >> b8) & 1;
    int sv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) sv[i] = keep ? s_l8[half][b8][k * 16 + i] : 0;
    store_levels(coef + h264::COEF_LUMA + b8 * 64 + k * 16, sv);
    int* dd = s_d8[half][b8];
    const int m = qp % 6, q6 = qp / 6;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int pos = kZz8[k * 16 + i];
      const int ls = 16 * kNorm8[m][pos8(pos & 7, pos >> 3)];
      const int c = sv[i];
      dd[pos] = q6 >= 6 ? (c * ls) << (q6 - 6) : (c * ls + (1 << (5 - q6))) >> (6 - q6);
    }
    wave_sync();
    idct8_pass(dd + (2 * k) * 8, 1);
    idct8_pass(dd + (2 * k + 1) * 8, 1);
    wave_sync();
    idct8_pass(dd + 2 * k, 8);
    idct8_pass(dd + 2 * k + 1, 8);
    wave_sync();
    const int lb8 = (lby >> 3) * 2 + (lbx >> 3), ox = lbx & 4, oy = lby & 4;
    const bool any8 = (s_t8[half][1] >> lb8) & 1;
    uint8_t* recy = a.rec_y + rcur * g.ysize() + static_cast<size_t>(Y0 + lby) * W + X0 + lbx;
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      int v4[4];
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const int r8 = any8 ? (s_d8[half][lb8][(oy + y) * 8 + ox + x] + 32) >> 6 : 0;
        v4[x] = h264::clip1(static_cast<int>(__builtin_amdgcn_ubfe(prw[y], 8 * x, 8)) + r8);
      }
      *reinterpret_cast<uint32_t*>(recy + static_cast<size_t>(y) * W) = pack4_u8(v4);
    }
    a.nz[o * 16 + (lbx >> 2) + lby] = any8;
  } else if (hl < 16) {
    const bool keep = (s_flags[half][0] >> (hl >> 2)) & 1;
    int sv[16];
    bool any = false;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      sv[i] = keep ? lv[h264::kZigzag4x4[i]] : 0;
      any |= sv[i] != 0;
    }
    store_levels(coef + h264::COEF_LUMA + hl * 16, sv);
#pragma unroll
    for (int r = 0; r < 16; ++r) res[r] = keep ? (lv[r] * dv[h264::kPosClass[r]]) << (qp / 6) : 0;
    if (any) h264::inverse_core4x4(res);
    uint8_t* recy = a.rec_y + rcur * g.ysize() + static_cast<size_t>(Y0 + lby) * W + X0 + lbx;
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      int v4[4];
#pragma unroll
      for (int x = 0; x < 4; ++x)
        v4[x] = h264::clip1(static_cast<int>(__builtin_amdgcn_ubfe(prw[y], 8 * x, 8)) + (any ? res[y * 4 + x] : 0));
      *reinterpret_cast<uint32_t*>(recy + static_cast<size_t>(y) * W) = pack4_u8(v4);
    }
    a.nz[o * 16 + (lbx >> 2) + lby] = any;
  } else if (hl < 24) {
    const bool keep_ac = (s_flags[half][1] >> comp) & 1;
    int sv[16];
    bool any_ac = false;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      sv[i] = (keep_ac && i > 0) ? lv[h264::kZigzag4x4[i]] : 0;
      any_ac |= sv[i] != 0;
    }
    store_levels(coef + h264::COEF_CHROMA_AC + (comp * 4 + cb) * 16, sv);
    const int* cl = s_clev[half][comp];
    // this block's row of the 2x2 Hadamard (signs by cb: no dynamically indexed array)
    const int c0 = cl[0], c1 = cl[1], c2 = cl[2], c3 = cl[3];
    const int fcb = cb == 0 ? c0 + c1 + c2 + c3 : (cb == 1 ? c0 - c1 + c2 - c3 : (cb == 2 ? c0 + c1 - c2 - c3 : c0 - c1 - c2 + c3));
    const int ls = 16 * dvc[0];
#pragma unroll
    for (int r = 0; r < 16; ++r) res[r] = (keep_ac && r > 0) ? (lv[r] * dvc[h264::kPosClass[r]]) << (qpc / 6) : 0;
    res[0] = ((fcb * ls) << (qpc / 6)) >> 5;
    const bool any = any_ac || c0 || c1 || c2 || c3;
    if (any) h264::inverse_core4x4(res);
    uint8_t* recc = (comp == 0 ? a.rec_u : a.rec_v) + rcur * g.csize() + static_cast<size_t>(my * 8 + cby) * cw + mx * 8 + cbx;
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      int v4[4];
#pragma unroll
      for (int x = 0; x < 4; ++x)
        v4[x] = h264::clip1(static_cast<int>(__builtin_amdgcn_ubfe(prw[y], 8 * x, 8)) + (any ? res[y * 4 + x] : 0));
      *reinterpret_cast<uint32_t*>(recc + static_cast<size_t>(y) * cw) = pack4_u8(v4);
    }
  } else if (hl == 24) {
    // chroma DC levels (Cb then Cr, 8 x int16 = 16 bytes at COEF_CHROMA_DC)
    const int* c0 = s_clev[half][0];
    const int* c1 = s_clev[half][1];
    auto p2 = [](int lo, int hi) { return (static_cast<uint32_t>(lo) & 0xFFFFu) | (static_cast<uint32_t>(hi) << 16); };
    *reinterpret_cast<uint4*>(coef + h264::COEF_CHROMA_DC) = make_uint4(p2(c0[0], c0[1]), p2(c0[2], c0[3]),
                                                                        p2(c1[0], c1[1]), p2(c1[2], c1[3]));
  } else if (hl == 25 || hl == 26) {
    // luma DC (unused for P16x16): zero
    reinterpret_cast<uint4*>(coef + h264::COEF_LUMA_DC)[hl - 25] = make_uint4(0, 0, 0, 0);
  } else if (hl == 27) {
    h->qp = static_cast<int8_t>(qp);
    h->i16_mode = 0;
    h->chroma_mode = 0;
    // transform_size_8x8_flag is only coded (and only matters) when luma levels exist
    h->flags = (use8 && s_t8[half][1]) ? h264::MBF_T8x8 : 0;
    a.intra_flag[o] = 0;
    if (a.bmode) return;  // kind / ref / mv are b_decide's
    const uint32_t mvw = (static_cast<uint32_t>(mvx) & 0xFFFFu) | (static_cast<uint32_t>(mvy) << 16);
    uint4 q4 = make_uint4(mvw, mvw, mvw, mvw);
    if (a.mv8) q4 = *reinterpret_cast<const uint4*>(a.mv8 + o * 8);
    // quadrant vectors -> the cheapest partition shape that carries them
    h->kind = (q4.x == q4.y && q4.z == q4.w) ? (q4.x == q4.z ? h264::MBK_P16x16 : h264::MBK_P16x8)
                                             : ((q4.x == q4.z && q4.y == q4.w) ? h264::MBK_P8x16 : h264::MBK_P8x8);
    uint4* mvp = reinterpret_cast<uint4*>(&h->mv[0][0][0]);  // 16-byte aligned
    mvp[0] = q4;
    const uint32_t r = a.mref ? static_cast<uint32_t>(a.mref[o]) * 0x01010101u : 0u;
    *reinterpret_cast<uint2*>(&h->ref[0][0]) = make_uint2(r, 0xFFFFFFFFu);  // L0 ref r, L1 unused
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
                                         const int8_t* aq, const uint8_t* ref1_u, const uint8_t* ref1_v, int bmode,
                                         int t8, const int16_t* mv8, void* stream, const int* w1, int nref,
                                         const uint8_t* const* xref_u, const uint8_t* const* xref_v,
                                         const int8_t* mref, const int* wp, int trellis, float trellis_lambda,
                                         const void* route, int nbuf) {
  InterArgs a;
  a.rt = static_cast<const SlotRoute*>(route);
  a.nbuf = nbuf;
  a.trellis = trellis;
  a.trellis_lambda = trellis_lambda;
  a.wp = bmode ? nullptr : wp;
  for (int r = 0; r < 4; ++r) {
    const int rr = r < nref ? r : 0;
    a.refs_u[r] = rr == 0 ? ref_u : xref_u[rr];
    a.refs_v[r] = rr == 0 ? ref_v : xref_v[rr];
  }
  a.mref = mref;
  for (int r = 0; r < 4; ++r) a.w1[r] = w1[r < nref ? r : 0];
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
  a.mv8 = bmode ? nullptr : mv8;
  a.me_cost = me_cost;
  a.intra_cost = intra_cost;
  a.qp = qp;
  a.chroma_qp_offset = chroma_qp_offset;
  a.hdr = static_cast<MbHeader*>(hdr);
  a.coef = coef;
  a.nz = nz;
  a.intra_flag = intra_flag;
  a.intra_count = intra_count;
  a.aq = aq;
  a.ref1_u = ref1_u;
  a.ref1_v = ref1_v;
  a.bmode = bmode;
  a.t8 = t8;
  hipLaunchKernelGGL(encode_inter_mb, dim3((wmb * hmb + 1) / 2, B), dim3(64), 0, static_cast<hipStream_t>(stream), a);
}
