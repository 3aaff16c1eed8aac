// Closed-loop intra coding in macroblock wavefront order.
//
// Intra prediction reads *reconstructed, unfiltered* neighbours, so MB (x, y)
// depends on (x-1, y), (x, y-1), (x+1, y-1) and (x-1, y-1).  One wave64 owns one
// MB row of one segment slot (rows are handed out by an atomic ticket, so row
// y-1 is always held by an already-running wave: deadlock-free under any
// dispatch order) and waits on the row above through an agent-scope
// release/acquire progress counter (MI355X guide §6 Guideline 16).
// Parallelism = B slots x hmb rows, e.g. 64 x 68 = 4352 waves at 1080p.
//
// For P frames only MBs flagged by encode_inter (intra_flag) are coded here; the
// others are already reconstructed and only advance the progress counter.
#include "kcommon.h"

namespace mivc {
namespace gpu {

using h264::MbHeader;

struct IntraArgs {
  Geom g;
  const uint8_t *src_y, *src_u, *src_v;
  uint8_t *rec_y, *rec_u, *rec_v;
  const int* qp;
  int chroma_qp_offset;
  MbHeader* hdr;
  int16_t* coef;
  uint8_t* nz;
  const uint8_t* intra_flag;  // null: every MB is intra (I frame)
  const int* intra_count;     // [B] (P frames)
  int* ticket;
  int* progress;              // [B * hmb]
  int* err;
  int use_i4x4;
};

constexpr int TS = 24;  // tile stride

struct IntraShared {
  uint8_t tile[17 * TS];   // reconstructed neighbourhood + current MB (luma)
  uint8_t t4[17 * TS];     // I4x4 trial reconstruction
  uint8_t src[256];
  uint8_t srcc[2][64];
  int16_t c4[16][16];      // I4x4 trial levels (scan order)
  int16_t c16[16][16];     // I16 AC levels (scan order)
  int lv16dc[16];          // I16 DC levels (raster of block positions)
  int dc16[16];            // forward DC coefficients (raster)
  uint8_t modes4[16];
  int cost4;
  int mode16, cost16;
  uint8_t ctop[2][9], cleft[2][8];  // chroma neighbours [comp][-1..7] (index 0 = top-left)
  int cmode;
  int ccost[4];
  int cdc[2][4];
  int clev[2][4];
  int cdeci[8];
  int left_modes[4];       // Intra4x4 modes of the left MB's right column (2 if not I4x4)
  int top_modes[4];        // bottom row of the top MB
  // right edge of the MB this wave coded last (kept in LDS: no global read-after-write
  // through the vector L1 on the next iteration)
  int saved_x;
  uint8_t saved_y[16];
  uint8_t saved_c[2][8];
  int saved_modes[4];
};

__device__ __forceinline__ void i4_neighbours(const uint8_t* t, int blk, int mbav, int* e, int* av_out) {
  int bx = h264::kBlkX[blk], by = h264::kBlkY[blk];
  bool left = bx > 0 || (mbav & h264::AV_LEFT), top = by > 0 || (mbav & h264::AV_TOP);
  int av = 0;
  if (left) av |= h264::AV_LEFT;
  if (top) av |= h264::AV_TOP;
  if (left && top) av |= h264::AV_TOPLEFT;
  bool tr;
  if (blk == 3 || blk == 7 || blk == 11 || blk == 13 || blk == 15) tr = false;
  else if (blk == 5) tr = (mbav & h264::AV_TOPRIGHT) != 0;
  else if (blk == 0 || blk == 1 || blk == 4) tr = (mbav & h264::AV_TOP) != 0;
  else tr = true;
  if (tr) av |= h264::AV_TOPRIGHT;
  const uint8_t* row = t + (by * 4) * TS + bx * 4;  // tile row above the block, col of x = -1
  e[0] = row[0];
#pragma unroll
  for (int i = 0; i < 4; ++i) e[1 + i] = row[1 + i];
#pragma unroll
  for (int i = 4; i < 8; ++i) e[1 + i] = tr ? row[1 + i] : row[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) e[9 + i] = t[(by * 4 + 1 + i) * TS + bx * 4];
  *av_out = av;
}

// forward transform + quantise (intra bias) + dequant + inverse of one 4x4 residual.
// res: raster residual in, raster reconstruction residual out.  scan_out: levels in scan order.
__device__ __forceinline__ bool tq_intra(int* res, int qp, int16_t* scan_out, bool skip_dc, int* dc_out) {
  h264::forward_core4x4(res);
  if (dc_out) *dc_out = res[0];
  int qbits = 15 + qp / 6;
  int lv[16];
  bool any = false;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    lv[r] = (skip_dc && r == 0) ? 0 : h264::quant_coef(res[r], h264::kQuantMF[qp % 6][h264::kPosClass[r]], qbits, 21);
    any |= lv[r] != 0;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) scan_out[i] = static_cast<int16_t>(lv[h264::kZigzag4x4[i]]);
#pragma unroll
  for (int r = 0; r < 16; ++r) res[r] = h264::dequant_coef(lv[r], qp, r);
  return any;
}

__device__ void encode_intra_mb(const IntraArgs& a, IntraShared& S, int slot, int mx, int my) {
  const Geom& g = a.g;
  const int lane = threadIdx.x;
  const int W = g.W, cw = g.cw();
  const int X0 = mx * 16, Y0 = my * 16;
  const size_t o = static_cast<size_t>(slot) * g.nmb() + my * g.wmb + mx;
  const int qp = a.qp[slot];
  const int qpc = h264::chroma_qp(qp, a.chroma_qp_offset);
  const int lambda = h264::kLambda[qp];
  const uint8_t* srcy = a.src_y + slot * g.ysize();
  uint8_t* recy = a.rec_y + slot * g.ysize();
  int mbav = 0;
  if (mx > 0) mbav |= h264::AV_LEFT;
  if (my > 0) mbav |= h264::AV_TOP;
  if (mx > 0 && my > 0) mbav |= h264::AV_TOPLEFT;
  if (my > 0 && mx < g.wmb - 1) mbav |= h264::AV_TOPRIGHT;

  // ---- stage source and reconstructed neighbourhood
  for (int i = lane; i < 256; i += 64) S.src[i] = srcy[static_cast<size_t>(Y0 + (i >> 4)) * W + X0 + (i & 15)];
  for (int i = lane; i < 128; i += 64) {
    int c = i >> 6, j = i & 63;
    const uint8_t* sc = (c == 0 ? a.src_u : a.src_v) + slot * g.csize();
    S.srcc[c][j] = sc[static_cast<size_t>(my * 8 + (j >> 3)) * cw + mx * 8 + (j & 7)];
  }
  if (lane < 21) {  // tile row 0: x = X0-1 .. X0+19
    int x = X0 - 1 + lane;
    bool ok = my > 0 && x >= 0 && x < W && (lane < 17 || (mbav & h264::AV_TOPRIGHT));
    S.tile[lane] = ok ? recy[static_cast<size_t>(Y0 - 1) * W + x] : 0;
  } else if (lane >= 32 && lane < 48) {  // tile col 0, rows 1..16
    int r = lane - 32;
    uint8_t v = 0;
    if (mx > 0) v = S.saved_x == mx - 1 ? S.saved_y[r] : recy[static_cast<size_t>(Y0 + r) * W + X0 - 1];
    S.tile[(r + 1) * TS] = v;
  }
  if (lane < 18) {  // chroma neighbours
    int c = lane / 9, i = lane % 9;  // i = 0 top-left, 1..8 top
    const uint8_t* rc = (c == 0 ? a.rec_u : a.rec_v) + slot * g.csize();
    int x = mx * 8 - 1 + i;
    bool ok = my > 0 && x >= 0;
    S.ctop[c][i] = ok ? rc[static_cast<size_t>(my * 8 - 1) * cw + x] : 0;
  } else if (lane >= 48 && lane < 64) {
    int c = (lane - 48) >> 3, i = (lane - 48) & 7;
    const uint8_t* rc = (c == 0 ? a.rec_u : a.rec_v) + slot * g.csize();
    uint8_t v = 0;
    if (mx > 0) v = S.saved_x == mx - 1 ? S.saved_c[c][i] : rc[static_cast<size_t>(my * 8 + i) * cw + mx * 8 - 1];
    S.cleft[c][i] = v;
  }
  if (lane < 4) {
    // most-probable-mode context: neighbours' Intra4x4 modes (2 when not I4x4)
    int lm = 2, tm = 2;
    if (mx > 0) {
      if (S.saved_x == mx - 1) {
        lm = S.saved_modes[lane];
      } else {
        const MbHeader& L = a.hdr[o - 1];
        lm = L.kind == h264::MBK_I4x4 ? L.i4_modes[h264::kRasterToBlk[3 + 4 * lane]] : 2;
      }
    }
    if (my > 0) {
      const MbHeader& T = a.hdr[o - g.wmb];
      tm = T.kind == h264::MBK_I4x4 ? T.i4_modes[h264::kRasterToBlk[lane + 12]] : 2;
    }
    S.left_modes[lane] = lm;
    S.top_modes[lane] = tm;
  }
  __syncthreads();

  // ---- Intra16x16 decision: lane = mode * 16 + block
  {
    int mode = lane >> 4, blk = lane & 15;
    bool ok = h264::i16_mode_ok(mode, mbav);
    int top[16], left[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      top[i] = S.tile[1 + i];
      left[i] = S.tile[(i + 1) * TS];
    }
    int tl = S.tile[0];
    int pa = 0, pb = 0, pc = 0, dc = 0;
    if (mode == 3 && ok) h264::i16_plane_params(top, left, tl, &pa, &pb, &pc);
    if (mode == 2) dc = h264::i16_dc(top, left, mbav);
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
        r[y * 4 + x] = static_cast<int>(S.src[Y * 16 + X]) - pv;
      }
    int s = h264::satd4x4(r);
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
    int key = ok ? ((s + lambda * 4) << 2) | mode : 0x7FFFFFFF;
    key = min(key, __shfl_xor(key, 16, 64));
    key = min(key, __shfl_xor(key, 32, 64));
    if (lane == 0) {
      S.mode16 = key & 3;
      S.cost16 = key >> 2;
    }
  }
  // ---- chroma mode decision: lane = mode * 8 + (comp*4 + block), lanes 0..31
  {
    int mode = (lane >> 3) & 3, cbk = lane & 7, comp = cbk >> 2, b = cbk & 3;
    bool ok = lane < 32 && h264::chroma_mode_ok(mode, mbav);
    int top[8], left[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      top[i] = S.ctop[comp][1 + i];
      left[i] = S.cleft[comp][i];
    }
    int tl = S.ctop[comp][0];
    int pa = 0, pb = 0, pc = 0;
    if (mode == 3 && ok) h264::chroma_plane_params(top, left, tl, &pa, &pb, &pc);
    int bx = (b & 1) * 4, by = (b >> 1) * 4;
    int r[16];
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        int X = bx + x, Y = by + y, pv;
        if (mode == 0) pv = h264::chroma_dc(top, left, mbav, b & 1, b >> 1);
        else if (mode == 1) pv = left[Y];
        else if (mode == 2) pv = top[X];
        else pv = h264::clip1((pa + pb * (X - 3) + pc * (Y - 3) + 16) >> 5);
        r[y * 4 + x] = static_cast<int>(S.srcc[comp][Y * 8 + X]) - pv;
      }
    int s = h264::satd4x4(r);
#pragma unroll
    for (int off = 4; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
    int key = ok ? (s << 2) | mode : 0x7FFFFFFF;
    key = min(key, __shfl_xor(key, 8, 64));
    key = min(key, __shfl_xor(key, 16, 64));
    if (lane == 0) S.cmode = key & 3;
  }
  __syncthreads();

  // ---- Intra4x4 trial (closed loop, sequential over the 16 blocks)
  bool use4 = false;
  if (a.use_i4x4) {
    for (int i = lane; i < 17 * TS; i += 64) S.t4[i] = S.tile[i];
    __syncthreads();
    int total = lambda * 8;
    for (int blk = 0; blk < 16; ++blk) {
      int e[13], av;
      i4_neighbours(S.t4, blk, mbav, e, &av);
      int bx = h264::kBlkX[blk], by = h264::kBlkY[blk];
      // predicted (most probable) mode
      int ma = bx > 0 ? S.modes4[h264::kRasterToBlk[(bx - 1) + 4 * by]] : S.left_modes[by];
      int mb_ = by > 0 ? S.modes4[h264::kRasterToBlk[bx + 4 * (by - 1)]] : S.top_modes[bx];
      bool dcpred = (bx == 0 && !(mbav & h264::AV_LEFT)) || (by == 0 && !(mbav & h264::AV_TOP));
      int pm = dcpred ? 2 : min(ma, mb_);
      int key = 0x7FFFFFFF;
      if (lane < 9 && h264::i4_mode_ok(lane, av)) {
        int r[16];
#pragma unroll
        for (int y = 0; y < 4; ++y)
#pragma unroll
          for (int x = 0; x < 4; ++x)
            r[y * 4 + x] = static_cast<int>(S.src[(by * 4 + y) * 16 + bx * 4 + x]) - h264::i4_pred_sample(lane, av, e, x, y);
        int cost = h264::satd4x4(r) + lambda * (lane == pm ? 1 : 4);
        key = (cost << 4) | lane;
      }
#pragma unroll
      for (int off = 8; off >= 1; off >>= 1) key = min(key, __shfl_xor(key, off, 64));
      int mode = key & 15;
      if (lane == 0) {
        total += key >> 4;
        S.modes4[blk] = static_cast<uint8_t>(mode);
        int pred[16], res[16];
#pragma unroll
        for (int y = 0; y < 4; ++y)
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            pred[y * 4 + x] = h264::i4_pred_sample(mode, av, e, x, y);
            res[y * 4 + x] = static_cast<int>(S.src[(by * 4 + y) * 16 + bx * 4 + x]) - pred[y * 4 + x];
          }
        tq_intra(res, qp, S.c4[blk], false, nullptr);
        h264::inverse_core4x4(res);
#pragma unroll
        for (int y = 0; y < 4; ++y)
#pragma unroll
          for (int x = 0; x < 4; ++x)
            S.t4[(by * 4 + 1 + y) * TS + bx * 4 + 1 + x] = static_cast<uint8_t>(h264::clip1(pred[y * 4 + x] + res[y * 4 + x]));
      }
      __syncthreads();
    }
    if (lane == 0) S.cost4 = total;
    __syncthreads();
    use4 = S.cost4 < S.cost16;
  }

  MbHeader* h = a.hdr + o;
  int16_t* coef = a.coef + o * h264::kCoefPerMb;
  if (use4) {
    // commit the I4x4 trial
    for (int i = lane; i < 256; i += 64) {
      int blk = i >> 4, k = i & 15;
      coef[h264::COEF_LUMA + i] = S.c4[blk][k];
    }
    if (lane < 16) coef[h264::COEF_LUMA_DC + lane] = 0;
    for (int i = lane; i < 256; i += 64) {
      int y = i >> 4, x = i & 15;
      S.tile[(y + 1) * TS + x + 1] = S.t4[(y + 1) * TS + x + 1];
    }
    if (lane < 16) {
      bool any = false;
      for (int k = 0; k < 16; ++k) any |= S.c4[lane][k] != 0;
      a.nz[o * 16 + h264::kBlkX[lane] + 4 * h264::kBlkY[lane]] = any;
      h->i4_modes[lane] = S.modes4[lane];
    }
  } else {
    // ---- Intra16x16 encode
    int mode = S.mode16;
    int top[16], left[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      top[i] = S.tile[1 + i];
      left[i] = S.tile[(i + 1) * TS];
    }
    int tl = S.tile[0];
    int pa = 0, pb = 0, pc = 0, dc = 0;
    if (mode == 3) h264::i16_plane_params(top, left, tl, &pa, &pb, &pc);
    if (mode == 2) dc = h264::i16_dc(top, left, mbav);
    int pred[16], res[16];
    int blk = lane & 15;
    int bx4 = h264::kBlkX[blk] * 4, by4 = h264::kBlkY[blk] * 4;
    if (lane < 16) {
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          int X = bx4 + x, Y = by4 + y, pv;
          if (mode == 0) pv = top[X];
          else if (mode == 1) pv = left[Y];
          else if (mode == 2) pv = dc;
          else pv = h264::clip1((pa + pb * (X - 7) + pc * (Y - 7) + 16) >> 5);
          pred[y * 4 + x] = pv;
          res[y * 4 + x] = static_cast<int>(S.src[Y * 16 + X]) - pv;
        }
      int dcc;
      tq_intra(res, qp, S.c16[blk], true, &dcc);
      S.dc16[h264::kBlkX[blk] + 4 * h264::kBlkY[blk]] = dcc;
    }
    __syncthreads();
    if (lane == 0) {
      int d[16];
      for (int i = 0; i < 16; ++i) d[i] = S.dc16[i];
      h264::hadamard4x4(d);
      int qbits = 15 + qp / 6;
      int lv[16];
      for (int r = 0; r < 16; ++r) lv[r] = h264::quant_coef(d[r] >> 1, h264::kQuantMF[qp % 6][0], qbits + 1, 21);
      for (int i = 0; i < 16; ++i) coef[h264::COEF_LUMA_DC + i] = static_cast<int16_t>(lv[h264::kZigzag4x4[i]]);
      h264::hadamard4x4(lv);
      int ls = 16 * h264::kDequantV[qp % 6][0];
      for (int r = 0; r < 16; ++r)
        S.lv16dc[r] = qp >= 36 ? (lv[r] * ls) << (qp / 6 - 6) : (lv[r] * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
    }
    __syncthreads();
    if (lane < 16) {
      res[0] = S.lv16dc[h264::kBlkX[blk] + 4 * h264::kBlkY[blk]];
      h264::inverse_core4x4(res);
      bool any = false;
      for (int k = 1; k < 16; ++k) any |= S.c16[blk][k] != 0;
      for (int k = 0; k < 16; ++k) coef[h264::COEF_LUMA + blk * 16 + k] = S.c16[blk][k];
      a.nz[o * 16 + h264::kBlkX[blk] + 4 * h264::kBlkY[blk]] = any;
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int x = 0; x < 4; ++x)
          S.tile[(by4 + y + 1) * TS + bx4 + x + 1] = static_cast<uint8_t>(h264::clip1(pred[y * 4 + x] + res[y * 4 + x]));
    }
  }
  __syncthreads();
  // ---- write luma reconstruction
  if (lane < 64) {
    int y = lane >> 2, x4 = (lane & 3) * 4;
    uint32_t word = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) word |= static_cast<uint32_t>(S.tile[(y + 1) * TS + x4 + k + 1]) << (8 * k);
    *reinterpret_cast<uint32_t*>(recy + static_cast<size_t>(Y0 + y) * W + X0 + x4) = word;
  }
  // ---- chroma encode (lanes 0..7: comp*4 + block)
  int cres[16], cpred[16], clv[16];
  int cx7[4] = {0, 0, 0, 0};
  const int cmode = S.cmode;
  if (lane < 8) {
    int comp = lane >> 2, b = lane & 3;
    int top[8], left[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      top[i] = S.ctop[comp][1 + i];
      left[i] = S.cleft[comp][i];
    }
    int tl = S.ctop[comp][0];
    int pa = 0, pb = 0, pc = 0;
    if (cmode == 3) h264::chroma_plane_params(top, left, tl, &pa, &pb, &pc);
    int bx = (b & 1) * 4, by = (b >> 1) * 4;
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        int X = bx + x, Y = by + y, pv;
        if (cmode == 0) pv = h264::chroma_dc(top, left, mbav, b & 1, b >> 1);
        else if (cmode == 1) pv = left[Y];
        else if (cmode == 2) pv = top[X];
        else pv = h264::clip1((pa + pb * (X - 3) + pc * (Y - 3) + 16) >> 5);
        cpred[y * 4 + x] = pv;
        cres[y * 4 + x] = static_cast<int>(S.srcc[comp][Y * 8 + X]) - pv;
      }
    h264::forward_core4x4(cres);
    S.cdc[comp][b] = cres[0];
    int qbits = 15 + qpc / 6;
#pragma unroll
    for (int r = 0; r < 16; ++r) clv[r] = r == 0 ? 0 : h264::quant_coef(cres[r], h264::kQuantMF[qpc % 6][h264::kPosClass[r]], qbits, 21);
  }
  __syncthreads();
  if (lane == 0 || lane == 4) {
    int c = lane >> 2;
    int d0 = S.cdc[c][0], d1 = S.cdc[c][1], d2 = S.cdc[c][2], d3 = S.cdc[c][3];
    int f[4] = {d0 + d1 + d2 + d3, d0 - d1 + d2 - d3, d0 + d1 - d2 - d3, d0 - d1 - d2 + d3};
    int qbits = 15 + qpc / 6;
    for (int i = 0; i < 4; ++i) S.clev[c][i] = h264::quant_coef(f[i], h264::kQuantMF[qpc % 6][0], qbits + 1, 21);
  }
  __syncthreads();
  if (lane < 8) {
    int comp = lane >> 2, b = lane & 3;
    int16_t* dst = coef + h264::COEF_CHROMA_AC + (comp * 4 + b) * 16;
    bool any_ac = false;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      int v = i == 0 ? 0 : clv[h264::kZigzag4x4[i]];
      dst[i] = static_cast<int16_t>(v);
      any_ac |= v != 0;
    }
    const int* cl = S.clev[comp];
    if (b == 0)
      for (int i = 0; i < 4; ++i) coef[h264::COEF_CHROMA_DC + comp * 4 + i] = static_cast<int16_t>(cl[i]);
    int f[4] = {cl[0] + cl[1] + cl[2] + cl[3], cl[0] - cl[1] + cl[2] - cl[3], cl[0] + cl[1] - cl[2] - cl[3],
                cl[0] - cl[1] - cl[2] + cl[3]};
    int ls = 16 * h264::kDequantV[qpc % 6][0];
#pragma unroll
    for (int r = 0; r < 16; ++r) cres[r] = r == 0 ? 0 : h264::dequant_coef(clv[r], qpc, r);
    cres[0] = ((f[b] * ls) << (qpc / 6)) >> 5;
    bool any = any_ac || cl[0] || cl[1] || cl[2] || cl[3];
    if (any) h264::inverse_core4x4(cres);
    uint8_t* recc = (comp == 0 ? a.rec_u : a.rec_v) + slot * g.csize();
    int bx = (b & 1) * 4, by = (b >> 1) * 4;
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      uint32_t word = 0;
#pragma unroll
      for (int x = 0; x < 4; ++x)
        word |= static_cast<uint32_t>(h264::clip1(cpred[y * 4 + x] + (any ? cres[y * 4 + x] : 0))) << (8 * x);
      *reinterpret_cast<uint32_t*>(recc + static_cast<size_t>(my * 8 + by + y) * cw + mx * 8 + bx) = word;
      cx7[y] = static_cast<int>(word >> 24);
    }
  }
  __syncthreads();
  if (lane < 16) {
    S.saved_y[lane] = S.tile[(lane + 1) * TS + 16];
    S.saved_modes[lane & 3] = use4 ? S.modes4[h264::kRasterToBlk[3 + 4 * (lane & 3)]] : 2;
  }
  if (lane < 8 && (lane & 1)) {  // right column chroma blocks (b = 1, 3) hold x = 7
    int comp = lane >> 2, b = lane & 3;
    for (int y = 0; y < 4; ++y) S.saved_c[comp][(b >> 1) * 4 + y] = static_cast<uint8_t>(cx7[y]);
  }
  if (lane == 0) S.saved_x = mx;
  if (lane == 63) {
    h->kind = use4 ? h264::MBK_I4x4 : h264::MBK_I16x16;
    h->qp = static_cast<int8_t>(qp);
    h->i16_mode = static_cast<uint8_t>(S.mode16);
    h->chroma_mode = static_cast<uint8_t>(cmode);
    h->flags = 0;
    for (int q = 0; q < 4; ++q) h->mv[q][0] = h->mv[q][1] = 0;
  }
  if (!use4 && lane >= 16 && lane < 32) h->i4_modes[lane - 16] = 2;
}

__global__ __launch_bounds__(64) void encode_intra_wavefront(IntraArgs a) {
  __shared__ IntraShared S;
  const Geom& g = a.g;
  const int t = draw_ticket(a.ticket);
  if (t >= g.B * g.hmb) return;
  const int slot = t / g.hmb, y = t % g.hmb;
  if (threadIdx.x == 0) S.saved_x = -2;
  __syncthreads();
  if (a.intra_flag && a.intra_count[slot] == 0) {
    publish_progress(a.progress + t, g.wmb);
    return;
  }
  for (int x = 0; x < g.wmb; ++x) {
    if (y > 0 && !wait_progress(a.progress + t - 1, min(x + 2, g.wmb), a.err)) {
      publish_progress(a.progress + t, g.wmb);  // unblock the rows below, then bail
      return;
    }
    const size_t o = static_cast<size_t>(slot) * g.nmb() + y * g.wmb + x;
    if (!a.intra_flag || a.intra_flag[o]) {
      encode_intra_mb(a, S, slot, x, y);
      publish_progress(a.progress + t, x + 1);
    } else if (x == g.wmb - 1 || (a.intra_flag[o + 1])) {
      // publish only when the next MB of this row is intra (or at row end): saves fences
      publish_progress(a.progress + t, x + 1);
    } else if (threadIdx.x == 0) {
      __hip_atomic_store(a.progress + t, x + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

extern "C" void mivc_launch_encode_intra(int B, int wmb, int hmb, const uint8_t* src_y, const uint8_t* src_u,
                                         const uint8_t* src_v, uint8_t* rec_y, uint8_t* rec_u, uint8_t* rec_v,
                                         const int* qp, int chroma_qp_offset, void* hdr, int16_t* coef, uint8_t* nz,
                                         const uint8_t* intra_flag, const int* intra_count, int* ticket, int* progress,
                                         int* err, int use_i4x4, void* stream) {
  IntraArgs a;
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.src_y = src_y;
  a.src_u = src_u;
  a.src_v = src_v;
  a.rec_y = rec_y;
  a.rec_u = rec_u;
  a.rec_v = rec_v;
  a.qp = qp;
  a.chroma_qp_offset = chroma_qp_offset;
  a.hdr = static_cast<MbHeader*>(hdr);
  a.coef = coef;
  a.nz = nz;
  a.intra_flag = intra_flag;
  a.intra_count = intra_count;
  a.ticket = ticket;
  a.progress = progress;
  a.err = err;
  a.use_i4x4 = use_i4x4;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipMemsetAsync(ticket, 0, sizeof(int), s);
  hipMemsetAsync(progress, 0, sizeof(int) * B * hmb, s);
  hipLaunchKernelGGL(encode_intra_wavefront, dim3(B * hmb), dim3(64), 0, s, a);
}
