// Closed-loop intra coding in macroblock wavefront order.
//
// Intra prediction reads *reconstructed, unfiltered* neighbours, so MB (x, y)
// depends on (x-1, y), (x, y-1), (x+1, y-1) and (x-1, y-1).  One workgroup of
// kWaves wave64s owns one frame (segment slot); wave w codes MB rows w, w+kWaves,
// ... and waits on the row above through an LDS progress counter (workgroup-scope
// release/acquire -- see kcommon.h).  Grid = B slots.
//
// For P frames only MBs flagged by encode_inter (intra_flag) are coded here; the
// others were reconstructed by encode_inter and only advance the row counter.
#include "kcommon.h"

namespace mivc {
namespace gpu {

using h264::MbHeader;

constexpr int kIntraWaves = 8;

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
  int* err;
  int use_i4x4;
};

constexpr int TS = 24;  // tile stride

struct IntraShared {
  uint8_t tile[17 * TS];   // reconstructed neighbourhood + current MB (luma); row 0 / col 0 = neighbours
  uint8_t t4[17 * TS];     // I4x4 trial reconstruction
  uint8_t src[256];
  uint8_t srcc[2][64];
  int16_t c4[16][16];      // I4x4 trial levels (scan order)
  int16_t c16[16][16];     // I16 AC levels (scan order)
  int lv16dc[16];          // I16 dequantised DC per block position (raster)
  int dc16[16];            // forward DC coefficients (raster)
  uint8_t top16[16], left16[16];
  uint8_t modes4[16];
  int cost4;
  int mode16, cost16;
  uint8_t ctop[2][9], cleft[2][8];  // chroma neighbours [comp][-1..7] (index 0 = top-left)
  int cmode;
  int cdc[2][4];
  int clev[2][4];
  int left_modes[4];       // Intra4x4 modes of the left MB's right column (2 if not I4x4)
  int top_modes[4];        // bottom row of the top MB
  // right edge of the MB this wave coded last (kept in LDS across iterations)
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

// 4x4 intra prediction sample at compile-time (x, y) for a runtime mode
__device__ __forceinline__ void i4_pred_block(int mode, int av, const int* e, int* pred) {
#pragma unroll
  for (int y = 0; y < 4; ++y)
#pragma unroll
    for (int x = 0; x < 4; ++x) pred[y * 4 + x] = h264::i4_pred_sample(mode, av, e, x, y);
}

// forward transform + quantise (intra bias) + dequant of one 4x4 residual (raster, in place).
__device__ __forceinline__ void tq_intra(int* res, int qp, int16_t* scan_out, bool skip_dc, int* dc_out) {
  h264::forward_core4x4(res);
  if (dc_out) *dc_out = res[0];
  int qbits = 15 + qp / 6;
  int lv[16];
#pragma unroll
  for (int r = 0; r < 16; ++r)
    lv[r] = (skip_dc && r == 0) ? 0 : h264::quant_coef(res[r], h264::kQuantMF[qp % 6][h264::kPosClass[r]], qbits, 21);
#pragma unroll
  for (int i = 0; i < 16; ++i) scan_out[i] = static_cast<int16_t>(lv[h264::kZigzag4x4[i]]);
#pragma unroll
  for (int r = 0; r < 16; ++r) res[r] = h264::dequant_coef(lv[r], qp, r);
}

__device__ __forceinline__ int i16_pred(int mode, const IntraShared& S, int dc, int pa, int pb, int pc, int X, int Y) {
  if (mode == 0) return S.top16[X];
  if (mode == 1) return S.left16[Y];
  if (mode == 2) return dc;
  return h264::clip1((pa + pb * (X - 7) + pc * (Y - 7) + 16) >> 5);
}

__device__ __forceinline__ int chroma_pred(int mode, const IntraShared& S, int comp, int mbav, int pa, int pb, int pc,
                                           int X, int Y) {
  if (mode == 0) return h264::chroma_dc(S.ctop[comp] + 1, S.cleft[comp], mbav, X >> 2, Y >> 2);
  if (mode == 1) return S.cleft[comp][Y];
  if (mode == 2) return S.ctop[comp][1 + X];
  return h264::clip1((pa + pb * (X - 3) + pc * (Y - 3) + 16) >> 5);
}

__device__ __forceinline__ void encode_intra_mb(const IntraArgs& a, IntraShared& S, int slot, int mx, int my) {
  const Geom& g = a.g;
  const int lane = lane_id();
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
  {
    // 64 lanes x 4 bytes = source MB
    int r = lane >> 2, c4 = (lane & 3) * 4;
    uint32_t w = *reinterpret_cast<const uint32_t*>(srcy + static_cast<size_t>(Y0 + r) * W + X0 + c4);
    *reinterpret_cast<uint32_t*>(S.src + r * 16 + c4) = w;
  }
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
  if (lane < 18) {  // chroma neighbours: top-left + top
    int c = lane / 9, i = lane % 9;
    const uint8_t* rc = (c == 0 ? a.rec_u : a.rec_v) + slot * g.csize();
    int x = mx * 8 - 1 + i;
    bool ok = my > 0 && x >= 0;
    S.ctop[c][i] = ok ? rc[static_cast<size_t>(my * 8 - 1) * cw + x] : 0;
  } else if (lane >= 48) {  // chroma left
    int c = (lane - 48) >> 3, i = (lane - 48) & 7;
    const uint8_t* rc = (c == 0 ? a.rec_u : a.rec_v) + slot * g.csize();
    uint8_t v = 0;
    if (mx > 0) v = S.saved_x == mx - 1 ? S.saved_c[c][i] : rc[static_cast<size_t>(my * 8 + i) * cw + mx * 8 - 1];
    S.cleft[c][i] = v;
  }
  if (lane >= 24 && lane < 28) {
    int i = lane - 24;  // most-probable-mode context
    int lm = 2, tm = 2;
    if (mx > 0) {
      if (S.saved_x == mx - 1) {
        lm = S.saved_modes[i];
      } else {
        const MbHeader& L = a.hdr[o - 1];
        lm = L.kind == h264::MBK_I4x4 ? L.i4_modes[h264::kRasterToBlk[3 + 4 * i]] : 2;
      }
    }
    if (my > 0) {
      const MbHeader& T = a.hdr[o - g.wmb];
      tm = T.kind == h264::MBK_I4x4 ? T.i4_modes[h264::kRasterToBlk[i + 12]] : 2;
    }
    S.left_modes[i] = lm;
    S.top_modes[i] = tm;
  }
  wave_sync();
  if (lane < 16) {
    S.top16[lane] = S.tile[1 + lane];
    S.left16[lane] = S.tile[(lane + 1) * TS];
  }
  wave_sync();

  // ---- Intra16x16 decision: lane = mode * 16 + block
  {
    int mode = lane >> 4, blk = lane & 15;
    bool ok = h264::i16_mode_ok(mode, mbav);
    int tl = S.tile[0];
    int pa = 0, pb = 0, pc = 0, dc = 0;
    if (mode == 3 && ok) h264::i16_plane_params(S.top16, S.left16, tl, &pa, &pb, &pc);
    if (mode == 2) dc = h264::i16_dc(S.top16, S.left16, mbav);
    int bx4 = (blk & 3) * 4, by4 = (blk >> 2) * 4;
    int r[16];
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int x = 0; x < 4; ++x)
        r[y * 4 + x] = static_cast<int>(S.src[(by4 + y) * 16 + bx4 + x]) - i16_pred(mode, S, dc, pa, pb, pc, bx4 + x, by4 + y);
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
    int tl = S.ctop[comp][0];
    int pa = 0, pb = 0, pc = 0;
    if (mode == 3 && ok) h264::chroma_plane_params(S.ctop[comp] + 1, S.cleft[comp], tl, &pa, &pb, &pc);
    int bx = (b & 1) * 4, by = (b >> 1) * 4;
    int r[16];
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int x = 0; x < 4; ++x)
        r[y * 4 + x] = static_cast<int>(S.srcc[comp][(by + y) * 8 + bx + x]) -
                       (ok ? chroma_pred(mode, S, comp, mbav, pa, pb, pc, bx + x, by + y) : 0);
    int s = h264::satd4x4(r);
#pragma unroll
    for (int off = 4; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
    int key = ok ? (s << 2) | mode : 0x7FFFFFFF;
    key = min(key, __shfl_xor(key, 8, 64));
    key = min(key, __shfl_xor(key, 16, 64));
    if (lane == 0) S.cmode = key & 3;
  }
  wave_sync();

  // ---- Intra4x4 trial (closed loop, sequential over the 16 blocks)
  bool use4 = false;
  if (a.use_i4x4) {
    for (int i = lane; i < 17 * TS; i += 64) S.t4[i] = S.tile[i];
    wave_sync();
    int total = lambda * 8;
    for (int blk = 0; blk < 16; ++blk) {
      int e[13], av;
      i4_neighbours(S.t4, blk, mbav, e, &av);
      int bx = h264::kBlkX[blk], by = h264::kBlkY[blk];
      int ma = bx > 0 ? S.modes4[h264::kRasterToBlk[(bx - 1) + 4 * by]] : S.left_modes[by];
      int mb_ = by > 0 ? S.modes4[h264::kRasterToBlk[bx + 4 * (by - 1)]] : S.top_modes[bx];
      bool dcpred = (bx == 0 && !(mbav & h264::AV_LEFT)) || (by == 0 && !(mbav & h264::AV_TOP));
      int pm = dcpred ? 2 : min(ma, mb_);
      int key = 0x7FFFFFFF;
      if (lane < 9 && h264::i4_mode_ok(lane, av)) {
        int pred[16], r[16];
        i4_pred_block(lane, av, e, pred);
#pragma unroll
        for (int y = 0; y < 4; ++y)
#pragma unroll
          for (int x = 0; x < 4; ++x) r[y * 4 + x] = static_cast<int>(S.src[(by * 4 + y) * 16 + bx * 4 + x]) - pred[y * 4 + x];
        int cost = h264::satd4x4(r) + lambda * (lane == pm ? 1 : 4);
        key = (cost << 4) | lane;
      }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) key = min(key, __shfl_xor(key, off, 64));  // wave-uniform
      int mode = key & 15;
      total += key >> 4;
      // TQ + recon of the chosen mode: 16 lanes, one sample each (transform via the block owner)
      if (lane == 0) {
        S.modes4[blk] = static_cast<uint8_t>(mode);
        int pred[16], res[16];
        i4_pred_block(mode, av, e, pred);
#pragma unroll
        for (int y = 0; y < 4; ++y)
#pragma unroll
          for (int x = 0; x < 4; ++x) res[y * 4 + x] = static_cast<int>(S.src[(by * 4 + y) * 16 + bx * 4 + x]) - pred[y * 4 + x];
        tq_intra(res, qp, S.c4[blk], false, nullptr);
        h264::inverse_core4x4(res);
#pragma unroll
        for (int y = 0; y < 4; ++y)
#pragma unroll
          for (int x = 0; x < 4; ++x)
            S.t4[(by * 4 + 1 + y) * TS + bx * 4 + 1 + x] = static_cast<uint8_t>(h264::clip1(pred[y * 4 + x] + res[y * 4 + x]));
      }
      wave_sync();
    }
    use4 = total < S.cost16;
  }

  MbHeader* h = a.hdr + o;
  int16_t* coef = a.coef + o * h264::kCoefPerMb;
  if (use4) {
    for (int i = lane; i < 256; i += 64) coef[h264::COEF_LUMA + i] = S.c4[i >> 4][i & 15];
    if (lane < 16) coef[h264::COEF_LUMA_DC + lane] = 0;
    for (int i = lane; i < 256; i += 64) {
      int y = i >> 4, x = i & 15;
      S.tile[(y + 1) * TS + x + 1] = S.t4[(y + 1) * TS + x + 1];
    }
    if (lane < 16) {
      bool any = false;
#pragma unroll
      for (int k = 0; k < 16; ++k) any |= S.c4[lane][k] != 0;
      a.nz[o * 16 + h264::kBlkX[lane] + 4 * h264::kBlkY[lane]] = any;
      h->i4_modes[lane] = S.modes4[lane];
    }
  } else {
    // ---- Intra16x16 encode
    const int mode = S.mode16;
    int tl = S.tile[0];
    int pa = 0, pb = 0, pc = 0, dc = 0;
    if (mode == 3) h264::i16_plane_params(S.top16, S.left16, tl, &pa, &pb, &pc);
    if (mode == 2) dc = h264::i16_dc(S.top16, S.left16, mbav);
    int pred[16], res[16];
    const int blk = lane & 15;
    const int bx4 = h264::kBlkX[blk] * 4, by4 = h264::kBlkY[blk] * 4;
    if (lane < 16) {
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          pred[y * 4 + x] = i16_pred(mode, S, dc, pa, pb, pc, bx4 + x, by4 + y);
          res[y * 4 + x] = static_cast<int>(S.src[(by4 + y) * 16 + bx4 + x]) - pred[y * 4 + x];
        }
      int dcc;
      tq_intra(res, qp, S.c16[blk], true, &dcc);
      S.dc16[h264::kBlkX[blk] + 4 * h264::kBlkY[blk]] = dcc;
    }
    wave_sync();
    if (lane == 0) {
      int d[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) d[i] = S.dc16[i];
      h264::hadamard4x4(d);
      int qbits = 15 + qp / 6;
      int lv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) lv[r] = h264::quant_coef(d[r] >> 1, h264::kQuantMF[qp % 6][0], qbits + 1, 21);
#pragma unroll
      for (int i = 0; i < 16; ++i) coef[h264::COEF_LUMA_DC + i] = static_cast<int16_t>(lv[h264::kZigzag4x4[i]]);
      h264::hadamard4x4(lv);
      int ls = 16 * h264::kDequantV[qp % 6][0];
#pragma unroll
      for (int r = 0; r < 16; ++r)
        S.lv16dc[r] = qp >= 36 ? (lv[r] * ls) << (qp / 6 - 6) : (lv[r] * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
    }
    wave_sync();
    if (lane < 16) {
      res[0] = S.lv16dc[h264::kBlkX[blk] + 4 * h264::kBlkY[blk]];
      h264::inverse_core4x4(res);
      bool any = false;
#pragma unroll
      for (int k = 1; k < 16; ++k) any |= S.c16[blk][k] != 0;
#pragma unroll
      for (int k = 0; k < 16; ++k) coef[h264::COEF_LUMA + blk * 16 + k] = S.c16[blk][k];
      a.nz[o * 16 + h264::kBlkX[blk] + 4 * h264::kBlkY[blk]] = any;
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int x = 0; x < 4; ++x)
          S.tile[(by4 + y + 1) * TS + bx4 + x + 1] = static_cast<uint8_t>(h264::clip1(pred[y * 4 + x] + res[y * 4 + x]));
    }
  }
  wave_sync();
  {  // ---- write luma reconstruction
    int y = lane >> 2, x4 = (lane & 3) * 4;
    uint32_t word = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) word |= static_cast<uint32_t>(S.tile[(y + 1) * TS + x4 + k + 1]) << (8 * k);
    *reinterpret_cast<uint32_t*>(recy + static_cast<size_t>(Y0 + y) * W + X0 + x4) = word;
  }
  // ---- chroma encode (lanes 0..7: comp*4 + block)
  int cres[16], cpred[16], clv[16];
  const int cmode = S.cmode;
  const int comp = (lane >> 2) & 1, cb = lane & 3;
  if (lane < 8) {
    int tl = S.ctop[comp][0];
    int pa = 0, pb = 0, pc = 0;
    if (cmode == 3) h264::chroma_plane_params(S.ctop[comp] + 1, S.cleft[comp], tl, &pa, &pb, &pc);
    int bx = (cb & 1) * 4, by = (cb >> 1) * 4;
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        cpred[y * 4 + x] = chroma_pred(cmode, S, comp, mbav, pa, pb, pc, bx + x, by + y);
        cres[y * 4 + x] = static_cast<int>(S.srcc[comp][(by + y) * 8 + bx + x]) - cpred[y * 4 + x];
      }
    h264::forward_core4x4(cres);
    S.cdc[comp][cb] = cres[0];
    int qbits = 15 + qpc / 6;
#pragma unroll
    for (int r = 0; r < 16; ++r)
      clv[r] = r == 0 ? 0 : h264::quant_coef(cres[r], h264::kQuantMF[qpc % 6][h264::kPosClass[r]], qbits, 21);
  }
  wave_sync();
  if (lane == 0 || lane == 4) {
    int c = lane >> 2;
    int d0 = S.cdc[c][0], d1 = S.cdc[c][1], d2 = S.cdc[c][2], d3 = S.cdc[c][3];
    int f0 = d0 + d1 + d2 + d3, f1 = d0 - d1 + d2 - d3, f2 = d0 + d1 - d2 - d3, f3 = d0 - d1 - d2 + d3;
    int qbits = 15 + qpc / 6, mf = h264::kQuantMF[qpc % 6][0];
    S.clev[c][0] = h264::quant_coef(f0, mf, qbits + 1, 21);
    S.clev[c][1] = h264::quant_coef(f1, mf, qbits + 1, 21);
    S.clev[c][2] = h264::quant_coef(f2, mf, qbits + 1, 21);
    S.clev[c][3] = h264::quant_coef(f3, mf, qbits + 1, 21);
  }
  wave_sync();
  int cx7[4] = {0, 0, 0, 0};
  if (lane < 8) {
    int16_t* dst = coef + h264::COEF_CHROMA_AC + (comp * 4 + cb) * 16;
    bool any_ac = false;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      int v = i == 0 ? 0 : clv[h264::kZigzag4x4[i]];
      dst[i] = static_cast<int16_t>(v);
      any_ac |= v != 0;
    }
    int c0 = S.clev[comp][0], c1 = S.clev[comp][1], c2 = S.clev[comp][2], c3 = S.clev[comp][3];
    if (cb == 0) {
      coef[h264::COEF_CHROMA_DC + comp * 4 + 0] = static_cast<int16_t>(c0);
      coef[h264::COEF_CHROMA_DC + comp * 4 + 1] = static_cast<int16_t>(c1);
      coef[h264::COEF_CHROMA_DC + comp * 4 + 2] = static_cast<int16_t>(c2);
      coef[h264::COEF_CHROMA_DC + comp * 4 + 3] = static_cast<int16_t>(c3);
    }
    int f;
    if (cb == 0) f = c0 + c1 + c2 + c3;
    else if (cb == 1) f = c0 - c1 + c2 - c3;
    else if (cb == 2) f = c0 + c1 - c2 - c3;
    else f = c0 - c1 - c2 + c3;
    int ls = 16 * h264::kDequantV[qpc % 6][0];
#pragma unroll
    for (int r = 0; r < 16; ++r) cres[r] = r == 0 ? 0 : h264::dequant_coef(clv[r], qpc, r);
    cres[0] = ((f * ls) << (qpc / 6)) >> 5;
    bool any = any_ac || c0 || c1 || c2 || c3;
    if (any) h264::inverse_core4x4(cres);
    uint8_t* recc = (comp == 0 ? a.rec_u : a.rec_v) + slot * g.csize();
    int bx = (cb & 1) * 4, by = (cb >> 1) * 4;
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
  // ---- keep this MB's right edge in LDS for the next iteration of this wave
  if (lane < 16) {
    S.saved_y[lane] = S.tile[(lane + 1) * TS + 16];
  }
  if (lane >= 16 && lane < 20) {
    int i = lane - 16;
    S.saved_modes[i] = use4 ? S.modes4[h264::kRasterToBlk[3 + 4 * i]] : 2;
  }
  if (lane < 8 && (cb & 1)) {  // right column chroma blocks (b = 1, 3) hold x = 7
#pragma unroll
    for (int y = 0; y < 4; ++y) S.saved_c[comp][(cb >> 1) * 4 + y] = static_cast<uint8_t>(cx7[y]);
  }
  if (lane == 63) {
    S.saved_x = mx;
    h->kind = use4 ? h264::MBK_I4x4 : h264::MBK_I16x16;
    h->qp = static_cast<int8_t>(qp);
    h->i16_mode = static_cast<uint8_t>(S.mode16);
    h->chroma_mode = static_cast<uint8_t>(cmode);
    h->flags = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) h->mv[q][0] = h->mv[q][1] = 0;
  }
  if (!use4 && lane >= 32 && lane < 48) h->i4_modes[lane - 32] = 2;
  wave_sync();
}

__global__ __launch_bounds__(64 * kIntraWaves) void encode_intra_wavefront(IntraArgs a) {
  __shared__ IntraShared SS[kIntraWaves];
  __shared__ int prog[kMaxRows];
  const Geom& g = a.g;
  const int slot = blockIdx.x;
  if (a.intra_flag && a.intra_count[slot] == 0) return;  // uniform per workgroup
  for (int i = threadIdx.x; i < g.hmb; i += blockDim.x) prog[i] = 0;
  const int w = wave_id();
  if (lane_id() == 0) SS[w].saved_x = -2;
  __syncthreads();
  IntraShared& S = SS[w];
  for (int y = w; y < g.hmb; y += kIntraWaves) {
    for (int x = 0; x < g.wmb; ++x) {
      const size_t o = static_cast<size_t>(slot) * g.nmb() + y * g.wmb + x;
      if (!a.intra_flag || a.intra_flag[o]) {
        if (y > 0) row_wait(prog, y - 1, min(x + 2, g.wmb), a.err);
        encode_intra_mb(a, S, slot, x, y);
      }
      row_publish(prog, y, x + 1);
    }
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

extern "C" void mivc_launch_encode_intra(int B, int wmb, int hmb, const uint8_t* src_y, const uint8_t* src_u,
                                         const uint8_t* src_v, uint8_t* rec_y, uint8_t* rec_u, uint8_t* rec_v,
                                         const int* qp, int chroma_qp_offset, void* hdr, int16_t* coef, uint8_t* nz,
                                         const uint8_t* intra_flag, const int* intra_count, int* err, int use_i4x4,
                                         void* stream) {
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
  a.err = err;
  a.use_i4x4 = use_i4x4;
  hipLaunchKernelGGL(encode_intra_wavefront, dim3(B), dim3(64 * kIntraWaves), 0, static_cast<hipStream_t>(stream), a);
}
