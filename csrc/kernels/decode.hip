// H.264 picture reconstruction on gfx950 from entropy-decoded records (SURVEY.md
// K-C1: the decode half of the transcode path, BASELINE config 3).
//
// The host parses CAVLC (csrc/host/h264_decoder.cc, parse-only mode) into the same
// per-MB decision records the encoder produces (MbHeader) plus the quantised levels,
// packed: only non-zero 4x4 blocks are stored, 16 levels each, located through a
// per-MB bit mask (bits 0-15 luma blkIdx, 16 Intra16x16 DC, 17 chroma DC Cb|Cr,
// 18-25 chroma AC comp*4+b) and the MB's first block index.  Reconstruction is then
// the encoder's own closed loop without the decisions:
//
//  * decode_inter_mb: every inter / P_Skip MB of a P picture in parallel (grid =
//    MBs x slots, one wave64 per MB): quarter-sample luma MC per 8x8 quadrant from an
//    LDS window of the reference, eighth-sample chroma MC, dequantisation and the
//    normative inverse transform with DPP quad exchanges (grp_inv4x4);
//  * decode_intra_wavefront: intra MBs in MB wavefront order (one workgroup per
//    slot, LDS row-progress counters, as the intra encoder) -- all MBs of an I
//    picture, only the intra MBs of a P picture (their inter neighbours are final);
//  * the in-loop filter is the encoder's deblock kernel (deblock.hip), fed with the
//    same MbHeader / non-zero flags this file writes.
//
// Reference parity: the reference decodes with ffmpeg inside the worker
// (client.go:115-118); the CPU decoder (h264_decoder.cc) is the bit-exact oracle.
#include "kcommon.h"

namespace mivc {
namespace gpu {

using h264::MbHeader;

struct DecodeArgs {
  Geom g;
  const uint8_t *ref_y, *ref_u, *ref_v;  // [B] reference picture per slot (P pictures)
  uint8_t *rec_y, *rec_u, *rec_v;        // [B] picture being reconstructed
  const MbHeader* hdr;                   // [B, nmb]
  const uint32_t* mask;                  // [B, nmb] present blocks
  const uint32_t* off;                   // [B, nmb] first block (units of 16 levels, into coef)
  const int16_t* coef;                   // packed levels
  const int8_t* run;                     // [B] 0 idle, 1 I picture, 2 P picture
  int chroma_qp_offset;
  uint8_t* nz;                           // [B, nmb, 16] luma non-zero flags (raster), for deblocking
  int* err;
};

// blkIdx -> 4x4 block column / row (no table: lane-varying lookups would be memory loads)
__device__ __forceinline__ int blk_x(int b) { return ((b >> 2) & 1) * 2 + (b & 1); }
__device__ __forceinline__ int blk_y(int b) { return ((b >> 3) & 1) * 2 + ((b >> 1) & 1); }

// level at scan position sp of block `bit` (0 if the block is absent)
__device__ __forceinline__ int level_at(const int16_t* coef, uint32_t mask, uint32_t off, int bit, int sp) {
  if (!((mask >> bit) & 1u)) return 0;
  const uint32_t idx = off + __builtin_popcount(mask & ((1u << bit) - 1u));
  return coef[static_cast<size_t>(idx) * 16 + sp];
}

// dequantised AC/4x4 residual row gy of a block: v[x] = LevelScale * level << qp/6 (flat
// weights; the >> 4 of 8.5.12.1 is folded into the table); skip_dc leaves (0, 0) at 0
__device__ __forceinline__ void dequant_row(const int16_t* coef, uint32_t mask, uint32_t off, int bit, int gy, int qp,
                                            bool skip_dc, int* v) {
  const int qm = qp % 6, qs = qp / 6;
  const int d0 = h264::kDequantV[qm][0], d1 = h264::kDequantV[qm][1], d2 = h264::kDequantV[qm][2];
  const bool have = (mask >> bit) & 1u;
  const int16_t* c = coef + static_cast<size_t>(off + __builtin_popcount(mask & ((1u << bit) - 1u))) * 16;
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    const int cls = pos_class(x, gy);
    const int dq = cls == 0 ? d0 : (cls == 1 ? d1 : d2);
    const int lv = (have && !(skip_dc && x == 0 && gy == 0)) ? c[zzinv(x, gy)] : 0;
    v[x] = (lv * dq) << qs;
  }
}

// chroma DC of block cb after the 2x2 inverse transform and scaling (8.5.11)
__device__ __forceinline__ int chroma_dc_value(const int16_t* coef, uint32_t mask, uint32_t off, int comp, int cb,
                                               int qpc) {
  if (!((mask >> 17) & 1u)) return 0;
  const int16_t* c = coef + static_cast<size_t>(off + __builtin_popcount(mask & ((1u << 17) - 1u))) * 16 + comp * 4;
  const int c0 = c[0], c1 = c[1], c2 = c[2], c3 = c[3];
  const int f = cb == 0 ? c0 + c1 + c2 + c3 : (cb == 1 ? c0 - c1 + c2 - c3 : (cb == 2 ? c0 + c1 - c2 - c3 : c0 - c1 - c2 + c3));
  const int ls = 16 * h264::kDequantV[qpc % 6][0];
  return ((f * ls) << (qpc / 6)) >> 5;
}

__device__ __forceinline__ uint32_t pack4(const int* p) {
  return static_cast<uint32_t>(p[0]) | static_cast<uint32_t>(p[1]) << 8 | static_cast<uint32_t>(p[2]) << 16 |
         static_cast<uint32_t>(p[3]) << 24;
}

// ============================================================== inter macroblocks
constexpr int kWin = 13;  // 8x8 quadrant + 6-tap support (-2 .. +3)

__global__ __launch_bounds__(64) void decode_inter_mb(DecodeArgs a) {
  const Geom& g = a.g;
  const int mb = blockIdx.x, slot = blockIdx.y;
  if (a.run[slot] != 2) return;
  const size_t o = static_cast<size_t>(slot) * g.nmb() + mb;
  const MbHeader* H = a.hdr + o;
  if (h264::mbk_is_intra(H->kind)) return;
  __shared__ uint8_t win[4][kWin * kWin];
  const int lane = threadIdx.x;
  const int mx = mb % g.wmb, my = mb / g.wmb;
  const int W = g.W, Hh = g.H, cw = g.cw(), ch = g.ch();
  const int X0 = mx * 16, Y0 = my * 16;
  const int qp = H->qp;
  const int qpc = h264::chroma_qp(qp, a.chroma_qp_offset);
  const uint32_t mask = a.mask[o], off = a.off[o];
  const int m0x = H->mv[0][0][0], m0y = H->mv[0][0][1], m1x = H->mv[0][1][0], m1y = H->mv[0][1][1];
  const int m2x = H->mv[0][2][0], m2y = H->mv[0][2][1], m3x = H->mv[0][3][0], m3y = H->mv[0][3][1];

  // ---- stage the four quadrant windows of the reference (clamped: unrestricted MVs)
  const uint8_t* refy = a.ref_y + slot * g.ysize();
  for (int i = lane; i < 4 * kWin * kWin; i += 64) {
    const int q = i / (kWin * kWin), j = i - q * kWin * kWin;
    const int r = j / kWin, c = j - r * kWin;
    const int qx = sel4(q, m0x, m1x, m2x, m3x), qy = sel4(q, m0y, m1y, m2y, m3y);
    const int x = clampi(X0 + (q & 1) * 8 + (qx >> 2) - 2 + c, 0, W - 1);
    const int y = clampi(Y0 + (q >> 1) * 8 + (qy >> 2) - 2 + r, 0, Hh - 1);
    win[q][j] = refy[static_cast<size_t>(y) * W + x];
  }
  __syncthreads();

  // ---- luma: lane = blkIdx * 4 + row
  {
    const int blk = lane >> 2, gy = lane & 3;
    const int bx = blk_x(blk), by = blk_y(blk);
    const int q = (bx >> 1) + 2 * (by >> 1);
    const int qx = sel4(q, m0x, m1x, m2x, m3x), qy = sel4(q, m0y, m1y, m2y, m3y);
    const uint8_t* w = win[q];
    auto ref = [&](int x, int y) { return static_cast<int>(w[(y + 2) * kWin + x + 2]); };
    const int lx = (bx & 1) * 4, ly = (by & 1) * 4 + gy;
    int pr[4], v[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) pr[x] = h264::mc_luma_sample(ref, lx + x, ly, qx & 3, qy & 3);
    dequant_row(a.coef, mask, off, blk, gy, qp, false, v);
    grp_inv4x4(v, lane & ~3, gy);
#pragma unroll
    for (int x = 0; x < 4; ++x) pr[x] = h264::clip1(pr[x] + v[x]);
    uint8_t* recy = a.rec_y + slot * g.ysize();
    *reinterpret_cast<uint32_t*>(recy + static_cast<size_t>(Y0 + by * 4 + gy) * W + X0 + bx * 4) = pack4(pr);
    if (lane < 16) a.nz[o * 16 + blk_x(lane) + 4 * blk_y(lane)] = (mask >> lane) & 1u;
  }
  // ---- chroma: (lane & 31) = comp * 16 + block * 4 + row; lanes 32-63 mirror 0-31
  {
    const int cl = lane & 31, comp = cl >> 4, cb = (cl >> 2) & 3, gy = cl & 3;
    const int cbx = (cb & 1) * 4, cby = (cb >> 1) * 4;
    const int cmx = sel4(cb, m0x, m1x, m2x, m3x), cmy = sel4(cb, m0y, m1y, m2y, m3y);
    const uint8_t* refc = (comp == 0 ? a.ref_u : a.ref_v) + slot * g.csize();
    const int xf = cmx & 7, yf = cmy & 7;
    const int yi = my * 8 + cby + gy + (cmy >> 3);
    const int y0 = clampi(yi, 0, ch - 1), y1 = clampi(yi + 1, 0, ch - 1);
    const int xb = mx * 8 + cbx + (cmx >> 3);
    int top[5], bot[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int xx = clampi(xb + k, 0, cw - 1);
      top[k] = refc[static_cast<size_t>(y0) * cw + xx];
      bot[k] = refc[static_cast<size_t>(y1) * cw + xx];
    }
    int pr[4], v[4];
#pragma unroll
    for (int x = 0; x < 4; ++x)
      pr[x] = ((8 - xf) * (8 - yf) * top[x] + xf * (8 - yf) * top[x + 1] + (8 - xf) * yf * bot[x] + xf * yf * bot[x + 1] +
               32) >> 6;
    dequant_row(a.coef, mask, off, 18 + comp * 4 + cb, gy, qpc, true, v);
    if (gy == 0) v[0] = chroma_dc_value(a.coef, mask, off, comp, cb, qpc);
    grp_inv4x4(v, lane & ~3, gy);
#pragma unroll
    for (int x = 0; x < 4; ++x) pr[x] = h264::clip1(pr[x] + v[x]);
    if (lane < 32) {
      uint8_t* recc = (comp == 0 ? a.rec_u : a.rec_v) + slot * g.csize();
      *reinterpret_cast<uint32_t*>(recc + static_cast<size_t>(my * 8 + cby + gy) * cw + mx * 8 + cbx) = pack4(pr);
    }
  }
}

// ============================================================== intra macroblocks
// Intra4x4 neighbour availability of block b (top-right per 6.4.11.4 / the blkIdx order)
__device__ __forceinline__ int i4_avail(int b, int mbav) {
  const int bx = blk_x(b), by = blk_y(b);
  const bool left = bx > 0 || (mbav & h264::AV_LEFT), top = by > 0 || (mbav & h264::AV_TOP);
  int av = 0;
  if (left) av |= h264::AV_LEFT;
  if (top) av |= h264::AV_TOP;
  if (left && top) av |= h264::AV_TOPLEFT;
  bool tr;
  if (b == 3 || b == 7 || b == 11 || b == 13 || b == 15) tr = false;
  else if (b == 5) tr = (mbav & h264::AV_TOPRIGHT) != 0;
  else if (b == 0 || b == 1 || b == 4) tr = (mbav & h264::AV_TOP) != 0;
  else tr = true;
  if (tr) av |= h264::AV_TOPRIGHT;
  return av;
}

constexpr int kDecIntraWaves = 8;
constexpr int TS = kTileStride;

struct DecIntraShared {
  uint8_t tile[17 * TS];            // luma: row 0 / col 0 = reconstructed neighbours
  int16_t res[16][16];              // Intra4x4 residual per blkIdx (raster)
  int e4[16];                       // Intra4x4 neighbour vector of the current block
  int lv16dc[16];                   // Intra16x16 DC after the inverse Hadamard + scaling (raster)
  uint8_t ctop[2][9], cleft[2][8];  // chroma neighbours [comp][-1..7]
  int cdcp[2][4];                   // chroma DC predictions per (comp, block)
  int saved_x;
  uint8_t saved_y[16];
  uint8_t saved_c[2][8];
};

__device__ __forceinline__ void decode_intra_mb(const DecodeArgs& a, DecIntraShared& S, int slot, int mx, int my) {
  const Geom& g = a.g;
  const int lane = lane_id();
  const int gy = lane & 3;
  const int W = g.W, cw = g.cw();
  const int X0 = mx * 16, Y0 = my * 16;
  const size_t o = static_cast<size_t>(slot) * g.nmb() + my * g.wmb + mx;
  const MbHeader* H = a.hdr + o;
  const int kind = __builtin_amdgcn_readfirstlane(H->kind);
  const int qp = __builtin_amdgcn_readfirstlane(H->qp);
  const int qpc = h264::chroma_qp(qp, a.chroma_qp_offset);
  const int mode16 = __builtin_amdgcn_readfirstlane(H->i16_mode);
  const int cmode = __builtin_amdgcn_readfirstlane(H->chroma_mode);
  const uint32_t mask = __builtin_amdgcn_readfirstlane(a.mask[o]);
  const uint32_t off = __builtin_amdgcn_readfirstlane(a.off[o]);
  uint8_t* recy = a.rec_y + slot * g.ysize();
  int mbav = 0;
  if (mx > 0) mbav |= h264::AV_LEFT;
  if (my > 0) mbav |= h264::AV_TOP;
  if (mx > 0 && my > 0) mbav |= h264::AV_TOPLEFT;
  if (my > 0 && mx < g.wmb - 1) mbav |= h264::AV_TOPRIGHT;

  // ---- stage the reconstructed neighbourhood
  if (lane < 21) {  // tile row 0: x = X0-1 .. X0+19
    const int x = X0 - 1 + lane;
    const bool ok = my > 0 && x >= 0 && x < W && (lane < 17 || (mbav & h264::AV_TOPRIGHT));
    S.tile[lane] = ok ? recy[static_cast<size_t>(Y0 - 1) * W + x] : 0;
  } else if (lane >= 32 && lane < 48) {  // tile col 0, rows 1..16
    const int r = lane - 32;
    uint8_t v = 0;
    if (mx > 0) v = S.saved_x == mx - 1 ? S.saved_y[r] : recy[static_cast<size_t>(Y0 + r) * W + X0 - 1];
    S.tile[(r + 1) * TS] = v;
  }
  if (lane < 18) {
    const int c = lane / 9, i = lane % 9;
    const uint8_t* rc = (c == 0 ? a.rec_u : a.rec_v) + slot * g.csize();
    const int x = mx * 8 - 1 + i;
    S.ctop[c][i] = (my > 0 && x >= 0) ? rc[static_cast<size_t>(my * 8 - 1) * cw + x] : 0;
  } else if (lane >= 48) {
    const int c = (lane - 48) >> 3, i = (lane - 48) & 7;
    const uint8_t* rc = (c == 0 ? a.rec_u : a.rec_v) + slot * g.csize();
    uint8_t v = 0;
    if (mx > 0) v = S.saved_x == mx - 1 ? S.saved_c[c][i] : rc[static_cast<size_t>(my * 8 + i) * cw + mx * 8 - 1];
    S.cleft[c][i] = v;
  }
  wave_sync();
  if (lane >= 16 && lane < 24) {
    const int c = (lane - 16) >> 2, b = (lane - 16) & 3;
    S.cdcp[c][b] = h264::chroma_dc(S.ctop[c] + 1, S.cleft[c], mbav, b & 1, b >> 1);
  }

  // ---- luma
  const int blk = lane >> 2;
  const int bx = blk_x(blk), by = blk_y(blk);
  if (kind == h264::MBK_I16x16) {
    if (lane == 0) {
      int d[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) d[h264::kZigzag4x4[i]] = level_at(a.coef, mask, off, 16, i);
      h264::hadamard4x4(d);
      const int ls = 16 * h264::kDequantV[qp % 6][0];
#pragma unroll
      for (int r = 0; r < 16; ++r)
        S.lv16dc[r] = qp >= 36 ? (d[r] * ls) << (qp / 6 - 6) : (d[r] * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
    }
    uint8_t top[16], left[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      top[i] = S.tile[1 + i];
      left[i] = S.tile[(i + 1) * TS];
    }
    int pa = 0, pb = 0, pc = 0;
    if (mode16 == 3) h264::i16_plane_params(top, left, static_cast<int>(S.tile[0]), &pa, &pb, &pc);
    const int dc = mode16 == 2 ? h264::i16_dc(top, left, mbav) : 0;
    int v[4], pr[4];
    dequant_row(a.coef, mask, off, blk, gy, qp, true, v);
    wave_sync();
    if (gy == 0) v[0] = S.lv16dc[bx + 4 * by];
    grp_inv4x4(v, lane & ~3, gy);
    const int Yr = by * 4 + gy;
    const int lft = S.tile[(Yr + 1) * TS];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int X = bx * 4 + x;
      const int p = mode16 == 0 ? static_cast<int>(S.tile[1 + X])
                  : (mode16 == 1 ? lft : (mode16 == 2 ? dc : h264::clip1((pa + pb * (X - 7) + pc * (Yr - 7) + 16) >> 5)));
      pr[x] = h264::clip1(p + v[x]);
    }
    wave_sync();
    uint8_t* row = S.tile + (Yr + 1) * TS + bx * 4 + 1;
#pragma unroll
    for (int x = 0; x < 4; ++x) row[x] = static_cast<uint8_t>(pr[x]);
  } else {
    // Intra4x4: all 16 residual blocks at once, then the 16 predictions in order
    {
      int v[4];
      dequant_row(a.coef, mask, off, blk, gy, qp, false, v);
      grp_inv4x4(v, lane & ~3, gy);
#pragma unroll
      for (int x = 0; x < 4; ++x) S.res[blk][gy * 4 + x] = static_cast<int16_t>(v[x]);
    }
    wave_sync();
    for (int b = 0; b < 16; ++b) {
      const int cbx = blk_x(b), cby = blk_y(b);
      const int av = i4_avail(b, mbav);
      if (lane < 13) {  // neighbour vector e[] of h264::i4_pred_sample, one entry per lane
        const uint8_t* rowp = S.tile + (cby * 4) * TS + cbx * 4;
        int v;
        if (lane == 0) v = rowp[0];
        else if (lane < 5) v = rowp[lane];
        else if (lane < 9) v = (av & h264::AV_TOPRIGHT) ? rowp[lane] : rowp[4];
        else v = S.tile[(cby * 4 + 1 + lane - 9) * TS + cbx * 4];
        S.e4[lane] = v;
      }
      wave_sync();
      const int mode = __builtin_amdgcn_readfirstlane(H->i4_modes[b]);
      if (lane < 4) {
        int pr[4];
#pragma unroll
        for (int x = 0; x < 4; ++x) pr[x] = h264::i4_pred_sample(mode, av, S.e4, x, gy);
        uint8_t* row = S.tile + (cby * 4 + gy + 1) * TS + cbx * 4 + 1;
#pragma unroll
        for (int x = 0; x < 4; ++x) row[x] = static_cast<uint8_t>(h264::clip1(pr[x] + S.res[b][gy * 4 + x]));
      }
      wave_sync();
    }
  }
  wave_sync();
  {  // write the luma reconstruction
    const int y = lane >> 2, x4 = (lane & 3) * 4;
    uint32_t word = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) word |= static_cast<uint32_t>(S.tile[(y + 1) * TS + x4 + k + 1]) << (8 * k);
    *reinterpret_cast<uint32_t*>(recy + static_cast<size_t>(Y0 + y) * W + X0 + x4) = word;
  }
  if (lane < 16) a.nz[o * 16 + blk_x(lane) + 4 * blk_y(lane)] = (mask >> lane) & 1u;

  // ---- chroma: (lane & 31) = comp * 16 + block * 4 + row
  {
    const int cl = lane & 31, comp = cl >> 4, cb = (cl >> 2) & 3;
    const int cbx = (cb & 1) * 4, cby = (cb >> 1) * 4;
    int pa = 0, pb = 0, pc = 0;
    if (cmode == 3) h264::chroma_plane_params(S.ctop[comp] + 1, S.cleft[comp], static_cast<int>(S.ctop[comp][0]), &pa, &pb, &pc);
    int v[4], pr[4];
    dequant_row(a.coef, mask, off, 18 + comp * 4 + cb, gy, qpc, true, v);
    if (gy == 0) v[0] = chroma_dc_value(a.coef, mask, off, comp, cb, qpc);
    grp_inv4x4(v, lane & ~3, gy);
    const int Yc = cby + gy;
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int X = cbx + x;
      const int p = cmode == 0 ? S.cdcp[comp][cb]
                  : (cmode == 1 ? S.cleft[comp][Yc]
                  : (cmode == 2 ? S.ctop[comp][1 + X] : h264::clip1((pa + pb * (X - 3) + pc * (Yc - 3) + 16) >> 5)));
      pr[x] = h264::clip1(p + v[x]);
    }
    const uint32_t word = pack4(pr);
    if (lane < 32) {
      uint8_t* recc = (comp == 0 ? a.rec_u : a.rec_v) + slot * g.csize();
      *reinterpret_cast<uint32_t*>(recc + static_cast<size_t>(my * 8 + Yc) * cw + mx * 8 + cbx) = word;
      if (cb & 1) S.saved_c[comp][(cb >> 1) * 4 + gy] = static_cast<uint8_t>(word >> 24);
    }
  }
  if (lane < 16) S.saved_y[lane] = S.tile[(lane + 1) * TS + 16];
  if (lane == 0) S.saved_x = mx;
  wave_sync();
}

__global__ __launch_bounds__(64 * kDecIntraWaves) void decode_intra_wavefront(DecodeArgs a) {
  __shared__ DecIntraShared SS[kDecIntraWaves];
  __shared__ int prog[kMaxRows];
  const Geom& g = a.g;
  const int slot = blockIdx.x;
  const int run = a.run[slot];
  if (run == 0) return;  // uniform per workgroup
  for (int i = threadIdx.x; i < g.hmb; i += blockDim.x) prog[i] = 0;
  const int w = wave_id();
  const int lane = lane_id();
  if (lane == 0) SS[w].saved_x = -2;
  __syncthreads();
  DecIntraShared& S = SS[w];
  for (int y = w; y < g.hmb; y += kDecIntraWaves) {
    if (run == 1) {  // I picture: every MB
      for (int x = 0; x < g.wmb; ++x) {
        if (y > 0) row_wait(prog, y - 1, min(x + 2, g.wmb), a.err);
        decode_intra_mb(a, S, slot, x, y);
        row_publish(prog, y, x + 1);
      }
      continue;
    }
    // P picture: visit only the intra MBs of the row (64 flags per ballot)
    const size_t rowo = static_cast<size_t>(slot) * g.nmb() + static_cast<size_t>(y) * g.wmb;
    for (int x0 = 0; x0 < g.wmb; x0 += 64) {
      const int xl = x0 + lane;
      unsigned long long m = __ballot(xl < g.wmb && h264::mbk_is_intra(a.hdr[rowo + xl].kind));
      while (m) {
        const int x = x0 + __builtin_ctzll(m);
        m &= m - 1;
        if (x > 0) row_publish(prog, y, x);
        if (y > 0) row_wait(prog, y - 1, min(x + 2, g.wmb), a.err);
        decode_intra_mb(a, S, slot, x, y);
        row_publish(prog, y, x + 1);
      }
    }
    row_publish(prog, y, g.wmb);
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

static DecodeArgs make_decode_args(int B, int wmb, int hmb, const uint8_t* ref_y, const uint8_t* ref_u,
                                   const uint8_t* ref_v, uint8_t* rec_y, uint8_t* rec_u, uint8_t* rec_v,
                                   const void* hdr, const uint32_t* mask, const uint32_t* off, const int16_t* coef,
                                   const int8_t* run, int chroma_qp_offset, uint8_t* nz, int* err) {
  DecodeArgs a;
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.ref_y = ref_y;
  a.ref_u = ref_u;
  a.ref_v = ref_v;
  a.rec_y = rec_y;
  a.rec_u = rec_u;
  a.rec_v = rec_v;
  a.hdr = static_cast<const MbHeader*>(hdr);
  a.mask = mask;
  a.off = off;
  a.coef = coef;
  a.run = run;
  a.chroma_qp_offset = chroma_qp_offset;
  a.nz = nz;
  a.err = err;
  return a;
}

// One picture of every slot: inter MBs (P pictures) then intra MBs in wavefront order.
extern "C" void mivc_launch_decode_picture(int B, int wmb, int hmb, const uint8_t* ref_y, const uint8_t* ref_u,
                                           const uint8_t* ref_v, uint8_t* rec_y, uint8_t* rec_u, uint8_t* rec_v,
                                           const void* hdr, const uint32_t* mask, const uint32_t* off,
                                           const int16_t* coef, const int8_t* run, int any_p, int chroma_qp_offset,
                                           uint8_t* nz, int* err, void* stream) {
  DecodeArgs a = make_decode_args(B, wmb, hmb, ref_y, ref_u, ref_v, rec_y, rec_u, rec_v, hdr, mask, off, coef, run,
                                  chroma_qp_offset, nz, err);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (any_p) hipLaunchKernelGGL(decode_inter_mb, dim3(wmb * hmb, B), dim3(64), 0, s, a);
  hipLaunchKernelGGL(decode_intra_wavefront, dim3(B), dim3(64 * kDecIntraWaves), 0, s, a);
}
