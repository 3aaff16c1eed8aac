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
#include "h264_trellis.h"
#include "../common/h264_i4_taps.h"

#include <atomic>
#include <cstdlib>

namespace mivc {
namespace gpu {

using h264::MbHeader;

constexpr int kIntraWaves = 16;  // default workgroup width of encode_intra_wavefront (see below)

#ifdef MIVC_INTRA_PROFILE
__device__ unsigned long long g_intra_prof[16][16];  // [mb][phase] for slot 0, wave 0
__device__ int g_intra_prof_n;
#define PROF(ph) do { if (slot == 0 && wave_id() == 0 && lane == 0 && prof_mb < 16) g_intra_prof[prof_mb][ph] = clock64(); } while (0)
#else
#define PROF(ph) do {} while (0)
#endif

struct IntraArgs {
  Geom g;
  const uint8_t *src_y, *src_u, *src_v;
  uint8_t *rec_y, *rec_u, *rec_v;
  const int* qp;
  const int8_t* aq;  // [B, nmb] adaptive-quantisation QP offsets (nullable)
  int chroma_qp_offset;
  MbHeader* hdr;
  int16_t* coef;
  uint8_t* nz;
  const uint8_t* intra_flag;  // null: every MB is intra (I frame)
  const int* intra_count;     // [B] (P frames)
  int* err;
  int use_i4x4;
  int use_i8x8;  // High profile: Intra8x8 trial (x264 --partitions i8x8, with --8x8dct)
  const SlotRoute* rt;  // routed (route.h): rec_* are pools, each slot's current picture
  int nbuf;
  // MB rows per slice (H264Params.slices): a slice's first row has no neighbours above
  // (6.4.8) and starts without waiting for the row above; 0 = one slice per picture
  int slice_rows;
  // x264 --trellis on the intra MBs' final levels (h264_trellis.h, the lane-parallel form):
  // 1 = 4x4 luma (Intra4x4, Intra16x16 AC), 2 = also Intra8x8 and chroma AC; 0 = dead-zone
  int trellis;
  float trellis_lambda;
  // workgroups per slice (I pictures of small batches): the slice's rows are dealt round-robin
  // to wg_per_slice x NW waves on as many CUs, their progress in gprog ([units][kMaxRows],
  // device memory, zeroed by the launcher); 1 = one workgroup, progress in LDS
  int wg_per_slice;
  int* gprog;
};

__device__ __forceinline__ bool top_in_slice(int my, int slice_rows) {
  return my > 0 && (slice_rows <= 0 || my % slice_rows != 0);
}

constexpr int TS = kTileStride;

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
  int e4[16];              // Intra4x4 neighbour vector of the current block
  int cdcp[2][4];          // chroma DC predictions per (comp, block)
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
  // Intra8x8 trial (High profile)
  uint8_t t8[17 * TS];     // I8x8 trial reconstruction
  uint8_t tr8[8];          // reconstructed row above the top-right MB (x = 16 .. 23)
  int16_t c8[4][64];       // I8x8 trial levels (8x8 zig-zag order)
  int e8t[16], e8l[8], e8tl;
  int f8t[16], f8l[8], f8tl;
  int h8[8][64];           // mode ranking: row Hadamards per (mode group, row, column)
  int d8[64];              // transform buffer
  uint8_t modes8[4];
  uint8_t nz8;
};

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
  (void)mbav;
  if (mode == 0) return S.cdcp[comp][(Y >> 2) * 2 + (X >> 2)];
  if (mode == 1) return S.cleft[comp][Y];
  if (mode == 2) return S.ctop[comp][1 + X];
  return h264::clip1((pa + pb * (X - 3) + pc * (Y - 3) + 16) >> 5);
}

__device__ __forceinline__ int i4_tap_lds(uint32_t t, const int* e) {
  return (static_cast<int>((t >> 12) & 7) * e[t & 15] + static_cast<int>((t >> 15) & 7) * e[(t >> 4) & 15] +
          static_cast<int>((t >> 18) & 7) * e[(t >> 8) & 15] + 2) >> 2;
}

__device__ __forceinline__ int wave_min(int v) { return min64(v); }
__device__ __forceinline__ int wave_sum(int v) { return sum64(v); }

// Lane layout used throughout: a 4x4 block is held by 4 consecutive lanes, one row each
// (see grp_* in kcommon.h), so a wave processes 16 blocks (a whole 16x16 MB) at once.
// tapw[x]: this lane's Intra4x4 tap word for (mode = lane >> 2, row = lane & 3, column x),
// loaded once per kernel (a lane-varying index into __constant__ would be a vector
// memory load on every block)
__device__ __forceinline__ void encode_intra_mb(const IntraArgs& a, IntraShared& S, int slot, int mx, int my,
                                                const uint32_t (&tapw)[4]) {
  const Geom& g = a.g;
  const int lane = lane_id();
#ifdef MIVC_INTRA_PROFILE
  const int prof_mb = my == 0 ? mx : 99;
#endif
  PROF(0);
  const int gb = lane & ~3, gy = lane & 3;
  const int W = g.W, cw = g.cw();
  const int X0 = mx * 16, Y0 = my * 16;
  const size_t o = static_cast<size_t>(slot) * g.nmb() + my * g.wmb + mx;
  // the left MB's edge is in LDS when this wave coded it last: keyed by raster index, not x, so a
  // P row whose first intra MB is one column right of its previous row's last reads global memory
  const bool left_saved = S.saved_x == my * g.wmb + mx - 1;
  const int qp = clampi(a.qp[slot] + (a.aq ? a.aq[o] : 0), 0, 51);
  const int qpc = h264::chroma_qp(qp, a.chroma_qp_offset);
  const int lambda = h264::kLambda[qp];
  const float lam4 = trellis_lambda4(a.trellis_lambda, qp);
  const int qbits = 15 + qp / 6, qbits_c = 15 + qpc / 6;
  const uint8_t* srcy = a.src_y + slot * g.ysize();
  const size_t rcur = route_index(a.rt, a.nbuf, slot, RO_CUR);
  uint8_t* recy = a.rec_y + rcur * g.ysize();
  const bool top = top_in_slice(my, a.slice_rows);
  int mbav = 0;
  if (mx > 0) mbav |= h264::AV_LEFT;
  if (top) mbav |= h264::AV_TOP;
  if (mx > 0 && top) mbav |= h264::AV_TOPLEFT;
  if (top && mx < g.wmb - 1) mbav |= h264::AV_TOPRIGHT;

  // ---- stage source and reconstructed neighbourhood
  {
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
    bool ok = top && x >= 0 && x < W && (lane < 17 || (mbav & h264::AV_TOPRIGHT));
    S.tile[lane] = ok ? recy[static_cast<size_t>(Y0 - 1) * W + x] : 0;
  } else if (lane >= 21 && lane < 29) {  // top-right MB's bottom row x = X0+16 .. X0+23 (Intra8x8 block 1)
    int x = X0 + 16 + lane - 21;
    bool ok = (mbav & h264::AV_TOPRIGHT) && x < W;
    S.tr8[lane - 21] = ok ? recy[static_cast<size_t>(Y0 - 1) * W + x] : 0;
  } else if (lane >= 32 && lane < 48) {  // tile col 0, rows 1..16
    int r = lane - 32;
    uint8_t v = 0;
    if (mx > 0) v = left_saved ? S.saved_y[r] : recy[static_cast<size_t>(Y0 + r) * W + X0 - 1];
    S.tile[(r + 1) * TS] = v;
  }
  if (lane < 18) {  // chroma neighbours: top-left + top
    int c = lane / 9, i = lane % 9;
    const uint8_t* rc = (c == 0 ? a.rec_u : a.rec_v) + rcur * g.csize();
    int x = mx * 8 - 1 + i;
    bool ok = top && x >= 0;
    S.ctop[c][i] = ok ? rc[static_cast<size_t>(my * 8 - 1) * cw + x] : 0;
  } else if (lane >= 48) {  // chroma left
    int c = (lane - 48) >> 3, i = (lane - 48) & 7;
    const uint8_t* rc = (c == 0 ? a.rec_u : a.rec_v) + rcur * g.csize();
    uint8_t v = 0;
    if (mx > 0) v = left_saved ? S.saved_c[c][i] : rc[static_cast<size_t>(my * 8 + i) * cw + mx * 8 - 1];
    S.cleft[c][i] = v;
  }
  if (lane >= 24 && lane < 28) {
    int i = lane - 24;  // most-probable-mode context
    int lm = 2, tm = 2;
    if (mx > 0) {
      if (left_saved) {
        lm = S.saved_modes[i];
      } else {
        const MbHeader& L = a.hdr[o - 1];
        lm = (L.kind == h264::MBK_I4x4 || L.kind == h264::MBK_I8x8) ? L.i4_modes[raster_to_blkidx(3 + 4 * i)] : 2;
      }
    }
    if (top) {
      const MbHeader& T = a.hdr[o - g.wmb];
      tm = (T.kind == h264::MBK_I4x4 || T.kind == h264::MBK_I8x8) ? T.i4_modes[raster_to_blkidx(i + 12)] : 2;
    }
    S.left_modes[i] = lm;
    S.top_modes[i] = tm;
  }
  wave_sync();
  if (lane < 16) {
    S.top16[lane] = S.tile[1 + lane];
    S.left16[lane] = S.tile[(lane + 1) * TS];
  } else if (lane < 24) {  // chroma DC predictions per (comp, block)
    int c = (lane - 16) >> 2, b = (lane - 16) & 3;
    S.cdcp[c][b] = h264::chroma_dc(S.ctop[c] + 1, S.cleft[c], mbav, b & 1, b >> 1);
  }
  wave_sync();
  PROF(1);

  // ---- Intra16x16 decision: one mode per pass, lane = raster block * 4 + row
  const int tl16 = S.tile[0];
  int pa16 = 0, pb16 = 0, pc16 = 0;
  if ((mbav & (h264::AV_TOP | h264::AV_LEFT | h264::AV_TOPLEFT)) == (h264::AV_TOP | h264::AV_LEFT | h264::AV_TOPLEFT))
    h264::i16_plane_params(S.top16, S.left16, tl16, &pa16, &pb16, &pc16);
  // wave-uniform: scalar registers (the LDS reads above leave them in vector registers,
  // which this kernel's 128-VGPR budget cannot spare)
  pa16 = __builtin_amdgcn_readfirstlane(pa16);
  pb16 = __builtin_amdgcn_readfirstlane(pb16);
  pc16 = __builtin_amdgcn_readfirstlane(pc16);
  const int dc16 = __builtin_amdgcn_readfirstlane(h264::i16_dc(S.top16, S.left16, mbav));
  int mode16 = 2, cost16 = 0x3FFFFFFF;
  {
    const int rb = lane >> 2, rbx = (rb & 3) * 4, rby = (rb >> 2) * 4;
    for (int m = 0; m < 4; ++m) {
      if (!h264::i16_mode_ok(m, mbav)) continue;
      int v[4];
#pragma unroll
      for (int x = 0; x < 4; ++x)
        v[x] = static_cast<int>(S.src[(rby + gy) * 16 + rbx + x]) - i16_pred(m, S, dc16, pa16, pb16, pc16, rbx + x, rby + gy);
      int sblk = grp_satd4x4(v, gy);
      int tot = wave_sum(gy == 0 ? sblk : 0) + lambda * 4;
      if (tot < cost16) {
        cost16 = tot;
        mode16 = m;
      }
    }
  }
  PROF(2);
  // ---- chroma decision: 2 passes; lanes 0-31 mode 2p, lanes 32-63 mode 2p+1; (lane&31) = cblk*4 + row
  const int cl = lane & 31, cblk = cl >> 2, ccomp = cblk >> 2, cb = cblk & 3;
  const int cbx = (cb & 1) * 4, cby = (cb >> 1) * 4;
  int cpa = 0, cpb = 0, cpc = 0;
  if ((mbav & (h264::AV_TOP | h264::AV_LEFT | h264::AV_TOPLEFT)) == (h264::AV_TOP | h264::AV_LEFT | h264::AV_TOPLEFT))
    h264::chroma_plane_params(S.ctop[ccomp] + 1, S.cleft[ccomp], static_cast<int>(S.ctop[ccomp][0]), &cpa, &cpb, &cpc);
  int cmode = 0;
  {
    int ckey = 0x7FFFFFFF;
    for (int pass = 0; pass < 2; ++pass) {
      int m = pass * 2 + (lane >> 5);
      bool ok = h264::chroma_mode_ok(m, mbav);
      int v[4];
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        int pv = chroma_pred(m, S, ccomp, mbav, cpa, cpb, cpc, cbx + x, cby + gy);
        v[x] = static_cast<int>(S.srcc[ccomp][(cby + gy) * 8 + cbx + x]) - pv;
      }
      int sblk = grp_satd4x4(v, gy);
      int t = sum32(gy == 0 ? sblk : 0);  // sum within the half-wave
      int key = ok ? (t << 2) | m : 0x7FFFFFFF;
      ckey = min(ckey, key);
    }
    ckey = wave_min(ckey);
    cmode = ckey & 3;
  }

  PROF(3);
  // ---- Intra4x4 trial (closed loop over the 16 blocks; 9 modes ranked in parallel)
  bool use4 = false;
  int cost4 = 0x3FFFFFFF;
  if (a.use_i4x4) {
    for (int i = lane; i < 17 * TS; i += 64) S.t4[i] = S.tile[i];
    wave_sync();
    int total = lambda * 8;
    const int qm = qp % 6, qs = qp / 6;
    const int mf0 = h264::kQuantMF[qm][0], mf1 = h264::kQuantMF[qm][1], mf2 = h264::kQuantMF[qm][2];
    const int dv0 = h264::kDequantV[qm][0], dv1 = h264::kDequantV[qm][1], dv2 = h264::kDequantV[qm][2];
    for (int blk = 0; blk < 16; ++blk) {
      int av;
      const int el = i4_neighbour_lane(S.t4, blk, mbav, lane, &av);
      if (lane < 13) S.e4[lane] = el;
      if (blk == 1) PROF(10);
      const int bx = blkidx_x(blk), by = blkidx_y(blk);
      int ma = bx > 0 ? S.modes4[raster_to_blkidx((bx - 1) + 4 * by)] : S.left_modes[by];
      int mb_ = by > 0 ? S.modes4[raster_to_blkidx(bx + 4 * (by - 1))] : S.top_modes[bx];
      bool dcpred = (bx == 0 && !(mbav & h264::AV_LEFT)) || (by == 0 && !(mbav & h264::AV_TOP));
      int pm = dcpred ? 2 : min(ma, mb_);
      wave_sync();
      int dcv;
      {
        bool t = av & h264::AV_TOP, l = av & h264::AV_LEFT;
        int st = S.e4[1] + S.e4[2] + S.e4[3] + S.e4[4], sl = S.e4[9] + S.e4[10] + S.e4[11] + S.e4[12];
        dcv = __builtin_amdgcn_readfirstlane((t && l) ? (st + sl + 4) >> 3 : (l ? (sl + 2) >> 2 : (t ? (st + 2) >> 2 : 128)));
      }
      if (blk == 1) PROF(11);
      // mode ranking: lane = mode * 4 + row (lanes 0..35)
      int m = lane >> 2;
      bool valid = m < 9 && h264::i4_mode_ok(m, av);
      int mm = m < 9 ? m : 0;
      int v[4];
      uint32_t pw = 0;
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        int pv = mm == 2 ? dcv : i4_tap_lds(tapw[x], S.e4);
        pw |= static_cast<uint32_t>(pv) << (8 * x);
        v[x] = static_cast<int>(S.src[(by * 4 + gy) * 16 + bx * 4 + x]) - pv;
      }
      int sblk = grp_satd4x4(v, gy);
      int key = (valid && gy == 0) ? ((sblk + lambda * (m == pm ? 1 : 4)) << 4) | m : 0x7FFFFFFF;
      key = wave_min(key);
      const int mode = key & 15;
      total += key >> 4;
      if (blk == 1) PROF(12);
      // transform / quantise / reconstruct the chosen mode (every group computes the same block)
      int pr[4];
      // the chosen mode's prediction row gy, from the lane that ranked it
      const uint32_t prw = static_cast<uint32_t>(__shfl(static_cast<int>(pw), mode * 4 + gy));
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        pr[x] = static_cast<int>((prw >> (8 * x)) & 255u);
        v[x] = static_cast<int>(S.src[(by * 4 + gy) * 16 + bx * 4 + x]) - pr[x];
      }
      grp_fwd4x4(v, gb, gy);
      int tl[4];
      if (a.trellis) grp_trellis4x4(v, tl, gy, mf0, mf1, mf2, qbits, lam4, false);
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        int cls = pos_class(x, gy);
        int mf = cls == 0 ? mf0 : (cls == 1 ? mf1 : mf2);
        int dq = cls == 0 ? dv0 : (cls == 1 ? dv1 : dv2);
        int lv = a.trellis ? tl[x] : h264::quant_coef(v[x], mf, qbits, 21);
        if (lane < 4) S.c4[blk][zzinv(x, gy)] = static_cast<int16_t>(lv);
        v[x] = (lv * dq) << qs;
      }
      grp_inv4x4(v, gb, gy);
      if (lane < 4) {
        uint8_t* row = S.t4 + (by * 4 + 1 + gy) * TS + bx * 4 + 1;
#pragma unroll
        for (int x = 0; x < 4; ++x) row[x] = static_cast<uint8_t>(h264::clip1(pr[x] + v[x]));
      }
      if (lane == 0) S.modes4[blk] = static_cast<uint8_t>(mode);
      wave_sync();
      if (blk == 1) PROF(13);
    }
    use4 = total < cost16;
    cost4 = __builtin_amdgcn_readfirstlane(total);
  }
  PROF(9);  // (profile builds: I4x4 trial done, I8x8 next)

  // ---- Intra8x8 trial (closed loop over the four 8x8 blocks, 9 modes ranked on sa8d)
  bool use8 = false;
  if (a.use_i8x8) {
    for (int i = lane; i < 17 * TS; i += 64) S.t8[i] = S.tile[i];
    wave_sync();
    int total8 = lambda * 8;
    const int qm = qp % 6, q6 = qp / 6, qbits8 = 16 + qp / 6;
    for (int b8 = 0; b8 < 4; ++b8) {
      const int bx = (b8 & 1) * 8, by = (b8 >> 1) * 8;
      // reference samples and their availability (8.3.2.2): block 1's top-right lies in the
      // top-right MB, block 2's in block 1, block 3 has none
      const bool has_top = by > 0 || (mbav & h264::AV_TOP);
      const bool has_left = bx > 0 || (mbav & h264::AV_LEFT);
      const bool has_tl = b8 == 3 || (b8 == 0 ? (mbav & h264::AV_TOPLEFT) != 0
                                              : (b8 == 1 ? (mbav & h264::AV_TOP) != 0 : (mbav & h264::AV_LEFT) != 0));
      const bool has_tr = b8 == 2 || (b8 == 0 ? (mbav & h264::AV_TOP) != 0 : (b8 == 1 && (mbav & h264::AV_TOPRIGHT)));
      const uint8_t* above = S.t8 + by * TS + bx + 1;  // row above the block, x = 0
      if (lane < 16) {
        S.e8t[lane] = lane < 8 ? above[lane] : (has_tr ? (b8 == 1 ? S.tr8[lane - 8] : above[lane]) : above[7]);
      } else if (lane < 24) {
        S.e8l[lane - 16] = S.t8[(by + 1 + lane - 16) * TS + bx];
      } else if (lane == 24) {
        S.e8tl = S.t8[by * TS + bx];
      }
      wave_sync();
      const int tl8 = S.e8tl;
      if (lane < 16 && has_top) {  // 8.3.2.2.1 reference sample filtering
        const int* t = S.e8t;
        int f;
        if (lane == 0) f = has_tl ? (tl8 + 2 * t[0] + t[1] + 2) >> 2 : (3 * t[0] + t[1] + 2) >> 2;
        else if (lane == 15) f = (t[14] + 3 * t[15] + 2) >> 2;
        else f = (t[lane - 1] + 2 * t[lane] + t[lane + 1] + 2) >> 2;
        S.f8t[lane] = f;
      } else if (lane >= 16 && lane < 24 && has_left) {
        const int* l = S.e8l;
        const int y = lane - 16;
        int f;
        if (y == 0) f = has_tl ? (tl8 + 2 * l[0] + l[1] + 2) >> 2 : (3 * l[0] + l[1] + 2) >> 2;
        else if (y == 7) f = (l[6] + 3 * l[7] + 2) >> 2;
        else f = (l[y - 1] + 2 * l[y] + l[y + 1] + 2) >> 2;
        S.f8l[y] = f;
      } else if (lane == 24) {
        int f = 0;
        if (has_tl) {
          if (has_top && has_left) f = (S.e8t[0] + 2 * tl8 + S.e8l[0] + 2) >> 2;
          else if (has_top) f = (3 * tl8 + S.e8t[0] + 2) >> 2;
          else if (has_left) f = (3 * tl8 + S.e8l[0] + 2) >> 2;
          else f = tl8;
        }
        S.f8tl = f;
      }
      wave_sync();
      int dc8 = 128;
      {
        int st = 0, sl = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          st += has_top ? S.f8t[i] : 0;
          sl += has_left ? S.f8l[i] : 0;
        }
        dc8 = (has_top && has_left) ? (st + sl + 8) >> 4 : (has_left ? (sl + 4) >> 3 : (has_top ? (st + 4) >> 3 : 128));
      }
      // predicted mode (8.3.2.1): the left / upper 8x8 block's mode; a neighbouring I4x4 MB
      // gives its 4x4 block next to this block's first 4x4 (the writers' rule)
      const int ma = bx > 0 ? S.modes8[b8 - 1] : S.left_modes[by >> 2];
      const int mb_ = by > 0 ? S.modes8[b8 - 2] : S.top_modes[bx >> 2];
      const bool dcpred = (bx == 0 && !(mbav & h264::AV_LEFT)) || (by == 0 && !(mbav & h264::AV_TOP));
      const int pm = dcpred ? 2 : min(ma, mb_);
      // mode ranking: lane = (mode group lane >> 3, row lane & 7); two passes cover modes 0..8
      int key = 0x7FFFFFFF;
      for (int pass = 0; pass < 2; ++pass) {
        const int m = pass * 8 + (lane >> 3), r = lane & 7;
        const bool valid = m < 9 && (m == 2 || ((m == 0 || m == 3 || m == 7) && has_top) || ((m == 1 || m == 8) && has_left) ||
                                     ((m == 4 || m == 5 || m == 6) && has_top && has_left && has_tl));
        int v[8];
#pragma unroll
        for (int x = 0; x < 8; ++x)
          v[x] = m < 9 ? static_cast<int>(S.src[(by + r) * 16 + bx + x]) - i8_pred_tap(m, x, r, S.f8t, dc8) : 0;
        had8_pass(v, 1);
#pragma unroll
        for (int x = 0; x < 8; ++x) S.h8[lane >> 3][r * 8 + x] = v[x];
        wave_sync();
        const int c = lane & 7;
#pragma unroll
        for (int y = 0; y < 8; ++y) v[y] = S.h8[lane >> 3][y * 8 + c];
        had8_pass(v, 1);
        int sa = 0;
#pragma unroll
        for (int y = 0; y < 8; ++y) sa += v[y] < 0 ? -v[y] : v[y];
        sa += __shfl_xor(sa, 1);
        sa += __shfl_xor(sa, 2);
        sa += __shfl_xor(sa, 4);
        const int cost = ((sa + 2) >> 2) + lambda * (m == pm ? 1 : 4);
        if (valid && c == 0) key = min(key, (cost << 4) | m);
        wave_sync();
      }
      key = wave_min(key);
      const int mode = key & 15;
      total8 += key >> 4;
      // transform / quantise / reconstruct the chosen mode: lane = sample (x, y) for the
      // prediction, rows / columns on lanes 0-7 for the transform, lane = scan index for the levels
      const int x = lane & 7, y = lane >> 3;
      const int pr = i8_pred_sample(mode, x, y, S.f8t, S.f8l, S.f8tl, dc8);
      S.d8[lane] = static_cast<int>(S.src[(by + y) * 16 + bx + x]) - pr;
      wave_sync();
      if (lane < 8) dct8_pass(S.d8 + lane * 8, 1);
      wave_sync();
      if (lane < 8) dct8_pass(S.d8 + lane, 8);
      wave_sync();
      {
        const int pos = kZz8[lane];
        const int cls = pos8(pos & 7, pos >> 3);
        const int mf8 = kQuant8MF[qm][cls];
        int lv;
        if (a.trellis >= 2) {  // the whole 8x8 block at once: lane = scan index
          const float az = fabsf(static_cast<float>(S.d8[pos]) * static_cast<float>(mf8) * exp2f(-static_cast<float>(qbits8)));
          int lf, lt;
          trellis_both(az, 1.0f, 1.0f, a.trellis_lambda * 0.136f, static_cast<int>(az + 0.5f), lf, lt);
          const unsigned long long fm = __ballot(lf != 0);
          const int istar = fm ? 63 - __builtin_clzll(fm) : -1;
          const int l = lane > istar ? 0 : (lane == istar ? lf : lt);
          lv = S.d8[pos] < 0 ? -l : l;
        } else {
          lv = h264::quant_coef(S.d8[pos], mf8, qbits8, 21);
        }
        S.c8[b8][lane] = static_cast<int16_t>(lv);
        const int ls = 16 * kNorm8[qm][cls];
        S.d8[pos] = q6 >= 6 ? (lv * ls) << (q6 - 6) : (lv * ls + (1 << (5 - q6))) >> (6 - q6);
        const unsigned long long nzm = __ballot(lv != 0);
        if (lane == 0) S.nz8 = static_cast<uint8_t>((b8 == 0 ? 0 : S.nz8) | ((nzm != 0) << b8));
      }
      wave_sync();
      if (lane < 8) idct8_pass(S.d8 + lane * 8, 1);
      wave_sync();
      if (lane < 8) idct8_pass(S.d8 + lane, 8);
      wave_sync();
      S.t8[(by + 1 + y) * TS + bx + 1 + x] = static_cast<uint8_t>(h264::clip1(pr + ((S.d8[lane] + 32) >> 6)));
      if (lane == 0) S.modes8[b8] = static_cast<uint8_t>(mode);
      wave_sync();
    }
    const int best_other = use4 ? cost4 : cost16;
    use8 = total8 < best_other;
    if (use8) use4 = false;
  }

  PROF(4);
  MbHeader* h = a.hdr + o;
  int16_t* coef = a.coef + o * h264::kCoefPerMb;
  if (use8) {
    for (int i = lane; i < 256; i += 64) coef[h264::COEF_LUMA + i] = S.c8[i >> 6][i & 63];
    if (lane < 16) coef[h264::COEF_LUMA_DC + lane] = 0;
    for (int i = lane; i < 256; i += 64) {
      int y = i >> 4, x = i & 15;
      S.tile[(y + 1) * TS + x + 1] = S.t8[(y + 1) * TS + x + 1];
    }
    if (lane < 16) {
      // nz per 4x4 (raster): the 8x8 block covering it has levels
      const int rx = lane & 3, ry = lane >> 2;
      a.nz[o * 16 + lane] = (S.nz8 >> ((ry >> 1) * 2 + (rx >> 1))) & 1;
      h->i4_modes[lane] = S.modes8[lane >> 2];  // luma4x4BlkIdx: 4 per 8x8 block
    }
  } else if (use4) {
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
      a.nz[o * 16 + blkidx_x(lane) + 4 * blkidx_y(lane)] = any;
      h->i4_modes[lane] = S.modes4[lane];
    }
  } else {
    // ---- Intra16x16 encode: lane = blkIdx * 4 + row
    const int blk = lane >> 2;
    const int bx4 = blkidx_x(blk) * 4, by4 = blkidx_y(blk) * 4;
    int pr[4], v[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      pr[x] = i16_pred(mode16, S, dc16, pa16, pb16, pc16, bx4 + x, by4 + gy);
      v[x] = static_cast<int>(S.src[(by4 + gy) * 16 + bx4 + x]) - pr[x];
    }
    grp_fwd4x4(v, gb, gy);
    if (gy == 0) S.dc16[blkidx_x(blk) + 4 * blkidx_y(blk)] = v[0];
    const int qm = qp % 6, qs = qp / 6;
    bool any = false;
    int tl[4];
    if (a.trellis)
      grp_trellis4x4(v, tl, gy, h264::kQuantMF[qm][0], h264::kQuantMF[qm][1], h264::kQuantMF[qm][2], qbits, lam4, true);
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      int cls = pos_class(x, gy);
      int lv = (gy == 0 && x == 0) ? 0 : (a.trellis ? tl[x] : h264::quant_coef(v[x], h264::kQuantMF[qm][cls], qbits, 21));
      S.c16[blk][zzinv(x, gy)] = static_cast<int16_t>(lv);
      any |= lv != 0;
      v[x] = (lv * h264::kDequantV[qm][cls]) << qs;
    }
    wave_sync();
    if (lane == 0) {
      int d[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) d[i] = S.dc16[i];
      h264::hadamard4x4(d);
      int lvd[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) lvd[r] = h264::quant_coef(d[r] >> 1, h264::kQuantMF[qm][0], qbits + 1, 21);
#pragma unroll
      for (int i = 0; i < 16; ++i) coef[h264::COEF_LUMA_DC + i] = static_cast<int16_t>(lvd[h264::kZigzag4x4[i]]);
      h264::hadamard4x4(lvd);
      int ls = 16 * h264::kDequantV[qm][0];
#pragma unroll
      for (int r = 0; r < 16; ++r)
        S.lv16dc[r] = qp >= 36 ? (lvd[r] * ls) << (qp / 6 - 6) : (lvd[r] * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
    }
    wave_sync();
    if (gy == 0) v[0] = S.lv16dc[blkidx_x(blk) + 4 * blkidx_y(blk)];
    grp_inv4x4(v, gb, gy);
    uint8_t* row = S.tile + (by4 + gy + 1) * TS + bx4 + 1;
#pragma unroll
    for (int x = 0; x < 4; ++x) row[x] = static_cast<uint8_t>(h264::clip1(pr[x] + v[x]));
    any = sum4(static_cast<int>(any)) != 0;
    if (gy == 0) a.nz[o * 16 + blkidx_x(blk) + 4 * blkidx_y(blk)] = any;
    wave_sync();
    for (int i = lane; i < 256; i += 64) coef[h264::COEF_LUMA + i] = S.c16[i >> 4][i & 15];
  }
  wave_sync();
  PROF(5);
  {  // ---- write luma reconstruction
    int y = lane >> 2, x4 = (lane & 3) * 4;
    uint32_t word = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) word |= static_cast<uint32_t>(S.tile[(y + 1) * TS + x4 + k + 1]) << (8 * k);
    *reinterpret_cast<uint32_t*>(recy + static_cast<size_t>(Y0 + y) * W + X0 + x4) = word;
  }
  // ---- chroma encode: (lane & 31) = cblk*4 + row; lanes 32-63 duplicate lanes 0-31
  {
    const int qm = qpc % 6, qs = qpc / 6;
    int pr[4], v[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      pr[x] = chroma_pred(cmode, S, ccomp, mbav, cpa, cpb, cpc, cbx + x, cby + gy);
      v[x] = static_cast<int>(S.srcc[ccomp][(cby + gy) * 8 + cbx + x]) - pr[x];
    }
    grp_fwd4x4(v, gb, gy);
    if (gy == 0 && lane < 32) S.cdc[ccomp][cb] = v[0];
    int tl[4];
    if (a.trellis >= 2)
      grp_trellis4x4(v, tl, gy, h264::kQuantMF[qm][0], h264::kQuantMF[qm][1], h264::kQuantMF[qm][2], qbits_c,
                     trellis_lambda4(a.trellis_lambda, qpc), true);
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      int cls = pos_class(x, gy);
      int lv = (gy == 0 && x == 0) ? 0
                                   : (a.trellis >= 2 ? tl[x] : h264::quant_coef(v[x], h264::kQuantMF[qm][cls], qbits_c, 21));
      if (lane < 32) coef[h264::COEF_CHROMA_AC + (ccomp * 4 + cb) * 16 + zzinv(x, gy)] = static_cast<int16_t>(lv);
      v[x] = (lv * h264::kDequantV[qm][cls]) << qs;
    }
    wave_sync();
    if (lane < 2) {
      int c = lane;
      int d0 = S.cdc[c][0], d1 = S.cdc[c][1], d2 = S.cdc[c][2], d3 = S.cdc[c][3];
      int f0 = d0 + d1 + d2 + d3, f1 = d0 - d1 + d2 - d3, f2 = d0 + d1 - d2 - d3, f3 = d0 - d1 - d2 + d3;
      int mf = h264::kQuantMF[qm][0];
      int l0 = h264::quant_coef(f0, mf, qbits_c + 1, 21), l1 = h264::quant_coef(f1, mf, qbits_c + 1, 21);
      int l2 = h264::quant_coef(f2, mf, qbits_c + 1, 21), l3 = h264::quant_coef(f3, mf, qbits_c + 1, 21);
      coef[h264::COEF_CHROMA_DC + c * 4 + 0] = static_cast<int16_t>(l0);
      coef[h264::COEF_CHROMA_DC + c * 4 + 1] = static_cast<int16_t>(l1);
      coef[h264::COEF_CHROMA_DC + c * 4 + 2] = static_cast<int16_t>(l2);
      coef[h264::COEF_CHROMA_DC + c * 4 + 3] = static_cast<int16_t>(l3);
      int g0 = l0 + l1 + l2 + l3, g1 = l0 - l1 + l2 - l3, g2 = l0 + l1 - l2 - l3, g3 = l0 - l1 - l2 + l3;
      int ls = 16 * h264::kDequantV[qm][0];
      S.clev[c][0] = ((g0 * ls) << qs) >> 5;
      S.clev[c][1] = ((g1 * ls) << qs) >> 5;
      S.clev[c][2] = ((g2 * ls) << qs) >> 5;
      S.clev[c][3] = ((g3 * ls) << qs) >> 5;
    }
    wave_sync();
    if (gy == 0) v[0] = S.clev[ccomp][cb];
    grp_inv4x4(v, gb, gy);
    uint32_t word = 0;
#pragma unroll
    for (int x = 0; x < 4; ++x) word |= static_cast<uint32_t>(h264::clip1(pr[x] + v[x])) << (8 * x);
    if (lane < 32) {
      uint8_t* recc = (ccomp == 0 ? a.rec_u : a.rec_v) + rcur * g.csize();
      *reinterpret_cast<uint32_t*>(recc + static_cast<size_t>(my * 8 + cby + gy) * cw + mx * 8 + cbx) = word;
      if (cb & 1) S.saved_c[ccomp][(cb >> 1) * 4 + gy] = static_cast<uint8_t>(word >> 24);
    }
  }
  PROF(6);
  // ---- keep this MB's right edge in LDS for the next iteration of this wave
  if (lane < 16) S.saved_y[lane] = S.tile[(lane + 1) * TS + 16];
  if (lane >= 16 && lane < 20) {
    int i = lane - 16;
    S.saved_modes[i] = use4 ? S.modes4[raster_to_blkidx(3 + 4 * i)] : (use8 ? S.modes8[(i >> 1) * 2 + 1] : 2);
  }
  if (lane == 63) {
    S.saved_x = my * g.wmb + mx;
    h->kind = use8 ? h264::MBK_I8x8 : (use4 ? h264::MBK_I4x4 : h264::MBK_I16x16);
    h->qp = static_cast<int8_t>(qp);
    h->i16_mode = static_cast<uint8_t>(mode16);
    h->chroma_mode = static_cast<uint8_t>(cmode);
    h->flags = use8 ? h264::MBF_T8x8 : 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) h->mv[0][q][0] = h->mv[0][q][1] = h->mv[1][q][0] = h->mv[1][q][1] = 0;
    *reinterpret_cast<uint2*>(&h->ref[0][0]) = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
  }
  if (!use4 && !use8 && lane >= 32 && lane < 48) h->i4_modes[lane - 32] = 2;
  wave_sync();
  PROF(7);
}

// NW waves per workgroup, one MB row each (rows y, y + NW, ...): 12 by default -- 1.5x the rows
// of a slot in flight of the 8-wave instance at a 168-VGPR budget (the 16-wave one spills 640
// B/lane at 128 VGPRs); same-box A/B of the headline (profiles/r5_intra_waves_ab.md): 12 waves
// 13,114 fps, 16 waves 13,071, 8 waves 13,012, identical bytes.  MIVC_INTRA_WAVES=8 / 16 select
// the other instances
template <int NW>
__global__ __launch_bounds__(64 * NW) void encode_intra_wavefront(IntraArgs a) {
  __shared__ IntraShared SS[NW];
  __shared__ int lprog[kMaxRows];
  const Geom& g = a.g;
  // one workgroup per slice, or wg_per_slice of them: intra prediction never crosses a slice's
  // top edge, so the slices of a picture are independent wavefronts (a 4K batch of 64 slots in
  // 4 slices fills the chip with 256 workgroups instead of 64); a 1080p I picture of 64 slots
  // deals each slice's rows to 4 workgroups.  Workgroup k of unit u is blockIdx k * units + u:
  // with units a multiple of 8 the unit's workgroups share an XCD (blockIdx mod 8).
  const int K = a.wg_per_slice;
  const int per = a.slice_rows > 0 ? (g.hmb + a.slice_rows - 1) / a.slice_rows : 1;
  const int units = g.B * per;
  const int kk = blockIdx.x / units, unit = blockIdx.x - kk * units;
  const int slot = unit / per, sl = unit - slot * per;
  const int y_begin = a.slice_rows > 0 ? sl * a.slice_rows : 0;
  const int y_end = a.slice_rows > 0 ? min(g.hmb, y_begin + a.slice_rows) : g.hmb;
  if (!route_active(a.rt, slot, -1)) return;  // uniform per workgroup
  if (a.intra_flag && a.intra_count[slot] == 0) return;
  int* prog = K > 1 ? a.gprog + static_cast<size_t>(unit) * kMaxRows : lprog;
  if (K == 1)
    for (int i = threadIdx.x; i < g.hmb; i += blockDim.x) lprog[i] = 0;
  const int w = wave_id();
  if (lane_id() == 0) SS[w].saved_x = -2;
  __syncthreads();
  IntraShared& S = SS[w];
  const int lane = lane_id();
  uint32_t tapw[4];
  {
    const int m = lane >> 2 < 9 ? lane >> 2 : 0, r = lane & 3;
#pragma unroll
    for (int x = 0; x < 4; ++x) tapw[x] = h264::kI4Taps[m][r * 4 + x];
  }
  // the row above's progress this wave has already acquired (device-scope waits only when it
  // is not far enough yet: one acquire covers every MB it admits)
  int seen = -1, seen_row = -1;
  auto wait = [&](int row, int target) {
    if (K == 1) {
      row_wait(prog, row, target, a.err);
      return;
    }
    if (seen_row == row && seen >= target) return;
    seen = __builtin_amdgcn_readfirstlane(row_wait_agent(prog, row, target, a.err));
    seen_row = row;
  };
  auto publish = [&](int row, int value) {
    if (K == 1) row_publish(prog, row, value);
    else row_publish_agent(prog, row, value);
  };
  for (int y = y_begin + kk * NW + w; y < y_end; y += K * NW) {
    if (!a.intra_flag) {  // I frame: every MB
      for (int x = 0; x < g.wmb; ++x) {
        if (top_in_slice(y, a.slice_rows)) wait(y - 1, min(x + 2, g.wmb));
        encode_intra_mb(a, S, slot, x, y, tapw);
        publish(y, x + 1);
#ifdef MIVC_INTRA_PROFILE
        if (slot == 0 && w == 0 && lane == 0 && y == 0 && x < 16) g_intra_prof[x][8] = clock64();
#endif
      }
      continue;
    }
    // P frame: fetch the row's intra flags 64 at a time and visit only flagged MBs
    const size_t rowo = static_cast<size_t>(slot) * g.nmb() + static_cast<size_t>(y) * g.wmb;
    for (int x0 = 0; x0 < g.wmb; x0 += 64) {
      const int xl = x0 + lane;
      unsigned long long mask = __ballot(xl < g.wmb && a.intra_flag[rowo + xl] != 0);
      while (mask) {
        const int x = x0 + __builtin_ctzll(mask);
        mask &= mask - 1;
        if (x > 0) publish(y, x);  // MBs before x in this row are final (inter)
        if (top_in_slice(y, a.slice_rows)) wait(y - 1, min(x + 2, g.wmb));
        encode_intra_mb(a, S, slot, x, y, tapw);
        publish(y, x + 1);
      }
    }
    publish(y, g.wmb);
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

// Workgroups of encode_intra_wavefront<nw> that can be resident on the current device at once
// (occupancy x CU count), per device: the multi-workgroup wavefront spins on progress across
// workgroups, so every one of them must be resident (a partitioned or smaller GPU, or CUs held
// by side-stream kernels, would otherwise leave a waiter spinning on an unscheduled producer).
static int intra_resident_capacity(int nw) {
  constexpr int kDev = 64;
  static std::atomic<int> cap[kDev][3];  // 0 = not measured yet
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kDev) return 0;
  const int slot = nw == 16 ? 2 : (nw == 12 ? 1 : 0);
  int c = cap[dev][slot].load(std::memory_order_relaxed);
  if (c > 0) return c;
  int per_cu = 0, cus = 0;
  hipError_t e;
  if (nw == 16) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, encode_intra_wavefront<16>, 64 * 16, 0);
  else if (nw == 12) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, encode_intra_wavefront<12>, 64 * 12, 0);
  else e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, encode_intra_wavefront<8>, 64 * 8, 0);
  if (e != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  c = per_cu * cus;
  cap[dev][slot].store(c > 0 ? c : 0, std::memory_order_relaxed);
  return c;
}

// gprog / gprog_ints: the caller's device buffer for the cross-workgroup row progress
// (per encoder, on the launch stream: no buffer is shared between streams or devices);
// K > 1 needs units * kMaxRows ints of it, else the launch runs one workgroup per slice
extern "C" void mivc_launch_encode_intra(int B, int wmb, int hmb, const uint8_t* src_y, const uint8_t* src_u,
                                         const uint8_t* src_v, uint8_t* rec_y, uint8_t* rec_u, uint8_t* rec_v,
                                         const int* qp, int chroma_qp_offset, void* hdr, int16_t* coef, uint8_t* nz,
                                         const uint8_t* intra_flag, const int* intra_count, int* err, int use_i4x4,
                                         const int8_t* aq, void* stream, int use_i8x8, const void* route, int nbuf,
                                         int slice_rows, int trellis, float trellis_lambda, int* gprog,
                                         long long gprog_ints) {
  IntraArgs a;
  a.trellis = trellis;
  a.trellis_lambda = trellis_lambda;
  a.rt = static_cast<const SlotRoute*>(route);
  a.nbuf = nbuf;
  a.slice_rows = slice_rows;
  a.aq = aq;
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
  a.use_i8x8 = use_i8x8;
  static const int nw = [] {
    const char* e = std::getenv("MIVC_INTRA_WAVES");
    const int v = e ? std::atoi(e) : 12;
    return (v == 8 || v == 16) ? v : 12;
  }();
  const int per = slice_rows > 0 ? (hmb + slice_rows - 1) / slice_rows : 1;
  // I pictures of a batch with fewer slice wavefronts than CUs / 4: several workgroups per
  // slice, each unit's in one XCD when the unit count is a multiple of 8, all of them resident
  // (units * K <= the device's resident capacity).  MIVC_INTRA_WG=1: one per slice.
  static const int wg_cap = [] {
    const char* e = std::getenv("MIVC_INTRA_WG");
    const int v = e ? std::atoi(e) : 4;
    return v < 1 ? 1 : (v > 8 ? 8 : v);
  }();
  const int units = B * per;
  int K = 1;
  if (!intra_flag && units % 8 == 0 && gprog != nullptr) {
    const int resident = std::min(256, intra_resident_capacity(nw));
    while (K * 2 <= wg_cap && units * K * 2 <= resident &&
           static_cast<long long>(units) * kMaxRows <= gprog_ints)
      K *= 2;
  }
  a.wg_per_slice = K;
  a.gprog = K > 1 ? gprog : nullptr;
  if (K > 1)
    (void)hipMemsetAsync(gprog, 0, static_cast<size_t>(units) * kMaxRows * sizeof(int),
                         static_cast<hipStream_t>(stream));
  if (nw == 16)
    hipLaunchKernelGGL(encode_intra_wavefront<16>, dim3(B * per * K), dim3(64 * 16), 0, static_cast<hipStream_t>(stream), a);
  else if (nw == 12)
    hipLaunchKernelGGL(encode_intra_wavefront<12>, dim3(B * per * K), dim3(64 * 12), 0, static_cast<hipStream_t>(stream), a);
  else
    hipLaunchKernelGGL(encode_intra_wavefront<8>, dim3(B * per * K), dim3(64 * 8), 0, static_cast<hipStream_t>(stream), a);
}

#ifdef MIVC_INTRA_PROFILE
extern "C" void mivc_intra_prof_read(unsigned long long* out) {
  hipMemcpyFromSymbol(out, HIP_SYMBOL(g_intra_prof), sizeof(unsigned long long) * 256);
}
#endif
