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
  // decoder use: boundary strengths computed by the parser ([B, nmb, 32], dir * 16 +
  // edge * 4 + segment; null: derive from the records) and the DPB layout of the planes
  // (rec_* = [B][dpb_n] pictures, filtering picture cur_idx[slot]; dpb_n 0: [B] pictures)
  const uint8_t* bs_in;
  int dpb_n;
  const int16_t* cur_idx;
  // encoder routing (route.h): rec_* are pools [B, nbuf, plane]; slots whose picture is not
  // flagged SF_DEBLOCK are left alone
  const SlotRoute* rt;
  int nbuf;
};

constexpr int kDeblockWaves = 16;
constexpr int kRing = 8;        // bottom-edge slots from a wave to the next wave
constexpr int kRingU = 4;       // bottom-edge slots from a wave's upper half to its lower half
constexpr int LT = 20;          // luma tile stride: 4 halo + 16 (rows -4..15, cols -4..15)
constexpr int CT = 12;          // chroma tile stride: 4 halo + 8 (rows -4..7, cols -4..7)
constexpr int kSlotWords = 24;  // luma rows 12..15 (16 words) + Cb/Cr rows 6..7 (2 x 4 words)
constexpr int kMaxCols = 480;   // MB columns (8K: 7680 / 16)

// Layout.  Wave w deblocks MB rows 2w + 32k (upper half-wave, lanes
// 0..31) and 2w + 32k + 1 (lower half, lanes 32..63) in lock step, the lower half two MBs
// behind: step x filters MB (x, y) and MB (x - 2, y + 1), which the raster-order
// dependencies allow (MB (x, y) needs (x - 1, y) and (x + 1, y - 1)).  In each half lanes
// 0..15 filter luma lines and 16..31 Cb / Cr lines, so all 64 lanes filter.
//
// The wavefront hands data on through LDS only: a row reads its top halo (the bottom 4
// luma / 2 chroma rows of the MB above, as they are after that MB's right neighbour ran)
// from the producer's ring, never from global memory, so no global store is waited on.
// Unfiltered inputs (reconstruction, decision records) are prefetched one MB ahead.
// Every output dword is stored exactly once, by the step after which it is final:
//   luma cols 0..11 rows 0..12 -> own step; cols 12..15 rows 0..12 -> right neighbour's
//   step; rows 13..15 -> the step of the MB below (from its top halo); last row / column:
//   own step (chroma alike with cols 0..3 / 4..7 and rows 0..6 / 7).
struct DeblockShared {
  alignas(16) uint8_t ty[LT * LT];
  alignas(16) uint8_t tc[2][CT * CT];
  alignas(16) uint32_t hdrw[3][12];  // first 48 B of the MbHeader of the current, left and top MB
  uint32_t nzw[3][4];                // their non-zero flags (16 bytes each)
  int bs[2][4][4];                   // [dir][edge][segment]
  int par[2][2][2][5];               // [dir][mb edge / inner][luma / chroma]: alpha, beta, tc0 for bS 1..3
  uint32_t left_y[16];               // previous MB's cols 12..15 (final but for rows 13..15)
  uint32_t left_c[2][8];             // previous MB's chroma cols 4..7
  uint32_t bot_y[4][3];              // previous MB's rows 12..15, cols 0..11
  uint32_t bot_c[2][2];              // previous MB's chroma rows 6..7, cols 0..3
};

struct DeblockTables {
  int alpha[52], beta[52], tc0[52][3], cqp[52];
};

// Filter one line across an edge (clause 8.7.2.3/8.7.2.4), branch-free.  P = p3 p2 p1 p0
// (bytes 0..3), Q = q0 q1 q2 q3.  Chroma lines use p1, p0, q0, q1 only (ap/aq forced off).
__device__ __forceinline__ void filt(uint32_t& P, uint32_t& Q, int bs, int alpha, int beta, int tc0, bool chroma) {
  const int p3 = __builtin_amdgcn_ubfe(P, 0, 8), p2 = __builtin_amdgcn_ubfe(P, 8, 8);
  const int p1 = __builtin_amdgcn_ubfe(P, 16, 8), p0 = __builtin_amdgcn_ubfe(P, 24, 8);
  const int q0 = __builtin_amdgcn_ubfe(Q, 0, 8), q1 = __builtin_amdgcn_ubfe(Q, 8, 8);
  const int q2 = __builtin_amdgcn_ubfe(Q, 16, 8), q3 = __builtin_amdgcn_ubfe(Q, 24, 8);
  const int ad0 = abs(p0 - q0);
  const bool on = bs > 0 && ad0 < alpha && abs(p1 - p0) < beta && abs(q1 - q0) < beta;
  const bool apb = !chroma && abs(p2 - p0) < beta, aqb = !chroma && abs(q2 - q0) < beta;
  int np0, np1, np2, nq0, nq1, nq2;
  if (bs < 4) {
    const int tc = chroma ? tc0 + 1 : tc0 + apb + aqb;
    const int delta = clampi((((q0 - p0) << 2) + (p1 - q1) + 4) >> 3, -tc, tc);
    np0 = h264::clip1(p0 + delta);
    nq0 = h264::clip1(q0 - delta);
    const int avg = (p0 + q0 + 1) >> 1;
    np1 = apb ? p1 + clampi((p2 + avg - (p1 << 1)) >> 1, -tc0, tc0) : p1;
    nq1 = aqb ? q1 + clampi((q2 + avg - (q1 << 1)) >> 1, -tc0, tc0) : q1;
    np2 = p2;
    nq2 = q2;
  } else {
    const bool strong = ad0 < ((alpha >> 2) + 2);
    const bool sp = apb && strong, sq = aqb && strong;
    np0 = sp ? (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3 : (2 * p1 + p0 + q1 + 2) >> 2;
    np1 = sp ? (p2 + p1 + p0 + q0 + 2) >> 2 : p1;
    np2 = sp ? (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3 : p2;
    nq0 = sq ? (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3 : (2 * q1 + q0 + p1 + 2) >> 2;
    nq1 = sq ? (p0 + q0 + q1 + q2 + 2) >> 2 : q1;
    nq2 = sq ? (2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3 : q2;
  }
  if (on) {
    const int pv[4] = {p3, np2, np1, np0}, qv[4] = {nq0, nq1, nq2, q3};
    P = pack4_u8(pv);
    Q = pack4_u8(qv);
  }
}

// The four edges of one direction on lane-local lines: d[0..4] = 4-sample groups across
// the line (luma: halo, 0..3, 4..7, 8..11, 12..15; chroma: halo, 0..3, 0..3, 4..7 -- the
// chroma edges 0 and 4 run as edges 0 and 2, which touch disjoint samples of the copy).
__device__ __forceinline__ void edges4(uint32_t (&d)[5], const DeblockShared& S, int dir, int line, bool chroma,
                                       bool has_nb) {
  const int seg = chroma ? (line >> 1) : (line >> 2);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    int bs = S.bs[dir][e][seg & 3];
    if (e == 0 && !has_nb) bs = 0;
    if (chroma && (e & 1)) bs = 0;
    const int* P = S.par[dir][e == 0 ? 0 : 1][chroma ? 1 : 0];
    const int tc0 = P[2 + (bs > 0 && bs < 4 ? bs - 1 : 0)];
    filt(d[e], d[e + 1], bs, P[0], P[1], tc0, chroma);
  }
}

__global__ __launch_bounds__(64 * kDeblockWaves) void deblock_wavefront(DeblockArgs a) {
  __shared__ DeblockShared SS[kDeblockWaves][2];
  __shared__ uint32_t ringL[kDeblockWaves - 1][kRing][kSlotWords];  // lower half -> next wave's upper half
  // The last wave's lower row feeds the FIRST row of the next band, which wave 0 starts only
  // after its own band is done: a short ring there would make the last wave wait on a row
  // that waits on it (a deadlock once the row is wider than the waves' combined slack), so
  // that hand-off gets one slot per MB column.
  __shared__ uint32_t ringB[kMaxCols][kSlotWords];
  __shared__ uint32_t ringU[kDeblockWaves][kRingU][kSlotWords];  // upper half -> own lower half
  __shared__ int prog[kMaxRows];
  __shared__ DeblockTables T;
  const Geom& g = a.g;
  const int slot = blockIdx.x;
  if (a.rt && (a.rt[slot].kind < 0 || !(a.rt[slot].flags & SF_DEBLOCK))) return;  // uniform per workgroup
  for (int i = threadIdx.x; i < g.hmb; i += blockDim.x) prog[i] = 0;
  for (int i = threadIdx.x; i < 52; i += blockDim.x) {
    T.alpha[i] = h264::kAlpha[i];
    T.beta[i] = h264::kBeta[i];
    T.tc0[i][0] = h264::kTc0[i][0];
    T.tc0[i][1] = h264::kTc0[i][1];
    T.tc0[i][2] = h264::kTc0[i][2];
    T.cqp[i] = h264::kChromaQp[i];
  }
  __syncthreads();
  const int w = wave_id();
  // lane-derived values are recomputed per step from an opaque lane id instead of being
  // hoisted out of the loops (at 16 waves the hoisted addresses spilled to scratch)
  auto opaque_lane = []() { int l = lane_id(); asm volatile("" : "+v"(l)); return l; };
  const int half = lane_id() >> 5;
  DeblockShared& S = SS[w][half];
#define DB_LANE_VALUES                                                     \
  const int lane = opaque_lane(), hl = lane & 31;                          \
  const bool is_c = hl >= 16; /* 0..15 luma lines, 16..23 Cb, 24..31 Cr */ \
  const int ccomp = (hl - 16) >> 3, cline = hl & 7;                        \
  const int line = is_c ? cline : hl;
  const int W = g.W, cw = g.cw(), wmb = g.wmb, hmb = g.hmb;
  const size_t pic = a.dpb_n ? static_cast<size_t>(slot) * a.dpb_n + a.cur_idx[slot]
                             : route_index(a.rt, a.nbuf, slot, RO_CUR);
  uint8_t* recy = a.rec_y + pic * g.ysize();
  uint8_t* const rcu = a.rec_u + pic * g.csize();
  uint8_t* const rcv = a.rec_v + pic * g.csize();
  const uint8_t* bs_in = a.bs_in ? a.bs_in + static_cast<size_t>(slot) * g.nmb() * 16 : nullptr;
  auto recc = [&](int c) { return c ? rcv : rcu; };
  const uint32_t* hdr32 = reinterpret_cast<const uint32_t*>(a.hdr) + static_cast<size_t>(slot) * g.nmb() * 16;
  const uint32_t* nz32 = reinterpret_cast<const uint32_t*>(a.nz) + static_cast<size_t>(slot) * g.nmb() * 4;

  // unfiltered inputs of MB (x, y), branch-free (three loads per lane, lane-selected
  // addresses) so that they stay in flight across the previous MB's filtering:
  //   luma lanes: their row (2 x 8 bytes); chroma lanes: their row (8 bytes); and every
  //   lane one record word: 0..11 current header, 12..23 top header, 24..27 current nz,
  //   28..31 top nz
  auto load_inputs = [&](int x, int y, uint32_t (&v)[5]) {
    DB_LANE_VALUES
    (void)line;
    const uint8_t* a1 = recy + static_cast<size_t>(y * 16 + (hl & 15)) * W + x * 16;
    const uint8_t* a2 = a1 + 8;
    if (is_c) a1 = a2 = recc(ccomp) + static_cast<size_t>(y * 8 + cline) * cw + x * 8;
    const size_t mb = static_cast<size_t>(y) * wmb + x;
    const size_t mbt = y > 0 ? mb - wmb : mb;
    const uint32_t* a3 = hl < 12 ? hdr32 + mb * 16 + hl
                                 : (hl < 24 ? hdr32 + mbt * 16 + (hl - 12)
                                            : (hl < 28 ? nz32 + mb * 4 + (hl - 24) : nz32 + mbt * 4 + (hl - 28)));
    const uint2 q1 = *reinterpret_cast<const uint2*>(a1);
    const uint2 q2 = *reinterpret_cast<const uint2*>(a2);
    v[0] = q1.x; v[1] = q1.y; v[2] = q2.x; v[3] = q2.y;
    v[4] = *a3;
  };

  for (int yu = 2 * w; yu < hmb; yu += 2 * kDeblockWaves) {
    const int yl = yu + 1;
    const int y = half ? yl : yu;
    const bool row_ok = y < hmb;
    const bool last_row = y == hmb - 1;
    const bool has_top = y > 0;
    // this wave's lower ring still holds bottom edges of row yl - 32 until row yl - 31 used them
    // (waves 0..14) this wave's lower ring still holds bottom edges of row yl - 32 until row
    // yl - 31 (the next wave's upper row of the previous band) used them.  The last wave's
    // band hand-off buffer is guarded per column instead (see below): a whole-row wait
    // there would wait on the next band's first row, which waits on this wave.
    if (half && w < kDeblockWaves - 1 && yl >= 2 * kDeblockWaves && row_ok && (lane_id() & 31) == 0)
      row_wait_lds(prog, yl - 2 * kDeblockWaves + 1, wmb, a.err);
    uint32_t nxt[5] = {0, 0, 0, 0, 0};
    if (!half) load_inputs(0, y, nxt);
    for (int step = 0; step < wmb + 2; ++step) {
      const int x = half ? step - 2 : step;
      const bool act = row_ok && x >= 0 && x < wmb;
      DB_LANE_VALUES
      const uint32_t cur[5] = {nxt[0], nxt[1], nxt[2], nxt[3], nxt[4]};
      if (row_ok && x + 1 >= 0 && x + 1 < wmb) load_inputs(x + 1, y, nxt);
      if (act) {
        const bool has_left = x > 0, last_col = x == wmb - 1;
        // ---- decision records -> LDS, boundary strengths, filter parameters
        {
          uint32_t* dst = hl < 12 ? &S.hdrw[0][hl]
                                  : (hl < 24 ? &S.hdrw[2][hl - 12] : (hl < 28 ? &S.nzw[0][hl - 24] : &S.nzw[2][hl - 28]));
          *dst = cur[4];
        }
        wave_sync();
        const MbHeader* HQ = reinterpret_cast<const MbHeader*>(S.hdrw[0]);
        {
          const int dir = hl >> 4, e = (hl >> 2) & 3, k = hl & 3;
          int bs = 0;
          const bool mbedge = e == 0;
          if (bs_in) {
            // 4 bits per segment (h264_decoder.h DecodedPicture::bs)
            bs = (bs_in[(static_cast<size_t>(y) * wmb + x) * 16 + (hl >> 1)] >> ((hl & 1) * 4)) & 15;
          } else if (!mbedge || (dir == 0 ? has_left : has_top)) {
            const int pw = mbedge ? (dir == 0 ? 1 : 2) : 0;
            const MbHeader* HP = reinterpret_cast<const MbHeader*>(S.hdrw[pw]);
            const uint8_t* nzbp = reinterpret_cast<const uint8_t*>(S.nzw[pw]);
            const uint8_t* nzb0 = reinterpret_cast<const uint8_t*>(S.nzw[0]);
            const int rq = dir == 0 ? (e + 4 * k) : (k + 4 * e);
            const int rp = dir == 0 ? (mbedge ? 3 + 4 * k : e - 1 + 4 * k) : (mbedge ? k + 12 : k + 4 * (e - 1));
            const bool iq = h264::mbk_is_intra(HQ->kind), ip = h264::mbk_is_intra(HP->kind);
            if ((e & 1) && (HQ->flags & h264::MBF_T8x8)) bs = 0;  // 8x8 transform: no 4-sample inner edges
            else if (mbedge && (iq || ip)) bs = 4;
            else if (iq || ip) bs = 3;
            else if (nzbp[rp] || nzb0[rq]) bs = 2;
            else {
              // bS 1: different reference pictures / number of vectors, or a vector component
              // differing by >= 4 quarter samples (clause 8.7.2.1).  Reference identity is
              // (list, ref_idx): the encoder's lists hold disjoint pictures (past anchors in
              // list 0, the future anchor in list 1), and the GPU decode path takes P only.
              const int qp_ = ((rp >> 3) & 1) * 2 + ((rp & 3) >> 1), qq_ = ((rq >> 3) & 1) * 2 + ((rq & 3) >> 1);
              bool diff = false;
#pragma unroll
              for (int l = 0; l < 2; ++l) {
                const int fp = HP->ref[l][qp_], fq = HQ->ref[l][qq_];
                if ((fp >= 0) != (fq >= 0) || (fp >= 0 && fp != fq)) {
                  diff = true;
                } else if (fp >= 0) {
                  const int dx = HP->mv[l][qp_][0] - HQ->mv[l][qq_][0], dy = HP->mv[l][qp_][1] - HQ->mv[l][qq_][1];
                  diff |= dx >= 4 || dx <= -4 || dy >= 4 || dy <= -4;
                }
              }
              bs = diff ? 1 : 0;
            }
          }
          S.bs[dir][e][k] = bs;
        }
        if (hl < 8) {
          const int dir = hl >> 2, inner = (hl >> 1) & 1, ch = hl & 1;
          const int qpq = HQ->qp;
          const int qpn = reinterpret_cast<const MbHeader*>(S.hdrw[dir == 0 ? 1 : 2])->qp;
          int qq = qpq, qn = inner ? qpq : qpn;
          if (ch) {
            qq = T.cqp[clampi(qq + a.chroma_qp_offset, 0, 51)];
            qn = T.cqp[clampi(qn + a.chroma_qp_offset, 0, 51)];
          }
          const int qpav = (qq + qn + 1) >> 1;
          const int ia = clampi(qpav + a.alpha_off, 0, 51), ib = clampi(qpav + a.beta_off, 0, 51);
          int* P = S.par[dir][inner][ch];
          P[0] = T.alpha[ia];
          P[1] = T.beta[ib];
          P[2] = T.tc0[ia][0];
          P[3] = T.tc0[ia][1];
          P[4] = T.tc0[ia][2];
        }
        // ---- top halo: upper half from the previous wave's lower ring (waits for
        // MB (x + 1, y - 1)), lower half from this wave's upper ring (written last step)
        if (has_top) {
          if (!half) row_wait_lds(prog, y - 1, min(x + 2, wmb), a.err);
          if (hl < kSlotWords) {
            const uint32_t v = half ? ringU[w][x % kRingU][hl]
                                    : (w == 0 ? ringB[x][hl] : ringL[w - 1][x % kRing][hl]);
            if (hl < 16) *reinterpret_cast<uint32_t*>(&S.ty[(hl >> 2) * LT + 4 + (hl & 3) * 4]) = v;
            else {
              const int c = (hl - 16) >> 2, r = ((hl - 16) >> 1) & 1, h = hl & 1;
              *reinterpret_cast<uint32_t*>(&S.tc[c][(2 + r) * CT + 4 + h * 4]) = v;
            }
          }
        }
        wave_sync();

        // ---- vertical edges on rows held in registers
        uint32_t d[5];
        if (!is_c) {
          d[0] = has_left ? S.left_y[hl] : 0u;
          d[1] = cur[0]; d[2] = cur[1]; d[3] = cur[2]; d[4] = cur[3];
        } else {
          d[0] = has_left ? S.left_c[ccomp][cline] : 0u;
          d[1] = cur[0]; d[2] = cur[0]; d[3] = cur[1]; d[4] = 0u;
        }
        edges4(d, S, 0, line, is_c, has_left);
        if (!is_c) {
          uint32_t* row = reinterpret_cast<uint32_t*>(&S.ty[(hl + 4) * LT]);
          row[0] = d[0]; row[1] = d[1]; row[2] = d[2]; row[3] = d[3]; row[4] = d[4];
        } else {
          uint32_t* row = reinterpret_cast<uint32_t*>(&S.tc[ccomp][(cline + 4) * CT]);
          row[0] = d[0];
          row[1] = (d[1] & 0x00FFFFFFu) | (d[2] & 0xFF000000u);
          row[2] = d[3];
        }
        wave_sync();

        // ---- horizontal edges on columns gathered from the tile
        {
          uint8_t* col = is_c ? &S.tc[ccomp][4 + cline] : &S.ty[4 + hl];
          const int pitch = is_c ? CT : LT;
          const int nw = is_c ? 3 : 5;
          uint32_t c[5] = {0, 0, 0, 0, 0};
#pragma unroll
          for (int k = 0; k < 5; ++k) {
            if (k < nw) {
              int v4[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) v4[r] = col[(4 * k + r) * pitch];
              c[k] = pack4_u8(v4);
            }
          }
          if (is_c) { c[4] = 0; c[3] = c[2]; c[2] = c[1]; }
          edges4(c, S, 1, line, is_c, has_top);
          if (is_c) { c[1] = (c[1] & 0x00FFFFFFu) | (c[2] & 0xFF000000u); c[2] = c[3]; }
#pragma unroll
          for (int k = 0; k < 5; ++k) {
            if (k < nw && (k > 0 || has_top)) {
#pragma unroll
              for (int r = 0; r < 4; ++r) col[(4 * k + r) * pitch] = static_cast<uint8_t>(c[k] >> (8 * r));
            }
          }
        }
        wave_sync();

        // ---- global stores (each output word exactly once, see the layout note)
        {
          const int r = hl & 15;
          const bool rowok = r <= 12 || last_row;
          if (!is_c) {
            if (rowok) {  // own cols 0..11
              const uint8_t* t = &S.ty[(r + 4) * LT + 4];
              uint32_t* o = reinterpret_cast<uint32_t*>(recy + static_cast<size_t>(y * 16 + r) * W + x * 16);
              const uint32_t* ti = reinterpret_cast<const uint32_t*>(t);
              o[0] = ti[0]; o[1] = ti[1]; o[2] = ti[2];
              if (last_col) o[3] = ti[3];
            }
          } else if (rowok && has_left) {  // left MB's cols 12..15
            *reinterpret_cast<uint32_t*>(recy + static_cast<size_t>(y * 16 + r) * W + x * 16 - 4) =
                *reinterpret_cast<const uint32_t*>(&S.ty[(r + 4) * LT]);
          }
          if (hl < 3) {  // MB (x, y-1) rows 13..15 from the top halo
            if (has_top) {
              const uint32_t* ti = reinterpret_cast<const uint32_t*>(&S.ty[(1 + hl) * LT + 4]);
              uint32_t* o = reinterpret_cast<uint32_t*>(recy + static_cast<size_t>(y * 16 - 3 + hl) * W + x * 16);
              o[0] = ti[0]; o[1] = ti[1]; o[2] = ti[2]; o[3] = ti[3];
            }
          } else if (hl < 5) {  // chroma MB (x, y-1) row 7
            if (has_top) {
              const int c = hl - 3;
              const uint32_t* ti = reinterpret_cast<const uint32_t*>(&S.tc[c][3 * CT + 4]);
              uint32_t* o = reinterpret_cast<uint32_t*>(recc(c) + static_cast<size_t>(y * 8 - 1) * cw + x * 8);
              o[0] = ti[0]; o[1] = ti[1];
            }
          } else if (hl >= 16) {
            const int c = (hl - 16) >> 3, rc = hl & 7;
            if (rc <= 6 || last_row) {
              const uint32_t* ti = reinterpret_cast<const uint32_t*>(&S.tc[c][(rc + 4) * CT]);
              uint32_t* o = reinterpret_cast<uint32_t*>(recc(c) + static_cast<size_t>(y * 8 + rc) * cw + x * 8);
              o[0] = ti[1];                   // own cols 0..3
              if (last_col) o[1] = ti[2];     // own cols 4..7
              if (has_left) o[-1] = ti[0];    // left MB's cols 4..7
            }
          }
        }

        // ---- bottom edges for the row below: MB x-1 now (its cols 12..15 just became
        // final but for rows 13..15), and MB x too at the end of the row
        if (!last_row && hl < kSlotWords) {
          uint32_t vp, vc;
          if (hl < 16) {
            const int r = hl >> 2, k = hl & 3;  // rows 12..15
            vp = k < 3 ? S.bot_y[r][k] : *reinterpret_cast<const uint32_t*>(&S.ty[(r + 16) * LT]);
            vc = *reinterpret_cast<const uint32_t*>(&S.ty[(r + 16) * LT + 4 + 4 * k]);
          } else {
            const int c = (hl - 16) >> 2, r = ((hl - 16) >> 1) & 1, h = hl & 1;  // rows 6..7
            vp = h == 0 ? S.bot_c[c][r] : *reinterpret_cast<const uint32_t*>(&S.tc[c][(r + 10) * CT]);
            vc = *reinterpret_cast<const uint32_t*>(&S.tc[c][(r + 10) * CT + 4 + 4 * h]);
          }
          if (half && w == kDeblockWaves - 1) {
            // column c of the previous band's hand-off was consumed by row y - 31 at its step c
            if (has_left) {
              if (y >= 2 * kDeblockWaves) row_wait_lds(prog, y - 2 * kDeblockWaves + 1, x, a.err);
              ringB[x - 1][hl] = vp;
            }
            if (last_col) {
              if (y >= 2 * kDeblockWaves) row_wait_lds(prog, y - 2 * kDeblockWaves + 1, x + 1, a.err);
              ringB[x][hl] = vc;
            }
          } else if (half) {
            if (has_left) {
              if (x - 1 >= kRing) row_wait_lds(prog, y + 1, x - kRing, a.err);
              ringL[w][(x - 1) % kRing][hl] = vp;
            }
            if (last_col) {
              if (x >= kRing) row_wait_lds(prog, y + 1, x + 1 - kRing, a.err);
              ringL[w][x % kRing][hl] = vc;
            }
          } else {
            if (has_left) ringU[w][(x - 1) % kRingU][hl] = vp;
            if (last_col) ringU[w][x % kRingU][hl] = vc;
          }
        }
        wave_sync();
        // ---- carry this MB's right part and records to the next step
        if (!is_c) S.left_y[hl] = *reinterpret_cast<const uint32_t*>(&S.ty[(hl + 4) * LT + 16]);
        else S.left_c[ccomp][cline] = *reinterpret_cast<const uint32_t*>(&S.tc[ccomp][(cline + 4) * CT + 8]);
        if (hl < 12) S.bot_y[hl / 3][hl % 3] = *reinterpret_cast<const uint32_t*>(&S.ty[(hl / 3 + 16) * LT + 4 + 4 * (hl % 3)]);
        else if (hl < 16) { const int i = hl - 12; S.bot_c[i >> 1][i & 1] = *reinterpret_cast<const uint32_t*>(&S.tc[i >> 1][((i & 1) + 10) * CT + 4]); }
        else if (hl < 28) S.hdrw[1][hl - 16] = S.hdrw[0][hl - 16];
        else S.nzw[1][hl - 28] = S.nzw[0][hl - 28];
        wave_sync();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        if (hl == 0) __hip_atomic_store(prog + y, x + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

extern "C" void mivc_launch_deblock(int B, int wmb, int hmb, uint8_t* rec_y, uint8_t* rec_u, uint8_t* rec_v,
                                    const void* hdr, const uint8_t* nz, int chroma_qp_offset, int alpha_off,
                                    int beta_off, int* err, void* stream, const void* route, int nbuf) {
  DeblockArgs a;
  a.rt = static_cast<const SlotRoute*>(route);
  a.nbuf = nbuf;
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
  a.bs_in = nullptr;
  a.dpb_n = 0;
  a.cur_idx = nullptr;
  hipLaunchKernelGGL(deblock_wavefront, dim3(B), dim3(64 * kDeblockWaves), 0, static_cast<hipStream_t>(stream), a);
}

// decoder: filter picture cur_idx[slot] of each slot's DPB with the parser's boundary strengths
extern "C" void mivc_launch_deblock_dpb(int B, int wmb, int hmb, int dpb_n, uint8_t* dpb_y, uint8_t* dpb_u,
                                        uint8_t* dpb_v, const int16_t* cur_idx, const void* hdr, const uint8_t* nz,
                                        const uint8_t* bs, int chroma_qp_offset, int alpha_off, int beta_off, int* err,
                                        void* stream) {
  DeblockArgs a;
  a.rt = nullptr;
  a.nbuf = 0;
  a.g = Geom{B, wmb, hmb, wmb * 16, hmb * 16};
  a.rec_y = dpb_y;
  a.rec_u = dpb_u;
  a.rec_v = dpb_v;
  a.hdr = static_cast<const mivc::h264::MbHeader*>(hdr);
  a.nz = nz;
  a.chroma_qp_offset = chroma_qp_offset;
  a.alpha_off = alpha_off;
  a.beta_off = beta_off;
  a.err = err;
  a.bs_in = bs;
  a.dpb_n = dpb_n;
  a.cur_idx = cur_idx;
  hipLaunchKernelGGL(deblock_wavefront, dim3(B), dim3(64 * kDeblockWaves), 0, static_cast<hipStream_t>(stream), a);
}
