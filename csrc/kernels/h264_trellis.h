// Rate-distortion quantisation (x264 --trellis, simplified to a greedy pass in reverse scan
// order) shared by the inter (encode_inter.hip) and intra (encode_intra.hip) encoders.
//
// Every coefficient chooses among 0 and the two levels around the rounded quotient by SSD
// (pixel domain: the error of 4x4 coefficient (i, j) weighs 1 / (n_i n_j), n = 4, 10, 4, 10
// the row norms of the core transform) + lambda * CABAC bits, with static bin costs for
// significance / last (a coefficient above every non-zero one would become the last one),
// greater-than-one and the unary level bins, and the sign.  Levels after the block's last
// non-zero one are never coded, so trailing small coefficients are dropped first.
//
// The pass is serial only through `seen` (a later coefficient kept a non-zero level), so the
// lane-parallel forms below evaluate both choices per coefficient and resolve `seen` with one
// max-reduction: scanning back from the end, every coefficient picks its seen = false choice
// until the first non-zero one (index i*), and every coefficient before i* its seen = true
// choice -- the same levels as the serial pass, decided in parallel over the block.
#pragma once
#include "h264_t8.h"

namespace mivc {
namespace gpu {

constexpr float kSig0 = 0.55f, kSig1 = 1.35f, kLast0 = 0.25f, kLast1 = 2.2f, kGt1No = 0.6f, kGt1Yes = 1.7f;

// static CABAC bits of a non-zero level l >= 1 (significance, last, sign, greater-than-one,
// unary and Exp-Golomb suffix); `seen`: a non-zero level follows in scan order
__device__ __forceinline__ float trellis_level_bits(int l, bool seen) {
  return kSig1 + (seen ? kLast0 : kLast1) + 1.0f +
         (l == 1 ? kGt1No : kGt1Yes + 0.9f * static_cast<float>(min(l - 2, 13)) +
                                (l > 15 ? 2.0f * (31 - __clz(l - 14)) + 1.0f : 0.0f));
}

// SSD lambda of the 4x4 choices at QP qp (x264's lambda2 scale), times the user's multiplier
__device__ __forceinline__ float trellis_lambda4(float mult, int qp) {
  return mult * 0.85f * exp2f((qp - 12) * (1.0f / 3.0f));
}

// start: first scan index coded (1 for chroma AC: the DC goes through the 2x2 Hadamard)
__device__ __forceinline__ void trellis_lite4x4(const int (&w)[16], int (&lv)[16], const int (&mf)[3], int qbits,
                                                float lam, int start = 0) {
  constexpr float kInvNorm[3] = {1.0f / 16.0f, 1.0f / 100.0f, 1.0f / 40.0f};
  // a block whose every rounded quotient is 0 quantises to zeros whatever the choice: most
  // blocks of B pictures -- skip the pass (wave-wide when every lane's block is such)
  int zmax = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int r = h264::kZigzag4x4[i];
    const int a = w[r] < 0 ? -w[r] : w[r];
    if (i >= start) zmax |= (a * mf[h264::kPosClass[r]] + (1 << (qbits - 1))) >> qbits;
  }
  if (zmax == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) lv[r] = 0;
    return;
  }
  bool seen = false;
#pragma unroll
  for (int i = 15; i >= 0; --i) {
    if (i < start) {
      lv[h264::kZigzag4x4[i]] = 0;
      continue;
    }
    const int r = h264::kZigzag4x4[i];
    const int cls = h264::kPosClass[r];
    const int a = w[r] < 0 ? -w[r] : w[r];
    const float fm = static_cast<float>(mf[cls]);
    const int zr = (a * mf[cls] + (1 << (qbits - 1))) >> qbits;  // |W| < 2^14, MF < 2^14
    const float step = static_cast<float>(1 << qbits) / fm;
    const float inv_n = kInvNorm[cls];
    float best = static_cast<float>(a) * static_cast<float>(a) * inv_n + lam * (seen ? kSig0 : 0.0f);
    int bl = 0;
#pragma unroll
    for (int d = 1; d >= 0; --d) {
      const int l = zr - d;
      if (l < 1) continue;
      const float e = static_cast<float>(a) - static_cast<float>(l) * step;
      const float j = e * e * inv_n + lam * trellis_level_bits(l, seen);
      if (j < best) {
        best = j;
        bl = l;
      }
    }
    lv[r] = w[r] < 0 ? -bl : bl;
    seen |= bl != 0;
  }
}

// The same greedy choice for one 16-coefficient chunk (scan positions 16k .. 16k + 15) of an 8x8
// block, in the quantiser's own domain: the 8x8 scaling gives every position the same
// pixel-domain step Qstep, so a level l of exact quotient z costs (z - l)^2 Qstep^2 of SSD and
// lambda / Qstep^2 = 0.85 * 2^((QP - 12) / 3) / (0.390625 * 2^(QP / 3)) = 0.136 per bit (QP-free).
// seen: a later chunk of the block keeps a non-zero level.  lv keeps its sign from z.
__device__ __forceinline__ void trellis_lite8_chunk(const float (&z)[16], int (&lv)[16], float lamq, bool seen) {
  float zmax = 0.0f;
#pragma unroll
  for (int i = 0; i < 16; ++i) zmax = fmaxf(zmax, fabsf(z[i]));
  if (zmax < 0.5f) {  // every rounded quotient is 0
#pragma unroll
    for (int i = 0; i < 16; ++i) lv[i] = 0;
    return;
  }
#pragma unroll
  for (int i = 15; i >= 0; --i) {
    const float az = fabsf(z[i]);
    const int zr = static_cast<int>(az + 0.5f);
    float best = az * az + lamq * (seen ? kSig0 : 0.0f);
    int bl = 0;
#pragma unroll
    for (int d = 1; d >= 0; --d) {
      const int l = zr - d;
      if (l < 1) continue;
      const float e = az - static_cast<float>(l);
      const float j = e * e + lamq * trellis_level_bits(l, seen);
      if (j < best) {
        best = j;
        bl = l;
      }
    }
    lv[i] = z[i] < 0.0f ? -bl : bl;
    seen |= bl != 0;
  }
}

// Both greedy choices of one coefficient: lf with no later non-zero level (seen = false), lt
// with one.  a = |coefficient|, step = the quantiser step in the same units, inv_n = the SSD
// weight of the position, zr = the rounded quotient.  Unsigned levels.
__device__ __forceinline__ void trellis_both(float a, float step, float inv_n, float lam, int zr, int& lf, int& lt) {
  const float d0 = a * a * inv_n;
  float bf = d0, bt = d0 + lam * kSig0;
  lf = 0;
  lt = 0;
#pragma unroll
  for (int d = 1; d >= 0; --d) {
    const int l = zr - d;
    if (l < 1) continue;
    const float e = a - static_cast<float>(l) * step;
    const float dist = e * e * inv_n;
    const float jf = dist + lam * trellis_level_bits(l, false), jt = dist + lam * trellis_level_bits(l, true);
    if (jf < bf) {
      bf = jf;
      lf = l;
    }
    if (jt < bt) {
      bt = jt;
      lt = l;
    }
  }
}

__device__ __forceinline__ int max4(int v) {  // within each group of 4 lanes
  v = max(v, dpp<kDppQuadXor1>(v));
  return max(v, dpp<kDppQuadXor2>(v));
}

// Row-per-lane form (grp_* layout: the 4 lanes of a group hold rows 0..3 of one 4x4 block):
// w = this lane's row of forward-transform coefficients, lv = its signed levels.  skip_dc: the
// block's DC is coded elsewhere (Intra16x16 / chroma AC blocks), so scan index 0 stays 0.
// mf0..2 = the quantiser multipliers of the three position classes.
__device__ __forceinline__ void grp_trellis4x4(const int (&w)[4], int (&lv)[4], int gy, int mf0, int mf1, int mf2,
                                               int qbits, float lam, bool skip_dc) {
  int lf[4], lt[4], istar = -1;
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    const int cls = pos_class(x, gy);
    const int mf = cls == 0 ? mf0 : (cls == 1 ? mf1 : mf2);
    const float inv_n = cls == 0 ? 1.0f / 16.0f : (cls == 1 ? 1.0f / 100.0f : 1.0f / 40.0f);
    const int a = w[x] < 0 ? -w[x] : w[x];
    const int zr = (a * mf + (1 << (qbits - 1))) >> qbits;
    trellis_both(static_cast<float>(a), static_cast<float>(1 << qbits) / static_cast<float>(mf), inv_n, lam, zr, lf[x],
                 lt[x]);
    const int i = zzinv(x, gy);
    if (skip_dc && i == 0) lf[x] = lt[x] = 0;
    if (lf[x] != 0) istar = max(istar, i);
  }
  istar = max4(istar);
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    const int i = zzinv(x, gy);
    const int l = i > istar ? 0 : (i == istar ? lf[x] : lt[x]);
    lv[x] = w[x] < 0 ? -l : l;
  }
}

}  // namespace gpu
}  // namespace mivc
