// H.264 High-profile 8x8 luma tools shared by the encoder kernels (encode_inter.hip,
// encode_intra.hip) and the decoder (decode.hip): the 8x8 core transform pair, the 8x8
// quantisation tables, the 8x8 zig-zag, the sa8d Hadamard and Intra8x8 sample prediction
// (clause 8.3.2.2 on filtered reference samples).
#pragma once
#include "kcommon.h"

namespace mivc {
namespace gpu {

// ---------------------------------------------------------------- 8x8 transform (High)
// position class of an 8x8 coefficient (normAdjust8x8 / quant8 column, 8.5.9)
__device__ __forceinline__ int pos8(int x, int y) {
  if ((x & 3) == 0 && (y & 3) == 0) return 0;
  if ((x & 1) && (y & 1)) return 1;
  if ((x & 3) == 2 && (y & 3) == 2) return 2;
  if (((x & 3) == 0 && (y & 1)) || ((x & 1) && (y & 3) == 0)) return 3;
  if (((x & 3) == 0 && (y & 3) == 2) || ((x & 3) == 2 && (y & 3) == 0)) return 4;
  return 5;
}
static __constant__ int kQuant8MF[6][6] = {{13107, 11428, 20972, 12222, 16777, 15481}, {11916, 10826, 19174, 11058, 14980, 14290},
                                   {10082, 8943, 15978, 9675, 12710, 11985},   {9362, 8228, 14913, 8931, 11984, 11259},
                                   {8192, 7346, 13159, 7740, 10486, 9777},     {7282, 6428, 11570, 6830, 9118, 8640}};
static __constant__ int kNorm8[6][6] = {{20, 18, 32, 19, 25, 24}, {22, 19, 35, 21, 28, 26}, {26, 23, 42, 24, 33, 31},
                                {28, 25, 45, 26, 35, 33}, {32, 28, 51, 30, 40, 38}, {36, 32, 58, 34, 46, 43}};
static __constant__ uint8_t kZz8[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                                 41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                                 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// forward 8-point core transform (the inverse of 8.5.13.2), in place, stride s
__device__ __forceinline__ void dct8_pass(int* d, int s) {
  const int a0 = d[0] + d[7 * s], a1 = d[s] + d[6 * s], a2 = d[2 * s] + d[5 * s], a3 = d[3 * s] + d[4 * s];
  const int a4 = d[0] - d[7 * s], a5 = d[s] - d[6 * s], a6 = d[2 * s] - d[5 * s], a7 = d[3 * s] - d[4 * s];
  const int b0 = a0 + a3, b1 = a1 + a2, b2 = a0 - a3, b3 = a1 - a2;
  const int b4 = a5 + a6 + ((a4 >> 1) + a4), b5 = a4 - a7 - ((a6 >> 1) + a6);
  const int b6 = a4 + a7 - ((a5 >> 1) + a5), b7 = a5 - a6 + ((a7 >> 1) + a7);
  d[0] = b0 + b1;
  d[4 * s] = b0 - b1;
  d[2 * s] = b2 + (b3 >> 1);
  d[6 * s] = (b2 >> 1) - b3;
  d[s] = b4 + (b7 >> 2);
  d[7 * s] = (b4 >> 2) - b7;
  d[3 * s] = b5 + (b6 >> 2);
  d[5 * s] = b6 - (b5 >> 2);
}
// inverse 8-point pass (8.5.13.2), in place, stride s
__device__ __forceinline__ void idct8_pass(int* d, int s) {
  const int d0 = d[0], d1 = d[s], d2 = d[2 * s], d3 = d[3 * s], d4 = d[4 * s], d5 = d[5 * s], d6 = d[6 * s],
            d7 = d[7 * s];
  const int a0 = d0 + d4, a4 = d0 - d4, a2 = (d2 >> 1) - d6, a6 = d2 + (d6 >> 1);
  const int b0 = a0 + a6, b2 = a4 + a2, b4 = a4 - a2, b6 = a0 - a6;
  const int a1 = -d3 + d5 - d7 - (d7 >> 1), a3 = d1 + d7 - d3 - (d3 >> 1);
  const int a5 = -d1 + d7 + d5 + (d5 >> 1), a7 = d3 + d5 + d1 + (d1 >> 1);
  const int b1 = a1 + (a7 >> 2), b7 = a7 - (a1 >> 2), b3 = a3 + (a5 >> 2), b5 = (a3 >> 2) - a5;
  d[0] = b0 + b7;
  d[s] = b2 + b5;
  d[2 * s] = b4 + b3;
  d[3 * s] = b6 + b1;
  d[4 * s] = b6 - b1;
  d[5 * s] = b4 - b3;
  d[6 * s] = b2 - b5;
  d[7 * s] = b0 - b7;
}
// 8-point Hadamard pass (sa8d), in place, stride s
__device__ __forceinline__ void had8_pass(int* d, int s) {
  const int a0 = d[0] + d[s], a1 = d[0] - d[s], a2 = d[2 * s] + d[3 * s], a3 = d[2 * s] - d[3 * s];
  const int a4 = d[4 * s] + d[5 * s], a5 = d[4 * s] - d[5 * s], a6 = d[6 * s] + d[7 * s], a7 = d[6 * s] - d[7 * s];
  const int b0 = a0 + a2, b1 = a1 + a3, b2 = a0 - a2, b3 = a1 - a3;
  const int b4 = a4 + a6, b5 = a5 + a7, b6 = a4 - a6, b7 = a5 - a7;
  d[0] = b0 + b4;
  d[s] = b1 + b5;
  d[2 * s] = b2 + b6;
  d[3 * s] = b3 + b7;
  d[4 * s] = b0 - b4;
  d[5 * s] = b1 - b5;
  d[6 * s] = b2 - b6;
  d[7 * s] = b3 - b7;
}

// Intra8x8 predicted sample (x, y) of mode 0..8 from the filtered references (8.3.2.2.2 -
// 8.3.2.2.10): ft[0..15] = p'[x, -1], fl[0..7] = p'[-1, y], ftl = p'[-1, -1]; dc precomputed
__device__ __forceinline__ int i8_pred_sample(int mode, int x, int y, const int* ft, const int* fl, int ftl, int dc) {
  auto T = [&](int i) { return i < 0 ? ftl : ft[i]; };
  auto L = [&](int i) { return i < 0 ? ftl : fl[i]; };
  switch (mode) {
    case 0: return ft[x];
    case 1: return fl[y];
    case 2: return dc;
    case 3:
      if (x == 7 && y == 7) return (ft[14] + 3 * ft[15] + 2) >> 2;
      return (T(x + y) + 2 * T(x + y + 1) + T(x + y + 2) + 2) >> 2;
    case 4:
      if (x > y) return (T(x - y - 2) + 2 * T(x - y - 1) + T(x - y) + 2) >> 2;
      if (x < y) return (L(y - x - 2) + 2 * L(y - x - 1) + L(y - x) + 2) >> 2;
      return (T(0) + 2 * ftl + L(0) + 2) >> 2;
    case 5: {
      const int z = 2 * x - y;
      if (z >= 0 && (z & 1) == 0) return (T(x - (y >> 1) - 1) + T(x - (y >> 1)) + 1) >> 1;
      if (z >= 0) return (T(x - (y >> 1) - 2) + 2 * T(x - (y >> 1) - 1) + T(x - (y >> 1)) + 2) >> 2;
      if (z == -1) return (L(0) + 2 * ftl + T(0) + 2) >> 2;
      return (L(y - 2 * x - 1) + 2 * L(y - 2 * x - 2) + L(y - 2 * x - 3) + 2) >> 2;
    }
    case 6: {
      const int z = 2 * y - x;
      if (z >= 0 && (z & 1) == 0) return (L(y - (x >> 1) - 1) + L(y - (x >> 1)) + 1) >> 1;
      if (z >= 0) return (L(y - (x >> 1) - 2) + 2 * L(y - (x >> 1) - 1) + L(y - (x >> 1)) + 2) >> 2;
      if (z == -1) return (L(0) + 2 * ftl + T(0) + 2) >> 2;
      return (T(x - 2 * y - 1) + 2 * T(x - 2 * y - 2) + T(x - 2 * y - 3) + 2) >> 2;
    }
    case 7:
      if ((y & 1) == 0) return (T(x + (y >> 1)) + T(x + (y >> 1) + 1) + 1) >> 1;
      return (T(x + (y >> 1)) + 2 * T(x + (y >> 1) + 1) + T(x + (y >> 1) + 2) + 2) >> 2;
    default: {
      const int z = x + 2 * y;
      if (z < 13 && (z & 1) == 0) return (L(y + (x >> 1)) + L(y + (x >> 1) + 1) + 1) >> 1;
      if (z < 13) return (L(y + (x >> 1)) + 2 * L(y + (x >> 1) + 1) + L(y + (x >> 1) + 2) + 2) >> 2;
      if (z == 13) return (L(6) + 3 * L(7) + 2) >> 2;
      return L(7);
    }
  }
}

// The same predictions as taps into the filtered references E = {ft[0..15], fl[0..7], ftl}
// (IntraShared's f8t / f8l / f8tl, contiguous): one table word per (mode, sample) -- for the mode
// ranking, where every 8 lanes evaluate another mode and the switch above would run all nine
// cases under divergent masks.  code = i0 | i1 << 5 | i2 << 10 | kind << 15; kind 0: E[i0],
// 1: (E[i0] + E[i1] + 1) >> 1, 2: (E[i0] + 2 E[i1] + E[i2] + 2) >> 2, 3: (E[i0] + 3 E[i1] + 2) >> 2.
namespace i8tap {
constexpr int T(int i) { return i < 0 ? 24 : i; }
constexpr int L(int i) { return i < 0 ? 24 : 16 + i; }
constexpr uint32_t t1(int a) { return static_cast<uint32_t>(a); }
constexpr uint32_t t2(int a, int b) { return static_cast<uint32_t>(a | b << 5 | 1 << 15); }
constexpr uint32_t t3(int a, int b, int c) { return static_cast<uint32_t>(a | b << 5 | c << 10 | 2 << 15); }
constexpr uint32_t t13(int a, int b) { return static_cast<uint32_t>(a | b << 5 | 3 << 15); }
constexpr uint32_t code(int mode, int x, int y) {
  switch (mode) {
    case 0: return t1(T(x));
    case 1: return t1(L(y));
    case 2: return 0;  // DC: the caller's value
    case 3:
      if (x == 7 && y == 7) return t13(T(14), T(15));
      return t3(T(x + y), T(x + y + 1), T(x + y + 2));
    case 4:
      if (x > y) return t3(T(x - y - 2), T(x - y - 1), T(x - y));
      if (x < y) return t3(L(y - x - 2), L(y - x - 1), L(y - x));
      return t3(T(0), 24, L(0));
    case 5: {
      const int z = 2 * x - y;
      if (z >= 0 && (z & 1) == 0) return t2(T(x - (y >> 1) - 1), T(x - (y >> 1)));
      if (z >= 0) return t3(T(x - (y >> 1) - 2), T(x - (y >> 1) - 1), T(x - (y >> 1)));
      if (z == -1) return t3(L(0), 24, T(0));
      return t3(L(y - 2 * x - 1), L(y - 2 * x - 2), L(y - 2 * x - 3));
    }
    case 6: {
      const int z = 2 * y - x;
      if (z >= 0 && (z & 1) == 0) return t2(L(y - (x >> 1) - 1), L(y - (x >> 1)));
      if (z >= 0) return t3(L(y - (x >> 1) - 2), L(y - (x >> 1) - 1), L(y - (x >> 1)));
      if (z == -1) return t3(L(0), 24, T(0));
      return t3(T(x - 2 * y - 1), T(x - 2 * y - 2), T(x - 2 * y - 3));
    }
    case 7:
      if ((y & 1) == 0) return t2(T(x + (y >> 1)), T(x + (y >> 1) + 1));
      return t3(T(x + (y >> 1)), T(x + (y >> 1) + 1), T(x + (y >> 1) + 2));
    default: {
      const int z = x + 2 * y;
      if (z < 13 && (z & 1) == 0) return t2(L(y + (x >> 1)), L(y + (x >> 1) + 1));
      if (z < 13) return t3(L(y + (x >> 1)), L(y + (x >> 1) + 1), L(y + (x >> 1) + 2));
      if (z == 13) return t13(L(6), L(7));
      return t1(L(7));
    }
  }
}
struct Table {
  uint32_t c[9][64];
  constexpr Table() : c() {
    for (int m = 0; m < 9; ++m)
      for (int i = 0; i < 64; ++i) c[m][i] = code(m, i & 7, i >> 3);
  }
};
}  // namespace i8tap
__device__ constexpr i8tap::Table kI8Taps{};

__device__ __forceinline__ int i8_pred_tap(int mode, int x, int y, const int* E, int dc) {
  if (mode == 2) return dc;
  const uint32_t c = kI8Taps.c[mode][y * 8 + x];
  const int kind = static_cast<int>(c >> 15);
  const int e0 = E[c & 31], e1 = E[(c >> 5) & 31], e2 = E[(c >> 10) & 31];
  const int w1 = kind == 0 ? 0 : (kind == 2 ? 2 : (kind == 3 ? 3 : 1));
  const int sh = kind == 0 ? 0 : (kind == 1 ? 1 : 2);
  return (e0 + w1 * e1 + (kind == 2 ? e2 : 0) + ((1 << sh) >> 1)) >> sh;
}

}  // namespace gpu
}  // namespace mivc
