// Encoder-side block arithmetic shared by the CPU reference encoder and the
// gfx950 HIP kernels (compiled as __host__ __device__).  The decoder does NOT
// use these: its inverse paths are written separately (h264_decoder.cc) so the
// round-trip test can catch a misreading on either side.
#pragma once
#include <cstdint>

#include "h264_tables.h"

namespace mivc {
namespace h264 {

// Forward 4x4 integer core transform W = Cf X Cf^T (raster x + 4*y, in place).
MIVC_HD void forward_core4x4(int* d) {
  for (int y = 0; y < 4; ++y) {
    int* r = d + 4 * y;
    int s03 = r[0] + r[3], d03 = r[0] - r[3], s12 = r[1] + r[2], d12 = r[1] - r[2];
    r[0] = s03 + s12;
    r[1] = 2 * d03 + d12;
    r[2] = s03 - s12;
    r[3] = d03 - 2 * d12;
  }
  for (int x = 0; x < 4; ++x) {
    int c0 = d[x], c1 = d[x + 4], c2 = d[x + 8], c3 = d[x + 12];
    int s03 = c0 + c3, d03 = c0 - c3, s12 = c1 + c2, d12 = c1 - c2;
    d[x] = s03 + s12;
    d[x + 4] = 2 * d03 + d12;
    d[x + 8] = s03 - s12;
    d[x + 12] = d03 - 2 * d12;
  }
}

// 4x4 Hadamard (unnormalised), raster in place: used for the I16x16 DC transform.
MIVC_HD void hadamard4x4(int* d) {
  for (int y = 0; y < 4; ++y) {
    int* r = d + 4 * y;
    int a = r[0] + r[1], b = r[2] + r[3], c = r[0] - r[1], e = r[2] - r[3];
    r[0] = a + b;
    r[1] = a - b;
    r[2] = c - e;
    r[3] = c + e;
  }
  for (int x = 0; x < 4; ++x) {
    int a = d[x] + d[x + 4], b = d[x + 8] + d[x + 12], c = d[x] - d[x + 4], e = d[x + 8] - d[x + 12];
    d[x] = a + b;
    d[x + 4] = a - b;
    d[x + 8] = c - e;
    d[x + 12] = c + e;
  }
}

// Quantise one coefficient: sign(w) * ((|w| * MF + f) >> qbits), f = bias * 2^qbits / 64
MIVC_HD int quant_coef(int w, int mf, int qbits, int bias64) {
  int a = w < 0 ? -w : w;
  int64_t f = (static_cast<int64_t>(1) << qbits) * bias64 / 64;
  int z = static_cast<int>((static_cast<int64_t>(a) * mf + f) >> qbits);
  return w < 0 ? -z : z;
}

// SATD of a 4x4 residual (sum |Hadamard| / 2), x264-style normalisation
MIVC_HD int satd4x4(const int* r) {
  int t[16];
  for (int i = 0; i < 16; ++i) t[i] = r[i];
  hadamard4x4(t);
  int s = 0;
  for (int i = 0; i < 16; ++i) s += t[i] < 0 ? -t[i] : t[i];
  return s >> 1;
}

// Approximate bit cost of an unsigned Exp-Golomb code
MIVC_HD int ue_bits(unsigned v) {
  unsigned x = v + 1;
  int n = 0;
  while (x > 1) {
    x >>= 1;
    ++n;
  }
  return 2 * n + 1;
}
MIVC_HD int se_bits(int v) { return ue_bits(v <= 0 ? static_cast<unsigned>(-2 * v) : static_cast<unsigned>(2 * v - 1)); }

// SATD-domain Lagrange multiplier, lambda(qp) = round(2^((qp-12)/6)) (x264 lambda_tab shape)
static constexpr uint16_t kLambda[52] = {
    1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 4, 4, 4, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 23, 25, 29, 32, 36, 40, 45, 51, 57, 64, 72, 81, 91};

}  // namespace h264
}  // namespace mivc
