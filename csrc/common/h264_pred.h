// Encoder-side intra predictors (clause 8.3) and quarter-sample motion
// compensation (clause 8.4.2.2), host + device.  Independent of the decoder's
// implementation in h264_decoder.cc.
#pragma once
#include <cstdint>

#include "h264_tables.h"

namespace mivc {
namespace h264 {

// Availability bits
enum : int { AV_LEFT = 1, AV_TOP = 2, AV_TOPLEFT = 4, AV_TOPRIGHT = 8 };

// Which Intra4x4 modes can be used with the given neighbour availability
MIVC_HD bool i4_mode_ok(int mode, int av) {
  switch (mode) {
    case 0: case 3: case 7: return (av & AV_TOP) != 0;
    case 1: case 8: return (av & AV_LEFT) != 0;
    case 2: return true;
    default: return (av & (AV_TOP | AV_LEFT | AV_TOPLEFT)) == (AV_TOP | AV_LEFT | AV_TOPLEFT);
  }
}
MIVC_HD bool i16_mode_ok(int mode, int av) {  // 0 V, 1 H, 2 DC, 3 Plane
  switch (mode) {
    case 0: return (av & AV_TOP) != 0;
    case 1: return (av & AV_LEFT) != 0;
    case 2: return true;
    default: return (av & (AV_TOP | AV_LEFT | AV_TOPLEFT)) == (AV_TOP | AV_LEFT | AV_TOPLEFT);
  }
}
MIVC_HD bool chroma_mode_ok(int mode, int av) {  // 0 DC, 1 H, 2 V, 3 Plane
  switch (mode) {
    case 0: return true;
    case 1: return (av & AV_LEFT) != 0;
    case 2: return (av & AV_TOP) != 0;
    default: return (av & (AV_TOP | AV_LEFT | AV_TOPLEFT)) == (AV_TOP | AV_LEFT | AV_TOPLEFT);
  }
}

// e[0] = p[-1,-1], e[1..8] = p[0..7,-1] (top + top-right, already substituted), e[9..12] = p[-1,0..3]
MIVC_HD int i4_pred_sample(int mode, int av, const int* e, int x, int y) {
  const int* T = e + 1;   // T[-1] == top-left
  const int* L = e + 9;
  auto l = [&](int i) { return i < 0 ? e[0] : L[i]; };
  switch (mode) {
    case 0: return T[x];
    case 1: return L[y];
    case 2: {
      int s = 0;
      if ((av & AV_TOP) && (av & AV_LEFT)) {
        for (int i = 0; i < 4; ++i) s += T[i] + L[i];
        return (s + 4) >> 3;
      }
      if (av & AV_LEFT) {
        for (int i = 0; i < 4; ++i) s += L[i];
        return (s + 2) >> 2;
      }
      if (av & AV_TOP) {
        for (int i = 0; i < 4; ++i) s += T[i];
        return (s + 2) >> 2;
      }
      return 128;
    }
    case 3:
      if (x == 3 && y == 3) return (T[6] + 3 * T[7] + 2) >> 2;
      return (T[x + y] + 2 * T[x + y + 1] + T[x + y + 2] + 2) >> 2;
    case 4:
      if (x > y) return (T[x - y - 2] + 2 * T[x - y - 1] + T[x - y] + 2) >> 2;
      if (x < y) return (l(y - x - 2) + 2 * l(y - x - 1) + l(y - x) + 2) >> 2;
      return (T[0] + 2 * e[0] + L[0] + 2) >> 2;
    case 5: {
      int z = 2 * x - y;
      if (z >= 0 && !(z & 1)) return (T[x - (y >> 1) - 1] + T[x - (y >> 1)] + 1) >> 1;
      if (z >= 0) return (T[x - (y >> 1) - 2] + 2 * T[x - (y >> 1) - 1] + T[x - (y >> 1)] + 2) >> 2;
      if (z == -1) return (L[0] + 2 * e[0] + T[0] + 2) >> 2;
      return (l(y - 1) + 2 * l(y - 2) + l(y - 3) + 2) >> 2;
    }
    case 6: {
      int z = 2 * y - x;
      if (z >= 0 && !(z & 1)) return (l(y - (x >> 1) - 1) + l(y - (x >> 1)) + 1) >> 1;
      if (z >= 0) return (l(y - (x >> 1) - 2) + 2 * l(y - (x >> 1) - 1) + l(y - (x >> 1)) + 2) >> 2;
      if (z == -1) return (L[0] + 2 * e[0] + T[0] + 2) >> 2;
      return (T[x - 1] + 2 * T[x - 2] + T[x - 3] + 2) >> 2;
    }
    case 7:
      if (!(y & 1)) return (T[x + (y >> 1)] + T[x + (y >> 1) + 1] + 1) >> 1;
      return (T[x + (y >> 1)] + 2 * T[x + (y >> 1) + 1] + T[x + (y >> 1) + 2] + 2) >> 2;
    default: {
      int z = x + 2 * y;
      if (z < 5 && !(z & 1)) return (L[y + (x >> 1)] + L[y + (x >> 1) + 1] + 1) >> 1;
      if (z < 5) return (L[y + (x >> 1)] + 2 * L[y + (x >> 1) + 1] + L[y + (x >> 1) + 2] + 2) >> 2;
      if (z == 5) return (L[2] + 3 * L[3] + 2) >> 2;
      return L[3];
    }
  }
}

// 16x16 luma: top[16], left[16], tl.  Plane parameters precomputed by the caller via i16_plane_params.
template <class T>
MIVC_HD void i16_plane_params(const T* top, const T* left, int tl, int* a, int* b, int* c) {
  int H = 0, V = 0;
  for (int i = 0; i < 8; ++i) {
    H += (i + 1) * (top[8 + i] - (i == 7 ? tl : top[6 - i]));
    V += (i + 1) * (left[8 + i] - (i == 7 ? tl : left[6 - i]));
  }
  *a = 16 * (left[15] + top[15]);
  *b = (5 * H + 32) >> 6;
  *c = (5 * V + 32) >> 6;
}
template <class T>
MIVC_HD int i16_dc(const T* top, const T* left, int av) {
  int st = 0, sl = 0;
  for (int i = 0; i < 16; ++i) {
    st += top[i];
    sl += left[i];
  }
  if ((av & AV_TOP) && (av & AV_LEFT)) return (st + sl + 16) >> 5;
  if (av & AV_LEFT) return (sl + 8) >> 4;
  if (av & AV_TOP) return (st + 8) >> 4;
  return 128;
}

// chroma 8x8 (4:2:0) DC for 4x4 block (bx,by)
template <class T>
MIVC_HD int chroma_dc(const T* top, const T* left, int av, int bx, int by) {
  int st = 0, sl = 0;
  for (int i = 0; i < 4; ++i) {
    st += top[bx * 4 + i];
    sl += left[by * 4 + i];
  }
  bool t = (av & AV_TOP) != 0, l = (av & AV_LEFT) != 0;
  if ((bx == 0 && by == 0) || (bx == 1 && by == 1)) {
    if (t && l) return (st + sl + 4) >> 3;
    if (l) return (sl + 2) >> 2;
    if (t) return (st + 2) >> 2;
    return 128;
  }
  if (bx == 1) {  // top-right block
    if (t) return (st + 2) >> 2;
    if (l) return (sl + 2) >> 2;
    return 128;
  }
  if (l) return (sl + 2) >> 2;  // bottom-left block
  if (t) return (st + 2) >> 2;
  return 128;
}
template <class T>
MIVC_HD void chroma_plane_params(const T* top, const T* left, int tl, int* a, int* b, int* c) {
  int H = 0, V = 0;
  for (int i = 0; i < 4; ++i) {
    H += (i + 1) * (top[4 + i] - (i == 3 ? tl : top[2 - i]));
    V += (i + 1) * (left[4 + i] - (i == 3 ? tl : left[2 - i]));
  }
  *a = 16 * (left[7] + top[7]);
  *b = (34 * H + 32) >> 6;
  *c = (34 * V + 32) >> 6;
}

// ---------------------------------------------------------------- motion compensation
// Quarter-sample luma interpolation at integer position (xi,yi) + fraction (xf,yf),
// reading the reference through clamped coordinates.  P must provide int operator()(x,y).
template <class P>
MIVC_HD int mc_luma_sample(const P& ref, int xi, int yi, int xf, int yf) {
  auto b1 = [&](int x, int y) {
    return tap6(ref(x - 2, y), ref(x - 1, y), ref(x, y), ref(x + 1, y), ref(x + 2, y), ref(x + 3, y));
  };
  auto h1 = [&](int x, int y) {
    return tap6(ref(x, y - 2), ref(x, y - 1), ref(x, y), ref(x, y + 1), ref(x, y + 2), ref(x, y + 3));
  };
  auto B = [&](int x, int y) { return clip1((b1(x, y) + 16) >> 5); };
  auto Hh = [&](int x, int y) { return clip1((h1(x, y) + 16) >> 5); };
  auto J = [&](int x, int y) {
    int j1 = tap6(h1(x - 2, y), h1(x - 1, y), h1(x, y), h1(x + 1, y), h1(x + 2, y), h1(x + 3, y));
    return clip1((j1 + 512) >> 10);
  };
  if (xf == 0 && yf == 0) return ref(xi, yi);
  if (yf == 0) {
    int b = B(xi, yi);
    if (xf == 1) return (ref(xi, yi) + b + 1) >> 1;
    if (xf == 2) return b;
    return (ref(xi + 1, yi) + b + 1) >> 1;
  }
  if (xf == 0) {
    int h = Hh(xi, yi);
    if (yf == 1) return (ref(xi, yi) + h + 1) >> 1;
    if (yf == 2) return h;
    return (ref(xi, yi + 1) + h + 1) >> 1;
  }
  if (xf == 2 && yf == 2) return J(xi, yi);
  if (xf == 2) {  // f (yf=1) or q (yf=3)
    int j = J(xi, yi);
    int b = yf == 1 ? B(xi, yi) : B(xi, yi + 1);
    return (b + j + 1) >> 1;
  }
  if (yf == 2) {  // i (xf=1) or k (xf=3)
    int j = J(xi, yi);
    int h = xf == 1 ? Hh(xi, yi) : Hh(xi + 1, yi);
    return (h + j + 1) >> 1;
  }
  // diagonal quarter positions e, g, p, r: average of the two nearest half samples
  int b = yf == 1 ? B(xi, yi) : B(xi, yi + 1);
  int h = xf == 1 ? Hh(xi, yi) : Hh(xi + 1, yi);
  return (b + h + 1) >> 1;
}

template <class P>
MIVC_HD int mc_chroma_sample(const P& ref, int xi, int yi, int xf, int yf) {
  return ((8 - xf) * (8 - yf) * ref(xi, yi) + xf * (8 - yf) * ref(xi + 1, yi) + (8 - xf) * yf * ref(xi, yi + 1) +
          xf * yf * ref(xi + 1, yi + 1) + 32) >>
         6;
}

}  // namespace h264
}  // namespace mivc
