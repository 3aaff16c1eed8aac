#include "lowres.h"

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <vector>

#include "../common/h264_enc_math.h"

namespace mivc {

namespace {

struct Low {
  int w, h;
  std::vector<uint8_t> p;
  int at(int x, int y) const {
    x = x < 0 ? 0 : (x >= w ? w - 1 : x);
    y = y < 0 ? 0 : (y >= h ? h - 1 : y);
    return p[static_cast<size_t>(y) * w + x];
  }
};

Low downscale(const uint8_t* y, int width, int height) {
  Low l;
  l.w = width / 2;
  l.h = height / 2;
  l.p.resize(static_cast<size_t>(l.w) * l.h);
  for (int j = 0; j < l.h; ++j)
    for (int i = 0; i < l.w; ++i) {
      const uint8_t* s = y + static_cast<size_t>(2 * j) * width + 2 * i;
      l.p[static_cast<size_t>(j) * l.w + i] = static_cast<uint8_t>((s[0] + s[1] + s[width] + s[width + 1] + 2) >> 2);
    }
  return l;
}

int satd8(const Low& cur, int x0, int y0, const int* pred) {
  int s = 0;
  for (int b = 0; b < 4; ++b) {
    int r[16];
    int bx = (b & 1) * 4, by = (b >> 1) * 4;
    for (int y = 0; y < 4; ++y)
      for (int x = 0; x < 4; ++x) r[y * 4 + x] = cur.at(x0 + bx + x, y0 + by + y) - pred[(by + y) * 8 + bx + x];
    s += h264::satd4x4(r);
  }
  return s;
}

int intra_cost(const Low& cur, int x0, int y0) {
  int top[8], left[8];
  bool has_top = y0 > 0, has_left = x0 > 0;
  int st = 0, sl = 0;
  for (int i = 0; i < 8; ++i) {
    top[i] = cur.at(x0 + i, y0 - 1);
    left[i] = cur.at(x0 - 1, y0 + i);
    st += top[i];
    sl += left[i];
  }
  int dc = has_top && has_left ? (st + sl + 8) >> 4 : has_top ? (st + 4) >> 3 : has_left ? (sl + 4) >> 3 : 128;
  int pred[64];
  int best = INT_MAX;
  for (int i = 0; i < 64; ++i) pred[i] = dc;
  best = std::min(best, satd8(cur, x0, y0, pred));
  if (has_top) {
    for (int i = 0; i < 64; ++i) pred[i] = top[i & 7];
    best = std::min(best, satd8(cur, x0, y0, pred));
  }
  if (has_left) {
    for (int i = 0; i < 64; ++i) pred[i] = left[i >> 3];
    best = std::min(best, satd8(cur, x0, y0, pred));
  }
  return best + 5;  // small mode-cost bias
}

int inter_cost(const Low& cur, const Low& ref, int x0, int y0) {
  auto sad = [&](int dx, int dy) {
    int s = 0;
    for (int y = 0; y < 8; ++y)
      for (int x = 0; x < 8; ++x) s += std::abs(cur.at(x0 + x, y0 + y) - ref.at(x0 + x + dx, y0 + y + dy));
    return s;
  };
  int bx = 0, by = 0, best = sad(0, 0);
  for (int it = 0; it < 16; ++it) {
    bool imp = false;
    static const int d[4][2] = {{1, 0}, {-1, 0}, {0, 1}, {0, -1}};
    for (auto& dd : d) {
      int cx = bx + dd[0], cy = by + dd[1];
      if (std::abs(cx) > 16 || std::abs(cy) > 16) continue;
      int c = sad(cx, cy);
      if (c < best) {
        best = c;
        bx = cx;
        by = cy;
        imp = true;
      }
    }
    if (!imp) break;
  }
  int pred[64];
  for (int y = 0; y < 8; ++y)
    for (int x = 0; x < 8; ++x) pred[y * 8 + x] = ref.at(x0 + x + bx, y0 + y + by);
  return satd8(cur, x0, y0, pred) + 2 * (std::abs(bx) + std::abs(by));
}

}  // namespace

void lowres_frame_costs(const uint8_t* frames, int width, int height, int nframes, float* intra, float* inter) {
  size_t fsize = static_cast<size_t>(width) * height * 3 / 2;
  Low prev;
  for (int f = 0; f < nframes; ++f) {
    Low cur = downscale(frames + f * fsize, width, height);
    double si = 0, sp = 0;
    for (int y0 = 0; y0 < cur.h; y0 += 8)
      for (int x0 = 0; x0 < cur.w; x0 += 8) {
        int ic = intra_cost(cur, x0, y0);
        si += ic;
        sp += f == 0 ? ic : std::min(ic, inter_cost(cur, prev, x0, y0));
      }
    intra[f] = static_cast<float>(si);
    inter[f] = static_cast<float>(sp);
    prev = std::move(cur);
  }
}

}  // namespace mivc
