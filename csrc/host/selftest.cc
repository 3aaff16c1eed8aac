// Host-side consistency checks of encoder-side tables/helpers that the GPU kernels use.
#include <cstdint>
#include <random>

#include "../common/h264_i4_taps.h"
#include "../common/h264_pred.h"

namespace mivc {

// Compare the Intra4x4 tap table (used by the GPU intra kernel) against the direct
// clause-8.3.1.2 formulas for random neighbourhoods; returns the number of mismatches.
int selftest_i4_taps(int trials, uint32_t seed) {
  std::mt19937 rng(seed);
  int bad = 0;
  for (int t = 0; t < trials; ++t) {
    int e[13];
    for (int i = 0; i < 13; ++i) e[i] = static_cast<int>(rng() & 255);
    for (int mode = 0; mode < 9; ++mode) {
      if (mode == 2) continue;
      for (int p = 0; p < 16; ++p) {
        int x = p & 3, y = p >> 2;
        int a = h264::i4_pred_sample(mode, 15, e, x, y);
        int b = h264::i4_tap_sample(h264::kI4Taps[mode][p], e);
        bad += a != b;
      }
    }
  }
  return bad;
}

}  // namespace mivc
