// Host H.264 parse throughput (the config-3 transcode's CPU stage) on real input pieces:
//   python tools/dump_4k_pieces.py 2            (on an MI355X: gpurun_out/pieces/p{0,1}.264)
//   g++ -O2 -std=c++17 -I csrc tools/bench_h264_parse.cc $(ls csrc/host/*.cc | grep -v bindings) \
//       -lpthread -o /tmp/bench_h264_parse && /tmp/bench_h264_parse gpurun_out/pieces/p0.264 ...
// Best of 6 single-threaded parses per file (the machine is shared), plus an FNV hash of every
// record the GPU path consumes (headers, levels, masks, offsets, boundary strengths, motion):
// parser changes must keep the hash.
#include <chrono>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>

#include "host/decode_batch.h"

static unsigned long long fnv(const void* p, size_t n, unsigned long long h) {
  const unsigned char* c = static_cast<const unsigned char*>(p);
  for (size_t i = 0; i < n; ++i) {
    h ^= c[i];
    h *= 1099511628211ull;
  }
  return h;
}

int main(int argc, char** argv) {
  unsigned long long h = 1469598103934665603ull;
  for (int a = 1; a < argc; ++a) {
    std::ifstream f(argv[a], std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string seg = ss.str();
    double best = 1e9;
    size_t pics = 0;
    for (int i = 0; i < 6; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      auto r = mivc::h264_parse_segment(seg);
      const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (!r.error.empty()) std::printf("%s: error %s\n", argv[a], r.error.c_str());
      best = dt < best ? dt : best;
      pics = r.pics.size();
      if (i == 0)
        for (auto& p : r.pics) {
          h = fnv(p.hdr.data(), p.hdr.size(), h);
          h = fnv(p.coef.data(), p.coef.size() * 2, h);
          h = fnv(p.blk_mask.data(), p.blk_mask.size() * 4, h);
          h = fnv(p.blk_off.data(), p.blk_off.size() * 4, h);
          h = fnv(p.bs.data(), p.bs.size(), h);
          h = fnv(p.sub.data(), p.sub.size() * 2, h);
          h = fnv(p.mv.data(), p.mv.size() * 2, h);
          h = fnv(p.ref.data(), p.ref.size(), h);
        }
    }
    std::printf("%s: %zu pictures, best %.1f ms (%.1f pictures/s per thread)\n", argv[a], pics, best * 1e3,
                pics / best);
  }
  std::printf("records hash %016llx\n", h);
  return 0;
}
