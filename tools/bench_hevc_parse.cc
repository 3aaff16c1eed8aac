// Host HEVC parse throughput (config 3's HEVC-input CPU stage) on real input pieces:
//   python tools/dump_4k_pieces.py 1            (on an MI355X: gpurun_out/pieces/p0.265)
//   g++ -O2 -std=c++17 -I csrc tools/bench_hevc_parse.cc $(ls csrc/host/*.cc | grep -v bindings) \
//       -lpthread -o /tmp/bench_hevc_parse && /tmp/bench_hevc_parse gpurun_out/pieces/p0.265 ...
// Best of 6 single-threaded parse-only decodes per file (recon off, GPU records on, exactly what
// hevc_parse_many runs), plus an FNV hash of every record the GPU path consumes: parser changes
// must keep the hash.
#include <chrono>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>

#include "host/decode_batch.h"

template <class T>
static unsigned long long fnv(const std::vector<T>& v, unsigned long long h) {
  const unsigned char* c = reinterpret_cast<const unsigned char*>(v.data());
  for (size_t i = 0; i < v.size() * sizeof(T); ++i) {
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
    const std::vector<std::string> segs{ss.str()};
    double best = 1e9;
    size_t pics = 0;
    for (int i = 0; i < 6; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      auto r = mivc::hevc_parse_many(segs, 1, false);
      const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (!r[0].error.empty()) std::printf("%s: error %s\n", argv[a], r[0].error.c_str());
      best = dt < best ? dt : best;
      auto& ps = r[0].dec->pictures();
      pics = ps.size();
      if (i == 0)
        for (auto& p : ps) {
          h = fnv(p.mvf, h);
          h = fnv(p.mvf_sub, h);
          h = fnv(p.bs, h);
          h = fnv(p.tus, h);
          h = fnv(p.coefs, h);
          h = fnv(p.ops, h);
          h = fnv(p.ops_off, h);
          h = fnv(p.ctbs, h);
          h = fnv(p.sao, h);
        }
    }
    std::printf("%s: %zu pictures, best %.1f ms (%.1f pictures/s per thread)\n", argv[a], pics, best * 1e3,
                pics / best);
  }
  std::printf("records hash %016llx\n", h);
  return 0;
}
