// CPU micro-benchmark of the HEVC CABAC slice writer on records dumped from the GPU
// encoder (tools/dump_hevc_records.py).  Build (optionally with -pg for gprof):
//   g++ -O2 -std=c++17 -Icsrc tools/bench_hevc_writer.cc csrc/host/hevc_writer.cc \
//       csrc/host/bitstream.cc -o /tmp/bench_hevc_writer   (+ whatever the writer links)
//   /tmp/bench_hevc_writer DIR [reps]
#include <chrono>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "host/hevc_codec.h"

using namespace mivc::hevc;

template <class T>
static std::vector<T> load(const std::string& path) {
  std::ifstream f(path, std::ios::binary | std::ios::ate);
  const size_t n = static_cast<size_t>(f.tellg());
  f.seekg(0);
  std::vector<T> v(n / sizeof(T));
  f.read(reinterpret_cast<char*>(v.data()), static_cast<std::streamsize>(n));
  return v;
}

int main(int argc, char** argv) {
  const std::string dir = argv[1];
  const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
  std::ifstream meta(dir + "/meta.txt");
  std::string line;
  double total_ms = 0;
  size_t total_bytes = 0;
  unsigned long long total_bins = 0;
  unsigned long long hash = 1469598103934665603ull;
  int pics = 0, distinct = 0;
  double total_best_ms = 0;  // per picture: the fastest repetition (robust on a shared host)
  while (std::getline(meta, line)) {
    std::istringstream is(line);
    int i;
    HevcConfig c;
    HevcFrameParams fp;
    is >> i >> c.width >> c.height >> c.bit_depth >> c.sao >> c.deblock >> c.max_merge >> fp.idr >> fp.poc >> fp.qp >>
        fp.slice_type;
    const std::string p = dir + "/" + std::to_string(i) + "_";
    auto ctu = load<uint8_t>(p + "ctu.bin");
    auto cu = load<uint8_t>(p + "cu.bin");
    auto cy = load<int16_t>(p + "cy.bin");
    auto cb = load<int16_t>(p + "cb.bin");
    auto cr = load<int16_t>(p + "cr.bin");
    double best = 1e30;
    for (int r = 0; r < reps; ++r) {
      HevcSliceStats st;
      auto t0 = std::chrono::steady_clock::now();
      auto nal = hevc_write_slice(c, fp, reinterpret_cast<const CtuInfo*>(ctu.data()),
                                  reinterpret_cast<const CuInfo*>(cu.data()), cy.data(), cb.data(), cr.data(), &st);
      auto t1 = std::chrono::steady_clock::now();
      const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
      total_ms += ms;
      best = ms < best ? ms : best;
      total_bytes += nal.size();
      total_bins += st.bins;
      for (uint8_t b : nal) hash = (hash ^ b) * 1099511628211ull;
      ++pics;
    }
    total_best_ms += best;
    ++distinct;
  }
  std::printf("%d pictures, %.3f ms/picture (best of reps %.3f), %.1f KB/picture, %.0f bins/picture, hash %016llx\n",
              pics, total_ms / pics, total_best_ms / distinct,
              total_bytes / 1024.0 / pics, static_cast<double>(total_bins) / pics, hash);
  return 0;
}
