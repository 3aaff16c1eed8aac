// CPU benchmark / gprof harness of the HEVC CABAC slice writer on a whole GOP's records dumped
// from the GPU encoder (tools/dump_hevc_gop_records.py: B pictures, TMVP, several list-0
// pictures, CTU 64, WPP, AQ -- the default tool set):
//   g++ -O3 -std=c++17 -Icsrc tools/bench_hevc_writer_gop.cc $(ls csrc/host/*.cc | grep -v bindings) \
//       -lpthread -o /tmp/bench_hevc_writer_gop   (add -pg for gprof)
//   /tmp/bench_hevc_writer_gop DIR [reps]
// Single-threaded (threads = 1), best of reps per slice; prints ms per picture and an FNV hash
// of every slice NAL (writer changes must keep it).
#include <chrono>
#include <cstdio>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "host/hevc_codec.h"

using namespace mivc::hevc;

template <class T>
static std::vector<T> load(const std::string& path) {
  std::ifstream f(path, std::ios::binary | std::ios::ate);
  if (!f) throw std::runtime_error("missing " + path);
  const size_t n = static_cast<size_t>(f.tellg());
  f.seekg(0);
  std::vector<T> v(n / sizeof(T));
  f.read(reinterpret_cast<char*>(v.data()), static_cast<std::streamsize>(n));
  return v;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s DIR [reps]\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const int reps = argc > 2 ? std::atoi(argv[2]) : 3;
  std::ifstream meta(dir + "/meta.txt");
  std::string line;
  std::map<int, std::vector<uint8_t>> cus;  // slice -> CU records (collocated pictures)
  double total_best = 0;
  size_t bytes = 0;
  unsigned long long bins = 0, hash = 1469598103934665603ull;
  int n = 0;
  while (std::getline(meta, line)) {
    std::istringstream is(line);
    int idx;
    is >> idx;
    HevcConfig c;
    HevcFrameParams fp;
    int col = -1;
    bool col_given[2] = {false, false};
    std::vector<int> col_l[2];
    std::string k;
    while (is >> k) {
      auto list = [&](std::vector<int>& v) {
        int m;
        is >> m;
        v.resize(m);
        for (int& x : v) is >> x;
      };
      int v = 0;
      if (k == "rps") {
        int m;
        is >> m;
        fp.n_rps = m;
        for (int i = 0; i < m; ++i) {
          int p, u;
          is >> p >> u;
          fp.rps_poc[i] = p;
          fp.rps_used[i] = static_cast<uint8_t>(u);
        }
        continue;
      }
      if (k == "refs0" || k == "refs1" || k == "col_refs0" || k == "col_refs1" || k == "wp") {
        std::vector<int> l;
        list(l);
        if (k == "wp") {
          fp.wp = 1;
          for (int ci = 0; ci < 3; ++ci) {
            fp.wp_w[ci] = l[2 * ci];
            fp.wp_o[ci] = l[2 * ci + 1];
          }
        } else if (k == "refs0" || k == "refs1") {
          const int L = k == "refs1";
          fp.num_ref[L] = static_cast<int>(l.size());
          for (size_t i = 0; i < l.size(); ++i) fp.list_poc[L][i] = l[i];
        } else {
          const int L = k == "col_refs1";
          col_given[L] = true;
          col_l[L] = l;
        }
        continue;
      }
      is >> v;
      if (k == "width") c.width = v;
      else if (k == "height") c.height = v;
      else if (k == "bit_depth") c.bit_depth = v;
      else if (k == "sao") c.sao = v;
      else if (k == "deblock") c.deblock = v;
      else if (k == "max_merge") c.max_merge = v;
      else if (k == "wpp") c.wpp = v;
      else if (k == "cu_qp_delta") c.cu_qp_delta = v;
      else if (k == "tu_inter_depth") c.tu_inter_depth = v;
      else if (k == "sdh") c.sdh = v;
      else if (k == "level_idc") c.level_idc = v;
      else if (k == "bframes") c.bframes = v;
      else if (k == "tmvp") c.tmvp = v;
      else if (k == "pyramid") c.pyramid = v;
      else if (k == "ctu64") c.ctu64 = v;
      else if (k == "weightp") c.weightp = v;
      else if (k == "refs") c.refs = v;
      else if (k == "idr") fp.idr = v;
      else if (k == "poc") fp.poc = v;
      else if (k == "qp") fp.qp = v;
      else if (k == "slice_type") fp.slice_type = v;
      else if (k == "nal_ref") fp.nal_ref = v;
      else if (k == "ref_poc0") fp.ref_poc[0] = v;
      else if (k == "ref_poc1") fp.ref_poc[1] = v;
      else if (k == "col_poc") { fp.col.set = 1; fp.col.poc = v; }
      else if (k == "col_ref_poc0") fp.col.ref_poc[0] = v;
      else if (k == "col_ref_poc1") fp.col.ref_poc[1] = v;
      else if (k == "col_cu") col = v;
    }
    for (int L = 0; L < 2; ++L)  // as the bindings: entries past a given list repeat ref_poc[L]
      for (int i = 0; i < kMaxRefs; ++i)
        fp.col.list_poc[L][i] = col_given[L] && i < static_cast<int>(col_l[L].size()) ? col_l[L][i] : fp.col.ref_poc[L];
    const std::string p = dir + "/" + std::to_string(idx) + "_";
    auto ctu = load<uint8_t>(p + "ctu.bin");
    cus[idx] = load<uint8_t>(p + "cu.bin");
    auto nz = load<uint64_t>(p + "nz.bin");
    auto off = load<uint32_t>(p + "off.bin");
    auto lv = load<int16_t>(p + "lv.bin");
    if (col >= 0) fp.col.cu = reinterpret_cast<const CuInfo*>(cus.at(col).data());
    PackedLevels pk;
    pk.nzmap = nz.data();
    pk.ctb_off = off.data();
    pk.levels = lv.data();
    pk.nblocks = lv.size() / 16;
    c.threads = 1;
    double best = 1e30;
    for (int r = 0; r < reps; ++r) {
      HevcSliceStats st;
      const auto t0 = std::chrono::steady_clock::now();
      auto nal = hevc_write_slice(c, fp, reinterpret_cast<const CtuInfo*>(ctu.data()),
                                  reinterpret_cast<const CuInfo*>(cus[idx].data()), nullptr, nullptr, nullptr, &st, &pk);
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      best = ms < best ? ms : best;
      if (r == 0) {
        bytes += nal.size();
        bins += st.bins;
        for (uint8_t b : nal) hash = (hash ^ b) * 1099511628211ull;
      }
    }
    total_best += best;
    ++n;
  }
  std::printf("%d slices, %.3f ms/picture (best of %d), %.1f KB/picture, %.0f bins/picture, hash %016llx\n", n,
              total_best / n, reps, bytes / 1024.0 / n, static_cast<double>(bins) / n, hash);
  return 0;
}
