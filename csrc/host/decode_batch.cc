#include "decode_batch.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <stdexcept>
#include <thread>

#include "../common/h264_mb.h"

namespace mivc {

H264Parsed h264_parse_segment(const std::string& s) {
  H264Parsed r;
  try {
    h264::Decoder dec;
    dec.set_parse_only(true);
    dec.decode(reinterpret_cast<const uint8_t*>(s.data()), s.size());
    dec.flush();
    r.pics = std::move(dec.out());
  } catch (const std::exception& e) {
    r.error = e.what();
  }
  return r;
}

template <class F>
static void parallel_for(size_t n, int threads, F&& f) {
  int nt = std::max(1, std::min<int>(threads, static_cast<int>(n)));
  if (nt == 1) {
    for (size_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::thread> pool;
  for (int t = 0; t < nt; ++t)
    pool.emplace_back([&] {
      for (size_t i = next++; i < n; i = next++) f(i);
    });
  for (std::thread& th : pool) th.join();
}

std::vector<H264Parsed> h264_parse_many(const std::vector<std::string>& segs, int threads) {
  std::vector<H264Parsed> res(segs.size());
  parallel_for(segs.size(), threads, [&](size_t i) { res[i] = h264_parse_segment(segs[i]); });
  return res;
}

static size_t align256(size_t v) { return (v + 255) & ~static_cast<size_t>(255); }

const h264::DecodedPicture* H264Batch::pic(int t, int seg) const {
  if (seg < 0) return nullptr;
  if (seg >= static_cast<int>(segs.size())) throw std::out_of_range("H264Batch: segment index");
  const H264Parsed& p = segs[seg];
  if (!p.error.empty() || t < 0 || t >= static_cast<int>(p.pics.size())) return nullptr;
  return &p.pics[t];
}

H264StepLayout H264Batch::layout(int t, const std::vector<int>& slots, int nmb) const {
  const size_t B = slots.size();
  size_t ncoef = 0, nsub = 0;
  for (size_t j = 0; j < B; ++j)
    if (const h264::DecodedPicture* d = pic(t, slots[j])) {
      if (d->blk_mask.size() != static_cast<size_t>(nmb)) throw std::runtime_error("H264Batch: picture size differs");
      ncoef += d->coef.size();
      nsub += d->sub.size();
    }
  H264StepLayout L;
  size_t o = 0;
  L.hdr = o;
  o = align256(o + B * nmb * sizeof(h264::MbHeader));
  L.mask = o;
  o = align256(o + B * nmb * 4);
  L.off = o;
  o = align256(o + B * nmb * 4);
  L.bs = o;
  o = align256(o + B * nmb * 16);
  L.wp = o;
  o = align256(o + B * h264::kWpEntries * 2);
  L.coef = o;
  o = align256(o + std::max<size_t>(ncoef, 16) * 2);
  L.sub = o;
  o = align256(o + std::max<size_t>(nsub, 16) * 2);
  L.total = o;
  return L;
}

void H264Batch::pack(int t, const std::vector<int>& slots, int nmb, uint8_t* dst, int threads) const {
  const H264StepLayout L = layout(t, slots, nmb);
  const size_t B = slots.size();
  // per-slot bases in the step's coef (units of 16 levels) and side-pool (entries) sections
  std::vector<size_t> cbase(B, 0), sbase(B, 0);
  size_t nc = 0, ns = 0;
  for (size_t j = 0; j < B; ++j) {
    cbase[j] = nc;
    sbase[j] = ns;
    if (const h264::DecodedPicture* d = pic(t, slots[j])) {
      nc += d->coef.size() / 16;
      ns += d->sub.size() / h264::kSubEntry;
    }
  }
  if (nc >= (1ull << 32) || ns >= (1ull << 32)) throw std::runtime_error("H264Batch: step too large for 32-bit offsets");
  parallel_for(B, threads, [&](size_t j) {
    const h264::DecodedPicture* d = pic(t, slots[j]);
    uint8_t* hdr = dst + L.hdr + j * nmb * sizeof(h264::MbHeader);
    uint32_t* mask = reinterpret_cast<uint32_t*>(dst + L.mask) + j * nmb;
    uint32_t* off = reinterpret_cast<uint32_t*>(dst + L.off) + j * nmb;
    uint8_t* bs = dst + L.bs + j * nmb * 16;
    int16_t* wp = reinterpret_cast<int16_t*>(dst + L.wp) + j * h264::kWpEntries;
    if (!d) {
      std::memset(hdr, 0, nmb * sizeof(h264::MbHeader));
      std::memset(mask, 0, nmb * 4);
      std::memset(off, 0, nmb * 4);
      std::memset(bs, 0, nmb * 16);
      std::memset(wp, 0, h264::kWpEntries * 2);
      return;
    }
    std::memcpy(hdr, d->hdr.data(), nmb * sizeof(h264::MbHeader));
    if (!d->sub.empty()) {
      const uint32_t sb = static_cast<uint32_t>(sbase[j]);
      for (int m = 0; m < nmb; ++m) {
        h264::MbHeader* h = reinterpret_cast<h264::MbHeader*>(hdr) + m;
        if (!(h->flags & h264::MBF_SUB4)) continue;
        uint32_t idx;
        std::memcpy(&idx, h->i4_modes, 4);
        idx += sb;
        std::memcpy(h->i4_modes, &idx, 4);
      }
      std::memcpy(reinterpret_cast<int16_t*>(dst + L.sub) + sbase[j] * h264::kSubEntry, d->sub.data(), d->sub.size() * 2);
    }
    std::memcpy(mask, d->blk_mask.data(), nmb * 4);
    const uint32_t cb = static_cast<uint32_t>(cbase[j]);
    for (int m = 0; m < nmb; ++m) off[m] = d->blk_off[m] + cb;
    if (d->bs.size() == static_cast<size_t>(nmb) * 16) std::memcpy(bs, d->bs.data(), nmb * 16);
    else std::memset(bs, 0, nmb * 16);
    if (d->wp.size() == static_cast<size_t>(h264::kWpEntries)) std::memcpy(wp, d->wp.data(), h264::kWpEntries * 2);
    else std::memset(wp, 0, h264::kWpEntries * 2);
    std::memcpy(reinterpret_cast<int16_t*>(dst + L.coef) + cbase[j] * 16, d->coef.data(), d->coef.size() * 2);
  });
}

}  // namespace mivc
