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

// ---------------------------------------------------------------- HEVC
std::vector<HevcParsed> hevc_parse_many(const std::vector<std::string>& segs, int threads, bool recon) {
  std::vector<HevcParsed> res(segs.size());
  parallel_for(segs.size(), threads, [&](size_t i) {
    hevc::DecodeOptions o;
    o.recon = recon;
    o.gpu_records = true;
    res[i].dec.reset(new hevc::HevcStreamDecoder(o));
    try {
      res[i].dec->decode(reinterpret_cast<const uint8_t*>(segs[i].data()), segs[i].size());
      res[i].order = res[i].dec->output_order();
    } catch (const std::exception& e) {
      res[i].error = e.what();
    }
  });
  return res;
}

const hevc::DecPicture* HevcBatch::pic(int t, int seg) const {
  if (seg < 0) return nullptr;
  if (seg >= static_cast<int>(segs.size())) throw std::out_of_range("HevcBatch: segment index");
  const HevcParsed& p = segs[seg];
  if (!p.error.empty() || !p.dec || t < 0 || t >= static_cast<int>(p.dec->pictures().size())) return nullptr;
  return &p.dec->pictures()[t];
}

HevcStepLayout HevcBatch::layout(int t, const std::vector<int>& slots) const {
  const size_t B = slots.size();
  const hevc::DecPicture* g = nullptr;
  size_t ntu = 0, ncoef = 0, nop = 0, nref = 0, nsl = 0, nsub = 0;
  HevcStepLayout L;
  for (size_t j = 0; j < B && !g; ++j) g = pic(t, slots[j]);
  const size_t n4 = g ? static_cast<size_t>(g->W / 4) * (g->H / 4) : 0;
  const size_t n8 = n4 / 4;
  const size_t nctb = g ? static_cast<size_t>(g->wctb) * g->hctb : 0;
  for (size_t j = 0; j < B; ++j)
    if (const hevc::DecPicture* d = pic(t, slots[j])) {
      // validated here, before pack() fans out over threads
      if (d->W != g->W || d->H != g->H || d->log2_ctb != g->log2_ctb)
        throw std::runtime_error("HevcBatch: slots of one step differ in geometry");
      if (d->mvf.size() != n8 || d->bs.size() != n4 || d->ctbs.size() != nctb || d->sao.size() != nctb ||
          d->ops_off.size() != nctb + 1)
        throw std::runtime_error("HevcBatch: picture records do not match the step geometry");
      ntu += d->tus.size();
      ncoef += d->coefs.size();
      nop += d->ops.size();
      nref += d->refs.size();
      nsl += d->slices.size();
      nsub += d->mvf_sub.size();
      L.max_tus = std::max<int>(L.max_tus, static_cast<int>(d->tus.size()));
      L.scaling_on = L.scaling_on || !d->scaling.empty();
      L.deblock_any = L.deblock_any || d->deblock_any;
      L.sao_any = L.sao_any || d->sao_any;
    }
  size_t o = 0;
  auto sec = [&](size_t& at, size_t bytes) {
    at = o;
    o = align256(o + std::max<size_t>(bytes, 16));
  };
  sec(L.meta, B * 24 * 4);
  sec(L.tu_base, (B + 1) * 4);
  sec(L.coef_base, B * 8);
  sec(L.op_base, B * 4);
  sec(L.ref_base, B * 4);
  sec(L.slice_base, B * 4);
  sec(L.ctb_ops, B * (nctb + 1) * 4);
  sec(L.mvf, B * n8 * sizeof(hevc::DecMv4));
  sec(L.mvf_sub, nsub * sizeof(hevc::DecMv4));
  sec(L.bs, B * n4);
  sec(L.ctbs, B * nctb * sizeof(hevc::DecCtb));
  sec(L.sao, B * nctb * sizeof(hevc::DecSao));
  sec(L.tus, ntu * sizeof(hevc::DecTu));
  sec(L.coefs, ncoef * 2);
  sec(L.ops, nop * sizeof(hevc::DecIntraOp));
  sec(L.refs, nref * sizeof(hevc::DecRefEntry));
  sec(L.slices, nsl * sizeof(hevc::DecSlice));
  sec(L.scaling, L.scaling_on ? B * hevc::kScalingBytes : 0);
  L.total = o;
  return L;
}

void HevcBatch::pack(int t, const std::vector<int>& slots, uint8_t* dst, int threads) const {
  const HevcStepLayout L = layout(t, slots);
  const size_t B = slots.size();
  const hevc::DecPicture* g = nullptr;
  for (size_t j = 0; j < B && !g; ++j) g = pic(t, slots[j]);
  const size_t n4 = g ? static_cast<size_t>(g->W / 4) * (g->H / 4) : 0;
  const size_t n8 = n4 / 4;
  const size_t nctb = g ? static_cast<size_t>(g->wctb) * g->hctb : 0;
  std::vector<uint32_t> sub_base(B, 0);  // first mvf_sub entry (units of 4 records) of each slot
  // per-slot bases into the step's concatenated record sections
  int32_t* tu_base = reinterpret_cast<int32_t*>(dst + L.tu_base);
  int64_t* coef_base = reinterpret_cast<int64_t*>(dst + L.coef_base);
  int32_t* op_base = reinterpret_cast<int32_t*>(dst + L.op_base);
  int32_t* ref_base = reinterpret_cast<int32_t*>(dst + L.ref_base);
  int32_t* slice_base = reinterpret_cast<int32_t*>(dst + L.slice_base);
  int64_t ntu = 0, ncoef = 0, nop = 0, nref = 0, nsl = 0, nsub = 0;
  for (size_t j = 0; j < B; ++j) {
    sub_base[j] = static_cast<uint32_t>(nsub);
    tu_base[j] = static_cast<int32_t>(ntu);
    coef_base[j] = ncoef;
    op_base[j] = static_cast<int32_t>(nop);
    ref_base[j] = static_cast<int32_t>(nref);
    slice_base[j] = static_cast<int32_t>(nsl);
    if (const hevc::DecPicture* d = pic(t, slots[j])) {
      ntu += d->tus.size();
      ncoef += d->coefs.size();
      nop += d->ops.size();
      nref += d->refs.size();
      nsl += d->slices.size();
      nsub += d->mvf_sub.size() / 4;
    }
  }
  tu_base[B] = static_cast<int32_t>(ntu);
  if (ntu >= (1ll << 31) || nop >= (1ll << 31)) throw std::runtime_error("HevcBatch: step too large");
  parallel_for(B, threads, [&](size_t j) {
    const hevc::DecPicture* d = pic(t, slots[j]);
    int32_t* meta = reinterpret_cast<int32_t*>(dst + L.meta) + j * 24;
    uint32_t* cops = reinterpret_cast<uint32_t*>(dst + L.ctb_ops) + j * (nctb + 1);
    uint8_t* mvf = dst + L.mvf + j * n8 * sizeof(hevc::DecMv4);
    uint8_t* bs = dst + L.bs + j * n4;
    uint8_t* ctbs = dst + L.ctbs + j * nctb * sizeof(hevc::DecCtb);
    uint8_t* sao = dst + L.sao + j * nctb * sizeof(hevc::DecSao);
    uint8_t* scal = L.scaling_on ? dst + L.scaling + j * hevc::kScalingBytes : nullptr;
    if (!d) {
      std::memset(meta, 0, 24 * 4);
      std::memset(cops, 0, (nctb + 1) * 4);
      std::memset(mvf, 0, n8 * sizeof(hevc::DecMv4));
      std::memset(bs, 0, n4);
      std::memset(ctbs, 0, nctb * sizeof(hevc::DecCtb));
      std::memset(sao, 0, nctb * sizeof(hevc::DecSao));
      if (scal) std::memset(scal, 16, hevc::kScalingBytes);
      return;
    }
    const int v[24] = {d->decode_idx, d->poc, d->cvs, d->output, d->irap, d->idr, d->slice_type, d->slice_qp,
                       d->W, d->H, d->width, d->height, d->crop_x, d->crop_y, d->bit_depth, d->bit_depth_c,
                       d->log2_ctb, d->constrained_intra, d->strong_intra, d->lf_across_tiles, d->cb_qp_off,
                       d->cr_qp_off, d->deblock_any, d->sao_any};
    std::memcpy(meta, v, sizeof(v));
    std::memcpy(cops, d->ops_off.data(), (nctb + 1) * 4);
    std::memcpy(mvf, d->mvf.data(), n8 * sizeof(hevc::DecMv4));
    if (!d->mvf_sub.empty()) {  // split-block entries become global to the step
      hevc::DecMv4* m = reinterpret_cast<hevc::DecMv4*>(mvf);
      for (size_t k = 0; k < n8; ++k) {
        if (!(m[k].flags & hevc::DM_SPLIT)) continue;
        uint32_t idx;
        std::memcpy(&idx, m[k].mv, 4);
        idx += sub_base[j];
        std::memcpy(m[k].mv, &idx, 4);
      }
      std::memcpy(dst + L.mvf_sub + static_cast<size_t>(sub_base[j]) * 4 * sizeof(hevc::DecMv4), d->mvf_sub.data(),
                  d->mvf_sub.size() * sizeof(hevc::DecMv4));
    }
    std::memcpy(bs, d->bs.data(), n4);
    std::memcpy(ctbs, d->ctbs.data(), nctb * sizeof(hevc::DecCtb));
    std::memcpy(sao, d->sao.data(), nctb * sizeof(hevc::DecSao));
    if (scal) {
      if (d->scaling.size() == static_cast<size_t>(hevc::kScalingBytes)) std::memcpy(scal, d->scaling.data(), hevc::kScalingBytes);
      else std::memset(scal, 16, hevc::kScalingBytes);
    }
    std::memcpy(dst + L.tus + tu_base[j] * sizeof(hevc::DecTu), d->tus.data(), d->tus.size() * sizeof(hevc::DecTu));
    std::memcpy(dst + L.coefs + coef_base[j] * 2, d->coefs.data(), d->coefs.size() * 2);
    std::memcpy(dst + L.ops + op_base[j] * sizeof(hevc::DecIntraOp), d->ops.data(), d->ops.size() * sizeof(hevc::DecIntraOp));
    std::memcpy(dst + L.refs + ref_base[j] * sizeof(hevc::DecRefEntry), d->refs.data(),
                d->refs.size() * sizeof(hevc::DecRefEntry));
    std::memcpy(dst + L.slices + slice_base[j] * sizeof(hevc::DecSlice), d->slices.data(),
                d->slices.size() * sizeof(hevc::DecSlice));
  });
}

}  // namespace mivc
