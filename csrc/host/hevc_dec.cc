// General HEVC Main / Main 10 decoder (see hevc_dec.h): slice data parsing (7.3.8),
// CABAC (9.3), motion vector prediction (8.5.3.2), CPU reconstruction (8.4, 8.5, 8.6),
// in-loop filters (8.7) and the GPU hand-off records.
#include "hevc_dec.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>

#include "hevc_ctx_tables.h"
#include "hevc_dec_ps.h"

namespace mivc {
namespace hevc {

using namespace dec;

namespace {

inline int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
inline int sgn(int v) { return (v > 0) - (v < 0); }

// renormalisation shift of an LPS range (ranges 6..255, indexed by range >> 3)
struct RenormTable {
  uint8_t t[32];
  constexpr RenormTable() : t() {
    for (int i = 0; i < 32; ++i) {
      int r = i << 3, n = 0;
      if (r == 0) r = 6;
      while ((r << n) < 256) ++n;
      t[i] = static_cast<uint8_t>(n);
    }
  }
};
constexpr RenormTable kRenorm{};

// scan orders (6.5.3-6.5.5) of every (scanIdx, log2 size 0..3) as position tables, and their
// inverse (raster position -> scan index): residual_coding looks positions up instead of
// walking the diagonal per coefficient (scan_pos is O(p))
struct ScanTables {
  uint8_t x[3][4][64], y[3][4][64], inv[3][4][64];
  ScanTables() : x(), y(), inv() {
    for (int s = 0; s < 3; ++s)
      for (int l = 0; l < 4; ++l)
        for (int p = 0; p < (1 << (2 * l)); ++p) {
          const int v = scan_pos(s, l, p);
          x[s][l][p] = static_cast<uint8_t>(v & 255);
          y[s][l][p] = static_cast<uint8_t>(v >> 8);
          inv[s][l][((v >> 8) << l) + (v & 255)] = static_cast<uint8_t>(p);
        }
  }
};
const ScanTables kScan;

// CABAC arithmetic decoding engine (9.3.4.3), byte-refilled: `value` holds the 9-bit
// offset scaled by 2^7 plus look-ahead bits.  After a terminating bin equal to 1 the
// next byte-aligned syntax (PCM samples, the next substream) starts at `p`.
class Engine {
 public:
  void start(const uint8_t* p, const uint8_t* end) {
    p_ = p;
    end_ = end;
    range_ = 510;
    bits_needed_ = -8;
    value_ = (byte() << 8) | byte();
  }
  int decode(CtxS& c) {
    const uint32_t lps = kRangeLps[c.state][(range_ >> 6) - 4];
    range_ -= lps;
    const uint32_t scaled = range_ << 7;
    int bin;
    if (value_ < scaled) {
      bin = c.mps;
      if (c.state < 62) ++c.state;
      if (scaled < (256u << 7)) {
        range_ = scaled >> 6;
        value_ <<= 1;
        if (++bits_needed_ == 0) {
          bits_needed_ = -8;
          value_ |= byte();
        }
      }
    } else {
      const int nb = kRenorm.t[lps >> 3];
      value_ = (value_ - scaled) << nb;
      range_ = lps << nb;
      bin = 1 - c.mps;
      if (c.state == 0) c.mps = static_cast<uint8_t>(1 - c.mps);
      c.state = kTransIdxLps[c.state];
      bits_needed_ += nb;
      if (bits_needed_ >= 0) {
        value_ |= byte() << bits_needed_;
        bits_needed_ -= 8;
      }
    }
    return bin;
  }
  int bypass() {
    value_ <<= 1;
    if (++bits_needed_ >= 0) {
      bits_needed_ = -8;
      value_ |= byte();
    }
    const uint32_t scaled = range_ << 7;
    if (value_ >= scaled) {
      value_ -= scaled;
      return 1;
    }
    return 0;
  }
  uint32_t bypass_bits(int n) {
    uint32_t v = 0;
    for (int i = 0; i < n; ++i) v = (v << 1) | static_cast<uint32_t>(bypass());
    return v;
  }
  int terminate() {
    range_ -= 2;
    const uint32_t scaled = range_ << 7;
    if (value_ >= scaled) return 1;
    if (scaled < (256u << 7)) {
      range_ = scaled >> 6;
      value_ <<= 1;
      if (++bits_needed_ == 0) {
        bits_needed_ = -8;
        value_ |= byte();
      }
    }
    return 0;
  }
  const uint8_t* pos() const { return p_; }
  const uint8_t* end() const { return end_; }

 private:
  uint32_t byte() {
    if (p_ >= end_) {
      if (++over_ > 16) fail("CABAC read past the end of the slice data");
      return 0;
    }
    return *p_++;
  }
  const uint8_t* p_ = nullptr;
  const uint8_t* end_ = nullptr;
  uint32_t range_ = 510, value_ = 0;
  int bits_needed_ = -8;
  int over_ = 0;
};

// raw bit reader for PCM samples at a byte position
struct RawBits {
  const uint8_t* p;
  const uint8_t* end;
  int bit = 0;
  uint32_t get(int n) {
    uint32_t v = 0;
    for (int i = 0; i < n; ++i) {
      if (p >= end) fail("PCM samples past the end of the slice data");
      v = (v << 1) | ((*p >> (7 - bit)) & 1u);
      if (++bit == 8) {
        bit = 0;
        ++p;
      }
    }
    return v;
  }
};

const int kLumaTaps[4][8] = {{0, 0, 0, 64, 0, 0, 0, 0},
                             {-1, 4, -10, 58, 17, -5, 1, 0},
                             {-1, 4, -11, 40, 40, -11, 4, -1},
                             {0, 1, -5, 17, 58, -10, 4, -1}};
const int kChromaTaps[8][4] = {{0, 64, 0, 0},    {-2, 58, 10, -2}, {-4, 54, 16, -2}, {-6, 46, 28, -4},
                               {-4, 36, 36, -4}, {-4, 28, 46, -6}, {-2, 16, 54, -4}, {-2, 10, 58, -2}};

// z-order of a 4x4 block (bx, by) inside a CTB of 2^l4 x 2^l4 blocks
inline uint32_t zorder(int bx, int by) {
  // interleave the 4 low bits of bx (even bit positions) and by (odd)
  auto spread = [](uint32_t v) {
    v &= 15u;
    v = (v | (v << 2)) & 0x33u;
    return (v | (v << 1)) & 0x55u;
  };
  return spread(static_cast<uint32_t>(bx)) | (spread(static_cast<uint32_t>(by)) << 1);
}

enum PartMode { P_2Nx2N = 0, P_2NxN, P_Nx2N, P_NxN, P_2NxnU, P_2NxnD, P_nLx2N, P_nRx2N };

struct MvField {
  int16_t mv[2][2];
  int8_t ref[2];
  uint8_t pred;  // bit 0: L0, bit 1: L1 (0: intra / not inter)
  uint8_t pad;
};

inline bool same_motion(const MvField& a, const MvField& b) {
  if (a.pred != b.pred) return false;
  for (int l = 0; l < 2; ++l)
    if (a.pred & (1 << l))
      if (a.ref[l] != b.ref[l] || a.mv[l][0] != b.mv[l][0] || a.mv[l][1] != b.mv[l][1]) return false;
  return true;
}

// per-slice reference lists as decoded (POCs + long-term marking), kept with a picture for
// the TMVP of later pictures (LongTermRefPic of the collocated picture)
struct SliceRefs {
  int n[2] = {0, 0};
  int poc[2][16] = {};
  uint8_t lt[2][16] = {};
  int pic[2][16] = {};  // decode_idx
};

struct StoredPic {
  int decode_idx = 0, poc = 0, cvs = 0;
  bool is_ref = true, is_lt = false;
  int W = 0, H = 0, w4 = 0, h4 = 0, log2_ctb = 4, wctb = 0;
  std::vector<uint16_t> pl[3];   // CPU reconstruction
  std::vector<MvField> mvf;      // per 4x4
  std::vector<uint16_t> ctb_slice;
  std::vector<SliceRefs> slices;
};

}  // namespace

// ======================================================================================
struct HevcStreamDecoder::Impl {
  DecodeOptions opt;
  std::vector<DecPicture>* out = nullptr;
  std::shared_ptr<Sps> sps_tab[16];
  std::shared_ptr<Pps> pps_tab[64];
  // the active parameter sets stay alive while a later NAL replaces a table entry
  std::shared_ptr<Sps> sps_hold;
  std::shared_ptr<Pps> pps_hold;
  const Sps* sps = nullptr;
  const Pps* pps = nullptr;

  // ---- sequence state
  int cvs = -1;
  bool first_pic = true, after_eos = false;
  int prev_tid0_poc = 0;
  bool no_rasl_output = true;
  std::vector<std::shared_ptr<StoredPic>> dpb;
  int decode_count = 0;

  // ---- current picture
  std::shared_ptr<StoredPic> cur;
  DecPicture* dp = nullptr;
  bool pic_open = false;
  int nal_type = 0, poc = 0;
  SliceHeader sh;
  bool have_indep = false;
  SliceHeader indep;             // last independent slice segment header of the picture
  int slice_idx = -1;
  int slice_addr_rs = 0;
  std::vector<SliceHeader> slices;  // per slice segment of the picture (index = slice_idx)
  StoredPic* ref_list[2][16] = {};
  int ref_poc[2][16] = {};
  bool ref_lt[2][16] = {};
  int ref_entry_base[2] = {0, 0};   // GPU refs table base of the current slice
  bool nobackward = true;
  int slice_qp = 26, init_type = 0;

  // picture geometry
  int W = 0, H = 0, bd = 8, bdc = 8, maxv = 255, maxvc = 255, log2_ctb = 4, ctb = 16, wctb = 0, hctb = 0, nctb = 0;
  int w4 = 0, h4 = 0, l4 = 2;  // l4: log2 of 4x4 blocks per CTB side
  int log2_min_cb = 3, log2_min_tb = 2, log2_max_tb = 5;
  std::vector<int> rs2ts, ts2rs, tile_id, col_bd, row_bd;

  // per 4x4
  std::vector<uint8_t> cu_flags;  // CF_* bits
  std::vector<uint8_t> ct_depth, ipm, edge, cbf_y;
  std::vector<int8_t> qp_y;
  std::vector<int16_t> ctb_slice;  // per CTB (raster): slice_idx or -1 (not decoded)
  std::vector<int32_t> ctb_saddr;  // per CTB (raster): SliceAddrRs of its slice
  enum : uint8_t { CF_INTRA = 1, CF_SKIP = 2, CF_PCM = 4, CF_BYPASS = 8, CF_INTER = 16 };
  enum : uint8_t { E_TU_V = 1, E_PU_V = 2, E_TU_H = 4, E_PU_H = 8 };

  // CABAC
  Engine eng;
  CtxS ctx[kNumDCtx], wpp_ctx[kNumDCtx], ds_ctx[kNumDCtx];
  bool wpp_saved = false, ds_saved = false;
  const uint8_t* data_end = nullptr;

  // QP
  int qp_prev = 26, cu_qp = 26, qg_pred = 26, log2_min_qg = 6;
  bool qp_delta_coded = false;
  int qp_bd = 0, qp_bd_c = 0;

  // current CU
  int cu_x = 0, cu_y = 0, cu_log2 = 3, cu_part = 0;
  bool cu_intra = false, cu_bypass = false, cu_pcm = false;
  int cu_chroma_mode = 0;      // IntraPredModeC
  bool merge_2nx2n = false;
  int ctb_addr_rs = 0, ctb_addr_ts = 0;

  // GPU records of the current picture
  std::vector<std::vector<DecIntraOp>> ctb_ops;
  std::map<int, int> refpic_index;  // decode_idx -> DecPicture::ref_ids index

  // encoder records (32x32 CTBs)
  bool enc_rec = false;

  // ======================================================================== NAL level
  void decode_nal(const NalUnit& u, const uint8_t* data) {
    const size_t hdr = u.offset + (data[u.offset + 2] == 1 ? 3 : 4);
    const int type = (data[hdr] >> 1) & 63;
    if (u.rbsp.empty()) return;
    const int layer = ((data[hdr] & 1) << 5) | (u.rbsp[0] >> 3);
    const int tid = (u.rbsp[0] & 7) - 1;
    if (layer != 0) return;  // multilayer extensions: base layer only
    BitReader br(u.rbsp.data() + 1, u.rbsp.size() - 1);
    if (type == VPS_NUT) return;
    if (type == SPS_NUT) {
      auto s = std::make_shared<Sps>();
      parse_sps(br, *s);
      const int id = s->id;
      sps_tab[id] = std::move(s);
      return;
    }
    if (type == PPS_NUT) {
      auto p = std::make_shared<Pps>();
      const Sps* tab[16];
      for (int i = 0; i < 16; ++i) tab[i] = sps_tab[i].get();
      parse_pps(br, *p, tab);
      const int id = p->id;
      pps_tab[id] = std::move(p);
      return;
    }
    if (type == EOS_NUT || type == EOB_NUT) {
      finish_picture();
      after_eos = true;
      return;
    }
    if (type > 21 || (type >= 10 && type <= 15)) return;  // reserved VCL, SEI, AUD, filler
    decode_slice_nal(u, type, tid);
  }

  // ======================================================================== slice
  void decode_slice_nal(const NalUnit& u, int type, int tid) {
    BitReader br(u.rbsp.data() + 1, u.rbsp.size() - 1);
    const Sps* stab[16];
    const Pps* ptab[64];
    for (int i = 0; i < 16; ++i) stab[i] = sps_tab[i].get();
    for (int i = 0; i < 64; ++i) ptab[i] = pps_tab[i].get();
    // first_slice_segment_in_pic_flag decides whether a new picture starts
    const bool first = (u.rbsp.size() > 1) && (u.rbsp[1] & 0x80);
    if (first) finish_picture();
    if (!first && !pic_open) return;  // slices of a skipped (RASL) or missing picture
    SliceHeader h;
    int npc = 0;
    parse_slice_header(br, type, stab, ptab, have_indep ? &indep : nullptr, h, &npc);
    if (first) {
      if (!start_picture(h, type, tid)) return;  // RASL skipped
    } else if (h.pps_id != sh.pps_id && !h.dependent) {
      fail("slices of one picture use different PPSs");
    }
    sh = h;
    if (!sh.dependent) {
      indep = sh;
      have_indep = true;
      slice_addr_rs = sh.segment_addr;
      build_ref_lists(npc);
    }
    slices.push_back(sh);
    slice_idx = static_cast<int>(slices.size()) - 1;
    slice_qp = pps->init_qp + sh.qp_delta;
    if (slice_qp < -qp_bd || slice_qp > 51) fail("SliceQpY out of range");
    init_type = sh.slice_type == 2 ? 0 : (sh.slice_type == 1 ? (sh.cabac_init ? 2 : 1) : (sh.cabac_init ? 1 : 2));
    add_slice_records();
    decode_slice_data(u);
  }

  // 8.3.1 POC, 8.3.2 RPS, DPB bookkeeping; returns false for a skipped RASL picture
  bool start_picture(const SliceHeader& h, int type, int tid) {
    pps_hold = pps_tab[h.pps_id];
    pps = pps_hold.get();
    sps_hold = sps_tab[pps->sps_id];
    const Sps* s = sps_hold.get();
    if (!s) fail("missing SPS");
    const bool irap = is_irap(type);
    if (irap) {
      no_rasl_output = is_idr(type) || is_bla(type) || first_pic || after_eos;
      if (no_rasl_output) {
        ++cvs;
        if (sps != s) sps = s;
      }
    }
    if (first_pic && !irap) fail("stream does not start with an IRAP picture");
    if (is_rasl(type) && no_rasl_output) return false;  // associated with a CRA that starts decoding
    if (sps != s) {
      if (!irap) fail("SPS change at a non-IRAP picture");
      sps = s;
    }
    first_pic = false;
    after_eos = false;
    nal_type = type;
    // ---- POC (8.3.1)
    const int maxlsb = 1 << sps->log2_max_poc_lsb;
    int msb = 0;
    if (!(irap && no_rasl_output)) {
      const int prev_lsb = prev_tid0_poc & (maxlsb - 1), prev_msb = prev_tid0_poc - prev_lsb;
      const int lsb = h.poc_lsb;
      if (lsb < prev_lsb && prev_lsb - lsb >= maxlsb / 2) msb = prev_msb + maxlsb;
      else if (lsb > prev_lsb && lsb - prev_lsb > maxlsb / 2) msb = prev_msb - maxlsb;
      else msb = prev_msb;
    }
    poc = msb + (is_idr(type) ? 0 : h.poc_lsb);
    if (tid == 0 && !is_rasl(type) && !is_radl(type) && !is_slnr(type)) prev_tid0_poc = poc;
    // ---- reference picture set (8.3.2): marking
    if (irap && no_rasl_output) {
      for (auto& p : dpb) p->is_ref = false;
    }
    std::vector<std::shared_ptr<StoredPic>> keep;
    if (!is_idr(type)) {
      for (int i = 0; i < h.st.num_delta(); ++i) {
        const int want = poc + h.st.delta[i];
        for (auto& p : dpb)
          if (p->is_ref && !p->is_lt && p->cvs == cvs && p->poc == want) keep.push_back(p);
      }
      for (int i = 0; i < h.num_lt; ++i) {
        int want = h.lt_poc[i];
        const bool full = h.lt_msb_present[i];
        if (full) want += poc - (poc & (maxlsb - 1));
        for (auto& p : dpb)
          if (p->is_ref && p->cvs == cvs && (full ? p->poc == want : (p->poc & (maxlsb - 1)) == want)) {
            p->is_lt = true;
            keep.push_back(p);
          }
      }
    }
    for (auto& p : dpb) {
      bool k = false;
      for (auto& q : keep) k |= q == p;
      if (!k) p->is_ref = false;
    }
    // drop pictures no longer referenced (their output is tracked by DecPicture)
    dpb.erase(std::remove_if(dpb.begin(), dpb.end(), [](const std::shared_ptr<StoredPic>& p) { return !p->is_ref; }),
              dpb.end());
    // ---- geometry and per-picture arrays
    W = sps->W;
    H = sps->H;
    bd = sps->bit_depth;
    bdc = sps->bit_depth_c;
    maxv = (1 << bd) - 1;
    maxvc = (1 << bdc) - 1;
    qp_bd = 6 * (bd - 8);
    qp_bd_c = 6 * (bdc - 8);
    log2_ctb = sps->log2_ctb;
    ctb = 1 << log2_ctb;
    wctb = sps->wctb;
    hctb = sps->hctb;
    nctb = wctb * hctb;
    w4 = W / 4;
    h4 = H / 4;
    l4 = log2_ctb - 2;
    log2_min_cb = sps->log2_min_cb;
    log2_min_tb = sps->log2_min_tb;
    log2_max_tb = sps->log2_max_tb;
    build_tiles();
    const size_t n4 = static_cast<size_t>(w4) * h4;
    cu_flags.assign(n4, 0);
    ct_depth.assign(n4, 0);
    ipm.assign(n4, 1);
    edge.assign(n4, 0);
    cbf_y.assign(n4, 0);
    qp_y.assign(n4, 0);
    ctb_slice.assign(nctb, -1);
    ctb_saddr.assign(nctb, -1);
    cur = std::make_shared<StoredPic>();
    cur->decode_idx = decode_count++;
    cur->poc = poc;
    cur->cvs = cvs;
    cur->W = W;
    cur->H = H;
    cur->w4 = w4;
    cur->h4 = h4;
    cur->log2_ctb = log2_ctb;
    cur->wctb = wctb;
    cur->mvf.assign(n4, MvField{{{0, 0}, {0, 0}}, {-1, -1}, 0, 0});
    cur->ctb_slice.assign(nctb, 0);
    if (opt.recon) {
      cur->pl[0].assign(n4 * 16, 0);
      cur->pl[1].assign(n4 * 4, 0);
      cur->pl[2].assign(n4 * 4, 0);
    }
    slices.clear();
    have_indep = false;
    // ---- output record
    out->emplace_back();
    dp = &out->back();
    DecPicture& d = *dp;
    d.decode_idx = cur->decode_idx;
    d.poc = poc;
    d.cvs = cvs;
    d.output = h.pic_output && !(is_rasl(type) && no_rasl_output);
    d.irap = irap;
    d.idr = is_idr(type);
    d.nal_type = type;
    d.slice_type = h.slice_type;
    d.W = W;
    d.H = H;
    d.crop_x = 2 * sps->conf[0];
    d.crop_y = 2 * sps->conf[2];
    d.width = W - 2 * (sps->conf[0] + sps->conf[1]);
    d.height = H - 2 * (sps->conf[2] + sps->conf[3]);
    d.bit_depth = bd;
    d.bit_depth_c = bdc;
    d.log2_ctb = log2_ctb;
    d.wctb = wctb;
    d.hctb = hctb;
    d.constrained_intra = pps->constrained_intra;
    d.strong_intra = sps->strong_intra;
    d.lf_across_tiles = pps->lf_across_tiles;
    d.cb_qp_off = pps->cb_qp_off;
    d.cr_qp_off = pps->cr_qp_off;
    if (opt.gpu_records) {
      d.mvf.clear();
      d.mvf_sub.clear();
      d.bs.assign(n4, 0);
      d.ctbs.assign(nctb, DecCtb{});
      d.sao.assign(nctb, DecSao{});
      d.ops_off.assign(nctb + 1, 0);
      ctb_ops.assign(nctb, {});
      refpic_index.clear();
      if (sps->scaling_enabled) {
        const ScalingList& sl = pps->scaling_present ? pps->scaling : sps->scaling;
        d.scaling.assign(sl.f.begin(), sl.f.end());
      }
    }
    // encoder records: per 32x32 block (the encoder's record unit) for 32x32 CTBs and for 64x64
    // CTUs over a picture of whole 32x32 blocks
    enc_rec = opt.enc_records && log2_min_cb == kMinCbLog2 &&
              (log2_ctb == kCtbLog2 || (log2_ctb == 6 && W % 32 == 0 && H % 32 == 0));
    if (enc_rec) {
      d.ctu.assign(static_cast<size_t>(W / 32) * (H / 32), CtuInfo{});
      d.cu.assign(static_cast<size_t>(W / 32) * (H / 32) * kCusPerCtb, CuInfo{});
      d.coef_y.assign(n4 * 16, 0);
      d.coef_cb.assign(n4 * 4, 0);
      d.coef_cr.assign(n4 * 4, 0);
    }
    pic_open = true;
    return true;
  }

  // 6.5.1 CTB raster <-> tile scan conversion
  void build_tiles() {
    const int cols = pps->tiles ? pps->tile_cols : 1, rows = pps->tiles ? pps->tile_rows : 1;
    std::vector<int> cw(cols), rh(rows);
    if (!pps->tiles || pps->uniform_spacing) {
      for (int i = 0; i < cols; ++i) cw[i] = ((i + 1) * wctb) / cols - (i * wctb) / cols;
      for (int j = 0; j < rows; ++j) rh[j] = ((j + 1) * hctb) / rows - (j * hctb) / rows;
    } else {
      int acc = 0;
      for (int i = 0; i < cols - 1; ++i) acc += (cw[i] = pps->col_width[i]);
      cw[cols - 1] = wctb - acc;
      acc = 0;
      for (int j = 0; j < rows - 1; ++j) acc += (rh[j] = pps->row_height[j]);
      rh[rows - 1] = hctb - acc;
    }
    for (int v : cw)
      if (v <= 0) fail("tile columns do not fit the picture");
    for (int v : rh)
      if (v <= 0) fail("tile rows do not fit the picture");
    col_bd.assign(cols + 1, 0);
    row_bd.assign(rows + 1, 0);
    for (int i = 0; i < cols; ++i) col_bd[i + 1] = col_bd[i] + cw[i];
    for (int j = 0; j < rows; ++j) row_bd[j + 1] = row_bd[j] + rh[j];
    rs2ts.assign(nctb, 0);
    ts2rs.assign(nctb, 0);
    tile_id.assign(nctb, 0);
    for (int rs = 0; rs < nctb; ++rs) {
      const int tbx = rs % wctb, tby = rs / wctb;
      int tx = 0, ty = 0;
      for (int i = 0; i < cols; ++i)
        if (tbx >= col_bd[i]) tx = i;
      for (int j = 0; j < rows; ++j)
        if (tby >= row_bd[j]) ty = j;
      int v = 0;
      for (int i = 0; i < tx; ++i) v += rh[ty] * cw[i];
      for (int j = 0; j < ty; ++j) v += wctb * rh[j];
      v += (tby - row_bd[ty]) * cw[tx] + tbx - col_bd[tx];
      rs2ts[rs] = v;
      ts2rs[v] = rs;
    }
    int tid = 0;
    for (int j = 0; j < rows; ++j)
      for (int i = 0; i < cols; ++i, ++tid)
        for (int y = row_bd[j]; y < row_bd[j + 1]; ++y)
          for (int x = col_bd[i]; x < col_bd[i + 1]; ++x) tile_id[rs2ts[y * wctb + x]] = tid;
  }

  // 8.3.4 reference picture lists of the current (independent) slice
  void build_ref_lists(int npc) {
    for (int l = 0; l < 2; ++l)
      for (int i = 0; i < 16; ++i) {
        ref_list[l][i] = nullptr;
        ref_poc[l][i] = 0;
        ref_lt[l][i] = false;
      }
    if (sh.slice_type == 2) return;
    std::vector<StoredPic*> before, after, lt;
    const int maxlsb = 1 << sps->log2_max_poc_lsb;
    auto find_st = [&](int want) -> StoredPic* {
      for (auto& p : dpb)
        if (p->is_ref && !p->is_lt && p->cvs == cvs && p->poc == want) return p.get();
      return nullptr;
    };
    for (int i = 0; i < sh.st.num_delta(); ++i) {
      if (!sh.st.used[i]) continue;
      StoredPic* p = find_st(poc + sh.st.delta[i]);
      if (!p) fail("a short-term reference picture is missing from the DPB");
      (i < sh.st.num_neg ? before : after).push_back(p);
    }
    for (int i = 0; i < sh.num_lt; ++i) {
      if (!sh.lt_used[i]) continue;
      int want = sh.lt_poc[i];
      const bool full = sh.lt_msb_present[i];
      if (full) want += poc - (poc & (maxlsb - 1));
      StoredPic* f = nullptr;
      for (auto& p : dpb)
        if (p->is_ref && p->is_lt && p->cvs == cvs && (full ? p->poc == want : (p->poc & (maxlsb - 1)) == want)) f = p.get();
      if (!f) fail("a long-term reference picture is missing from the DPB");
      lt.push_back(f);
    }
    if (static_cast<int>(before.size() + after.size() + lt.size()) != npc) fail("NumPicTotalCurr mismatch");
    for (int l = 0; l < (sh.slice_type == 0 ? 2 : 1); ++l) {
      const int n = std::max(sh.num_ref[l], npc);
      std::vector<StoredPic*> tmp;
      std::vector<bool> tlt;
      while (static_cast<int>(tmp.size()) < n) {
        auto& a = l == 0 ? before : after;
        auto& b = l == 0 ? after : before;
        for (size_t i = 0; i < a.size() && static_cast<int>(tmp.size()) < n; ++i) {
          tmp.push_back(a[i]);
          tlt.push_back(false);
        }
        for (size_t i = 0; i < b.size() && static_cast<int>(tmp.size()) < n; ++i) {
          tmp.push_back(b[i]);
          tlt.push_back(false);
        }
        for (size_t i = 0; i < lt.size() && static_cast<int>(tmp.size()) < n; ++i) {
          tmp.push_back(lt[i]);
          tlt.push_back(true);
        }
      }
      for (int i = 0; i < sh.num_ref[l]; ++i) {
        const int k = sh.list_mod[l] ? sh.list_entry[l][i] : i;
        ref_list[l][i] = tmp[k];
        ref_poc[l][i] = tmp[k]->poc;
        ref_lt[l][i] = tlt[k];
      }
    }
    // NoBackwardPredFlag (8.5.3.2.9): no reference picture follows the current one
    nobackward = true;
    for (int l = 0; l < 2; ++l)
      for (int i = 0; i < sh.num_ref[l]; ++i)
        if (ref_poc[l][i] > poc) nobackward = false;
  }

  // per slice segment: GPU slice / reference tables and the TMVP reference record
  void add_slice_records() {
    SliceRefs sr;
    for (int l = 0; l < 2; ++l) {
      sr.n[l] = sh.num_ref[l];
      for (int i = 0; i < sh.num_ref[l]; ++i) {
        sr.poc[l][i] = ref_poc[l][i];
        sr.lt[l][i] = ref_lt[l][i];
        sr.pic[l][i] = ref_list[l][i] ? ref_list[l][i]->decode_idx : -1;
      }
    }
    cur->slices.push_back(sr);
    if (!opt.gpu_records) return;
    DecPicture& d = *dp;
    DecSlice ds;
    ds.beta_off = static_cast<int8_t>(sh.beta_off);
    ds.tc_off = static_cast<int8_t>(sh.tc_off);
    ds.deblock_off = sh.deblock_disabled;
    ds.lf_across = sh.lf_across_slices;
    ds.addr_rs = static_cast<uint32_t>(slice_addr_rs);
    d.slices.push_back(ds);
    for (int l = 0; l < 2; ++l) {
      ref_entry_base[l] = static_cast<int>(d.refs.size());
      for (int i = 0; i < sh.num_ref[l]; ++i) {
        DecRefEntry e{};
        const int id = ref_list[l][i]->decode_idx;
        auto it = refpic_index.find(id);
        if (it == refpic_index.end()) {
          it = refpic_index.emplace(id, static_cast<int>(d.ref_ids.size())).first;
          d.ref_ids.push_back(id);
        }
        e.pic = static_cast<int8_t>(it->second);
        e.weighted = sh.weighted;
        e.log2wd_y = static_cast<uint8_t>(sh.pw.log2_denom_y);
        e.log2wd_c = static_cast<uint8_t>(sh.pw.log2_denom_c);
        for (int c = 0; c < 3; ++c) {
          e.w[c] = static_cast<int16_t>(sh.weighted ? sh.pw.w[l][i][c] : 1);
          e.o[c] = static_cast<int16_t>(sh.weighted ? sh.pw.o[l][i][c] * (1 << ((c ? bdc : bd) - 8)) : 0);
        }
        d.refs.push_back(e);
      }
    }
    if (d.refs.size() > 255 || d.ref_ids.size() > 16) fail("too many reference entries for the GPU records");
  }

  // ======================================================================== slice data (7.3.8.1)
  void decode_slice_data(const NalUnit& u) {
    const uint8_t* base = u.rbsp.data() + 1;
    const uint8_t* end = u.rbsp.data() + u.rbsp.size();
    data_end = end;
    const uint8_t* p = base + sh.data_byte;
    if (sh.segment_addr >= nctb) fail("slice_segment_address out of range");
    ctb_addr_rs = sh.segment_addr;
    ctb_addr_ts = rs2ts[ctb_addr_rs];
    if (ctb_slice[ctb_addr_rs] >= 0) fail("slice segment overlaps decoded CTBs");
    log2_min_qg = log2_ctb - pps->diff_cu_qp_delta_depth;
    eng.start(p, end);
    start_contexts(true);
    while (true) {
      if (ctb_addr_ts >= nctb) fail("slice data runs past the last CTB");
      ctb_addr_rs = ts2rs[ctb_addr_ts];
      ctb_slice[ctb_addr_rs] = static_cast<int16_t>(slice_idx);
      ctb_saddr[ctb_addr_rs] = slice_addr_of(slice_idx);
      cur->ctb_slice[ctb_addr_rs] = static_cast<uint16_t>(slice_idx);
      if (opt.gpu_records) {
        DecCtb& c = dp->ctbs[ctb_addr_rs];
        c.slice = static_cast<uint16_t>(slice_idx);
        c.tile = static_cast<uint16_t>(tile_id[ctb_addr_ts]);
        c.ts = static_cast<uint32_t>(ctb_addr_ts);
      }
      coding_tree_unit();
      const int end_of_slice = eng.terminate();
      // 9.3.2.x: WPP storage after the second CTB of a row (of the tile)
      const int rx = ctb_addr_rs % wctb;
      if (pps->wpp && rx == tile_col_start(rx) + 1) {
        std::memcpy(wpp_ctx, ctx, sizeof(ctx));
        wpp_saved = true;
      }
      ++ctb_addr_ts;
      if (end_of_slice) {
        if (pps->dependent_slices) {
          std::memcpy(ds_ctx, ctx, sizeof(ctx));
          ds_saved = true;
        }
        break;
      }
      if (ctb_addr_ts >= nctb) fail("end_of_slice_segment_flag missing at the last CTB");
      const int nrs = ts2rs[ctb_addr_ts];
      const bool new_tile = pps->tiles && tile_id[ctb_addr_ts] != tile_id[ctb_addr_ts - 1];
      const bool new_row = pps->wpp && (nrs % wctb) == tile_col_start(nrs % wctb);
      if (new_tile || new_row) {
        if (eng.terminate() != 1) fail("end_of_subset_one_bit != 1");
        // byte_alignment() was consumed with the terminating bin: continue at the next byte
        eng.start(eng.pos(), end);
        start_contexts(false);
      }
    }
  }

  int tile_col_start(int x) const {
    int s = 0;
    for (size_t i = 0; i + 1 < col_bd.size(); ++i)
      if (x >= col_bd[i]) s = col_bd[i];
    return s;
  }

  // context initialisation / synchronisation at the start of a slice segment, tile or WPP row
  void start_contexts(bool slice_start) {
    const int rs = ctb_addr_rs = ts2rs[ctb_addr_ts];
    const int rx = rs % wctb, ry = rs / wctb;
    const bool first_in_tile = ctb_addr_ts == 0 || tile_id[ctb_addr_ts] != tile_id[ctb_addr_ts - 1];
    const bool row_start = rx == tile_col_start(rx);
    if (first_in_tile && (slice_start ? true : pps->tiles)) {
      init_ctx(ctx, init_type, slice_qp);
    } else if (pps->wpp && row_start) {
      // sync from the CTB above-right when it is available (same slice and tile)
      const int tx = (rx + 1) * ctb, ty = (ry - 1) * ctb;
      bool avail = false;
      if (ty >= 0 && tx < W) {
        const int nrs = (ry - 1) * wctb + rx + 1;
        avail = ctb_slice[nrs] >= 0 && slices[ctb_slice[nrs]].segment_addr >= 0 &&
                slice_addr_of(ctb_slice[nrs]) == slice_addr_rs && tile_id[rs2ts[nrs]] == tile_id[ctb_addr_ts];
      }
      if (avail && wpp_saved) std::memcpy(ctx, wpp_ctx, sizeof(ctx));
      else init_ctx(ctx, init_type, slice_qp);
    } else if (slice_start && sh.dependent) {
      if (!ds_saved) fail("dependent slice segment without stored contexts");
      std::memcpy(ctx, ds_ctx, sizeof(ctx));
    } else {
      init_ctx(ctx, init_type, slice_qp);
    }
    // 8.6.1 qPY_PREV: SliceQpY at the first QG of a slice, of a tile and of a WPP row
    if ((slice_start && !sh.dependent) || first_in_tile || (pps->wpp && row_start)) qp_prev = slice_qp;
  }

  int slice_addr_of(int sidx) const {
    // SliceAddrRs of slice segment sidx: its own address, or the independent segment's
    for (int k = sidx; k >= 0; --k)
      if (!slices[k].dependent) return slices[k].segment_addr;
    return 0;
  }

  // ======================================================================== availability (6.4.1 / 6.4.2)
  size_t g4(int x, int y) const { return static_cast<size_t>(y >> 2) * w4 + (x >> 2); }
  uint32_t zaddr(int x, int y) const {
    const int rs = (y >> log2_ctb) * wctb + (x >> log2_ctb);
    const int m = (1 << l4) - 1;
    return (static_cast<uint32_t>(rs2ts[rs]) << (2 * l4)) | zorder((x >> 2) & m, (y >> 2) & m);
  }
  // z-scan availability of (xn, yn) for the block at (xc, yc)
  bool avail_z(int xc, int yc, int xn, int yn) const {
    if (xn < 0 || yn < 0 || xn >= W || yn >= H) return false;
    const int rsn = (yn >> log2_ctb) * wctb + (xn >> log2_ctb);
    const int rsc = (yc >> log2_ctb) * wctb + (xc >> log2_ctb);
    if (rsn == rsc) {  // same CTB (so same slice segment and tile): z-order alone decides
      const int m = (1 << l4) - 1;
      return zorder((xn >> 2) & m, (yn >> 2) & m) <= zorder((xc >> 2) & m, (yc >> 2) & m);
    }
    if (ctb_slice[rsn] < 0) return false;
    const int tsn = rs2ts[rsn], tsc = rs2ts[rsc];
    if (tsn > tsc) return false;
    if (ctb_saddr[rsn] != ctb_saddr[rsc]) return false;
    if (tile_id[tsn] != tile_id[tsc]) return false;
    return true;
  }
  // 6.4.2 prediction block availability
  bool avail_pb(int xcb, int ycb, int ncbs, int xpb, int ypb, int npbw, int npbh, int part_idx, int xn, int yn) const {
    bool same_cb = xcb <= xn && ycb <= yn && xcb + ncbs > xn && ycb + ncbs > yn;
    bool av;
    if (!same_cb) av = avail_z(xpb, ypb, xn, yn);
    else if ((npbw << 1) == ncbs && (npbh << 1) == ncbs && part_idx == 1 && ycb + npbh <= yn && xcb + npbw > xn) av = false;
    else av = true;
    if (av && (cu_flags[g4(xn, yn)] & CF_INTRA)) av = false;
    return av;
  }

  // ======================================================================== CTU (7.3.8.2)
  void coding_tree_unit() {
    const int rx = ctb_addr_rs % wctb, ry = ctb_addr_rs / wctb;
    const int x0 = rx << log2_ctb, y0 = ry << log2_ctb;
    if (sh.sao_luma || sh.sao_chroma) parse_sao(rx, ry);
    coding_quadtree(x0, y0, log2_ctb, 0);
  }

  // 7.3.8.3 sao()
  std::vector<DecSao> sao_params;  // per CTB (kept even without GPU records: CPU SAO)
  void parse_sao(int rx, int ry) {
    if (sao_params.size() != static_cast<size_t>(nctb)) sao_params.assign(nctb, DecSao{});
    DecSao& t = sao_params[ctb_addr_rs];
    t = DecSao{};
    bool merge_left = false, merge_up = false;
    if (rx > 0) {
      const bool in_slice = ctb_addr_rs > slice_addr_rs;  // leftCtbInSliceSeg
      const bool in_tile = tile_id[ctb_addr_ts] == tile_id[rs2ts[ctb_addr_rs - 1]];
      if (in_slice && in_tile) merge_left = eng.decode(ctx[C_SAO_MERGE]);
    }
    if (ry > 0 && !merge_left) {
      const int up = ctb_addr_rs - wctb;
      const bool in_slice = up >= slice_addr_rs;  // upCtbInSliceSeg
      const bool in_tile = tile_id[ctb_addr_ts] == tile_id[rs2ts[up]];
      if (in_slice && in_tile) merge_up = eng.decode(ctx[C_SAO_MERGE]);
    }
    if (merge_left || merge_up) {
      t = sao_params[merge_left ? ctb_addr_rs - 1 : ctb_addr_rs - wctb];
    } else {
      for (int ci = 0; ci < 3; ++ci) {
        if ((ci == 0 && !sh.sao_luma) || (ci > 0 && !sh.sao_chroma)) {
          t.type[ci] = 0;
          continue;
        }
        if (ci < 2) {
          int type = 0;
          if (eng.decode(ctx[C_SAO_TYPE])) type = eng.bypass() ? 2 : 1;
          t.type[ci] = static_cast<uint8_t>(type);
        } else {
          t.type[2] = t.type[1];
        }
        if (!t.type[ci]) continue;
        const int cmax = (1 << (std::min(ci ? bdc : bd, 10) - 5)) - 1;
        int a[4];
        for (int i = 0; i < 4; ++i) {
          int v = 0;
          while (v < cmax && eng.bypass()) ++v;
          a[i] = v;
        }
        if (t.type[ci] == 1) {
          for (int i = 0; i < 4; ++i) t.off[ci][i] = static_cast<int8_t>(a[i] && eng.bypass() ? -a[i] : a[i]);
          t.band[ci] = static_cast<uint8_t>(eng.bypass_bits(5));
        } else {
          t.off[ci][0] = static_cast<int8_t>(a[0]);
          t.off[ci][1] = static_cast<int8_t>(a[1]);
          t.off[ci][2] = static_cast<int8_t>(-a[2]);
          t.off[ci][3] = static_cast<int8_t>(-a[3]);
          if (ci == 0) t.eo[0] = static_cast<uint8_t>(eng.bypass_bits(2));
          if (ci == 1) t.eo[1] = static_cast<uint8_t>(eng.bypass_bits(2));
          if (ci == 2) t.eo[2] = t.eo[1];
        }
      }
    }
    // a merged CTB takes the neighbour's parameters; components this slice has off stay off
    if (!sh.sao_luma) t.type[0] = 0;
    if (!sh.sao_chroma) t.type[1] = t.type[2] = 0;
    if (opt.gpu_records) dp->sao[ctb_addr_rs] = t;
    if (enc_rec) {  // every 32x32 record block of the CTB carries its parameters
      const int x0 = (ctb_addr_rs % wctb) << log2_ctb, y0 = (ctb_addr_rs / wctb) << log2_ctb;
      for (int y = y0; y < std::min(H, y0 + ctb); y += 32)
        for (int x = x0; x < std::min(W, x0 + ctb); x += 32) {
          CtuInfo& c = enc_blk(x, y);
          c.sao_type[0] = t.type[0];
          c.sao_type[1] = t.type[1];
          c.sao_class[0] = t.eo[0];
          c.sao_class[1] = t.eo[1];
          for (int ci = 0; ci < 3; ++ci) {
            c.sao_band[ci] = t.band[ci];
            for (int i = 0; i < 4; ++i) c.sao_off[ci][i] = t.off[ci][i];
          }
        }
    }
  }

  // 7.3.8.4 coding_quadtree()
  void coding_quadtree(int x0, int y0, int log2, int depth) {
    const int n = 1 << log2;
    bool split;
    if (x0 + n <= W && y0 + n <= H && log2 > log2_min_cb) {
      int c = 0;
      if (avail_z(x0, y0, x0 - 1, y0) && ct_depth[g4(x0 - 1, y0)] > depth) ++c;
      if (avail_z(x0, y0, x0, y0 - 1) && ct_depth[g4(x0, y0 - 1)] > depth) ++c;
      split = eng.decode(ctx[C_SPLIT_CU + c]);
    } else {
      split = log2 > log2_min_cb;
    }
    if (pps->cu_qp_delta && log2 >= log2_min_qg) start_qg(x0, y0, n);
    if (split) {
      if (enc_rec) {  // split bits of the 32x32 record block (a 64x64 split has no bit)
        CtuInfo& t = enc_blk(x0, y0);
        if (log2 == 5) t.split |= 1;
        else if (log2 == 4) t.split |= static_cast<uint8_t>(1 << (1 + ((x0 & 31) >= 16) + 2 * ((y0 & 31) >= 16)));
      }
      const int h = n >> 1;
      for (int q = 0; q < 4; ++q) {
        const int x1 = x0 + (q & 1) * h, y1 = y0 + (q >> 1) * h;
        if (x1 < W && y1 < H) coding_quadtree(x1, y1, log2 - 1, depth + 1);
      }
      return;
    }
    coding_unit(x0, y0, log2, depth);
  }

  // 8.6.1: a quantization group starts (n: the size of the coding quadtree node it starts at)
  int qg_x = 0, qg_y = 0, qg_n = 32;
  void start_qg(int x0, int y0, int n) {
    qg_x = x0;
    qg_y = y0;
    qg_n = n;
    qp_delta_coded = false;
    const int cm = ~(ctb - 1);
    auto nb = [&](int x, int y) {
      if (!avail_z(x0, y0, x, y) || (x & cm) != (x0 & cm) || (y & cm) != (y0 & cm)) return qp_prev;
      return static_cast<int>(qp_y[g4(x, y)]);
    };
    qg_pred = (nb(x0 - 1, y0) + nb(x0, y0 - 1) + 1) >> 1;
    cu_qp = qg_pred;
    if (enc_rec && (x0 & 31) == 0 && (y0 & 31) == 0)
      for_qg_blocks([&](CtuInfo& t) {
        t.qp = static_cast<int8_t>(qg_pred);
        t.qp_pred = static_cast<int8_t>(qg_pred);
        t.qp_first = 16;
      });
  }
  // the 32x32 record blocks of the current quantization group (one, or four for a 64x64 node)
  template <class F>
  void for_qg_blocks(F f) {
    for (int y = qg_y; y < std::min(H, qg_y + std::max(qg_n, 32)); y += 32)
      for (int x = qg_x; x < std::min(W, qg_x + std::max(qg_n, 32)); x += 32) f(enc_blk(x, y));
  }

  // ======================================================================== coding unit (7.3.8.5)
  void coding_unit(int x0, int y0, int log2, int depth) {
    if (!pps->cu_qp_delta) cu_qp = slice_qp;
    const int n = 1 << log2;
    cu_x = x0;
    cu_y = y0;
    cu_log2 = log2;
    cu_bypass = false;
    cu_pcm = false;
    cu_intra = false;
    cu_part = P_2Nx2N;
    merge_2nx2n = false;
    if (pps->transquant_bypass) cu_bypass = eng.decode(ctx[C_TQ_BYPASS]);
    bool skip = false;
    if (sh.slice_type != 2) {
      int c = 0;
      if (avail_z(x0, y0, x0 - 1, y0) && (cu_flags[g4(x0 - 1, y0)] & CF_SKIP)) ++c;
      if (avail_z(x0, y0, x0, y0 - 1) && (cu_flags[g4(x0, y0 - 1)] & CF_SKIP)) ++c;
      skip = eng.decode(ctx[C_SKIP + c]);
    }
    // CU-level state on the 4x4 grid (needed by the CU's own PUs / TUs)
    uint8_t flags = static_cast<uint8_t>((skip ? CF_SKIP : 0) | (cu_bypass ? CF_BYPASS : 0));
    if (skip) {
      fill_cu(x0, y0, n, static_cast<uint8_t>(flags | CF_INTER), depth);
      mark_edges_cu(x0, y0, n);
      prediction_unit(x0, y0, n, n, 0, true);
      if (enc_rec) enc_cu(x0, y0, n, CU_INTER, 0);
      finish_cu(x0, y0, n);
      return;
    }
    if (sh.slice_type != 2) cu_intra = eng.decode(ctx[C_PRED_MODE]);
    else cu_intra = true;
    if (!cu_intra || log2 == log2_min_cb) cu_part = parse_part_mode(log2);
    fill_cu(x0, y0, n, static_cast<uint8_t>(flags | (cu_intra ? CF_INTRA : CF_INTER)), depth);
    mark_edges_cu(x0, y0, n);
    if (cu_intra) {
      if (cu_part == P_2Nx2N && sps->pcm && log2 >= sps->log2_min_pcm && log2 <= sps->log2_max_pcm)
        cu_pcm = eng.terminate();
      if (cu_pcm) {
        for (int y = y0; y < y0 + n; y += 4)
          for (int x = x0; x < x0 + n; x += 4) cu_flags[g4(x, y)] |= CF_PCM;
        pcm_sample(x0, y0, log2);
        if (enc_rec) enc_cu(x0, y0, n, CU_INTRA, 1);
        finish_cu(x0, y0, n);
        return;
      }
      intra_modes(x0, y0, log2);
    } else {
      const int h = n / 2, q = n / 4;
      switch (cu_part) {
        case P_2Nx2N: prediction_unit(x0, y0, n, n, 0, false); break;
        case P_2NxN:
          prediction_unit(x0, y0, n, h, 0, false);
          prediction_unit(x0, y0 + h, n, h, 1, false);
          break;
        case P_Nx2N:
          prediction_unit(x0, y0, h, n, 0, false);
          prediction_unit(x0 + h, y0, h, n, 1, false);
          break;
        case P_2NxnU:
          prediction_unit(x0, y0, n, q, 0, false);
          prediction_unit(x0, y0 + q, n, n - q, 1, false);
          break;
        case P_2NxnD:
          prediction_unit(x0, y0, n, n - q, 0, false);
          prediction_unit(x0, y0 + n - q, n, q, 1, false);
          break;
        case P_nLx2N:
          prediction_unit(x0, y0, q, n, 0, false);
          prediction_unit(x0 + q, y0, n - q, n, 1, false);
          break;
        case P_nRx2N:
          prediction_unit(x0, y0, n - q, n, 0, false);
          prediction_unit(x0 + n - q, y0, q, n, 1, false);
          break;
        default:  // P_NxN
          prediction_unit(x0, y0, h, h, 0, false);
          prediction_unit(x0 + h, y0, h, h, 1, false);
          prediction_unit(x0, y0 + h, h, h, 2, false);
          prediction_unit(x0 + h, y0 + h, h, h, 3, false);
      }
    }
    bool root = true;
    if (!cu_intra && !(cu_part == P_2Nx2N && merge_2nx2n)) root = eng.decode(ctx[C_ROOT_CBF]);
    if (enc_rec) enc_cu(x0, y0, n, cu_intra ? CU_INTRA : CU_INTER, 0);
    if (root) {
      const int intra_split = cu_intra && cu_part == P_NxN;
      const int max_depth = cu_intra ? sps->depth_intra + intra_split : sps->depth_inter;
      transform_tree(x0, y0, x0, y0, log2, 0, 0, max_depth, intra_split, 1, 1);
    }
    finish_cu(x0, y0, n);
  }

  int parse_part_mode(int log2) {
    if (eng.decode(ctx[C_PART_MODE])) return P_2Nx2N;
    if (cu_intra) return P_NxN;
    if (log2 == log2_min_cb) {
      if (eng.decode(ctx[C_PART_MODE + 1])) return P_2NxN;
      if (log2 == 3) return P_Nx2N;
      if (eng.decode(ctx[C_PART_MODE + 2])) return P_Nx2N;
      return P_NxN;
    }
    if (!sps->amp) return eng.decode(ctx[C_PART_MODE + 1]) ? P_2NxN : P_Nx2N;
    if (eng.decode(ctx[C_PART_MODE + 1])) {
      if (eng.decode(ctx[C_PART_MODE + 3])) return P_2NxN;
      return eng.bypass() ? P_2NxnD : P_2NxnU;
    }
    if (eng.decode(ctx[C_PART_MODE + 3])) return P_Nx2N;
    return eng.bypass() ? P_nRx2N : P_nLx2N;
  }

  void fill_cu(int x0, int y0, int n, uint8_t flags, int depth) {
    for (int y = y0; y < y0 + n && y < H; y += 4)
      for (int x = x0; x < x0 + n && x < W; x += 4) {
        const size_t k = g4(x, y);
        cu_flags[k] = flags;
        ct_depth[k] = static_cast<uint8_t>(depth);
        cbf_y[k] = 0;
        ipm[k] = 1;
        if (flags & CF_INTRA) {
          MvField& m = cur->mvf[k];
          m.pred = 0;
          m.ref[0] = m.ref[1] = -1;
          m.mv[0][0] = m.mv[0][1] = m.mv[1][0] = m.mv[1][1] = 0;
        }
      }
  }
  void mark_edges_cu(int x0, int y0, int n) {
    // the CU boundary is a TU and PU boundary
    for (int k = 0; k < n; k += 4) {
      if (y0 + k < H) edge[g4(x0, y0 + k)] |= E_TU_V | E_PU_V;
      if (x0 + k < W) edge[g4(x0 + k, y0)] |= E_TU_H | E_PU_H;
    }
  }
  void finish_cu(int x0, int y0, int n) {
    for (int y = y0; y < y0 + n && y < H; y += 4)
      for (int x = x0; x < x0 + n && x < W; x += 4) qp_y[g4(x, y)] = static_cast<int8_t>(cu_qp);
    qp_prev = cu_qp;
  }

  // ---------------------------------------------------------------- PCM (7.3.8.7, 8.4.4.1)
  void pcm_sample(int x0, int y0, int log2) {
    // pcm_flag's terminating bin left the engine at a byte boundary (alignment zeros included)
    RawBits rb{eng.pos(), data_end, 0};
    const int n = 1 << log2, nc = n / 2;
    std::vector<int16_t> ys(n * n), cb(nc * nc), cr(nc * nc);
    for (int i = 0; i < n * n; ++i) ys[i] = static_cast<int16_t>(rb.get(sps->pcm_bd) << (bd - sps->pcm_bd));
    for (int i = 0; i < nc * nc; ++i) cb[i] = static_cast<int16_t>(rb.get(sps->pcm_bd_c) << (bdc - sps->pcm_bd_c));
    for (int i = 0; i < nc * nc; ++i) cr[i] = static_cast<int16_t>(rb.get(sps->pcm_bd_c) << (bdc - sps->pcm_bd_c));
    if (rb.bit) fail("PCM samples do not end on a byte boundary");
    eng.start(rb.p, data_end);  // 9.3.2.5: engine re-initialised after the samples
    const int16_t* src[3] = {ys.data(), cb.data(), cr.data()};
    for (int c = 0; c < 3; ++c) {
      const int xc = c ? x0 / 2 : x0, yc = c ? y0 / 2 : y0, l2 = c ? log2 - 1 : log2, m = 1 << l2;
      if (opt.recon) {
        const int stride = c ? W / 2 : W;
        for (int y = 0; y < m; ++y)
          for (int x = 0; x < m; ++x) cur->pl[c][static_cast<size_t>(yc + y) * stride + xc + x] = static_cast<uint16_t>(src[c][y * m + x]);
      }
      if (opt.gpu_records) {
        const uint32_t t = push_tu(xc, yc, l2, c, 0, DT_PCM, src[c]);
        push_op(xc, yc, l2, c, 0xFF, t);
      }
    }
  }

  // ---------------------------------------------------------------- intra modes (7.3.8.5, 8.4.2, 8.4.3)
  int pu_modes[4] = {1, 1, 1, 1};
  void intra_modes(int x0, int y0, int log2) {
    const int n = 1 << log2;
    const int npu = cu_part == P_NxN ? 4 : 1, h = cu_part == P_NxN ? n / 2 : n;
    int prev[4], mpm[4] = {}, rem[4] = {};
    for (int k = 0; k < npu; ++k) prev[k] = eng.decode(ctx[C_PREV_INTRA]);
    for (int k = 0; k < npu; ++k) {
      if (prev[k]) {
        mpm[k] = eng.bypass();
        if (mpm[k]) mpm[k] += eng.bypass();
      } else {
        rem[k] = static_cast<int>(eng.bypass_bits(5));
      }
    }
    for (int k = 0; k < npu; ++k) {
      const int xp = x0 + (k & 1) * h, yp = y0 + (k >> 1) * h;
      const int m = luma_mode(xp, yp, prev[k], mpm[k], rem[k]);
      pu_modes[k] = m;
      for (int y = yp; y < yp + h; y += 4)
        for (int x = xp; x < xp + h; x += 4) ipm[g4(x, y)] = static_cast<uint8_t>(m);
    }
    int cm = 4;
    if (eng.decode(ctx[C_CHROMA_MODE])) cm = static_cast<int>(eng.bypass_bits(2));
    const int m0 = pu_modes[0];
    if (cm == 4) {
      cu_chroma_mode = m0;
    } else {
      const int tab[4] = {0, 26, 10, 1};
      cu_chroma_mode = tab[cm] == m0 ? 34 : tab[cm];
    }
  }
  // 8.4.2: candModeList from the left / above neighbours (above: inside the CTB only)
  int luma_mode(int xp, int yp, int prev, int mpm, int rem) {
    auto cand = [&](int x, int y, bool above) {
      if (!avail_z(xp, yp, x, y)) return 1;
      const uint8_t f = cu_flags[g4(x, y)];
      if (!(f & CF_INTRA) || (f & CF_PCM)) return 1;
      if (above && y < ((yp >> log2_ctb) << log2_ctb)) return 1;
      return static_cast<int>(ipm[g4(x, y)]);
    };
    const int a = cand(xp - 1, yp, false), b = cand(xp, yp - 1, true);
    int c[3];
    if (a == b) {
      if (a < 2) {
        c[0] = 0;
        c[1] = 1;
        c[2] = 26;
      } else {
        c[0] = a;
        c[1] = 2 + ((a + 29) % 32);
        c[2] = 2 + ((a - 2 + 1) % 32);
      }
    } else {
      c[0] = a;
      c[1] = b;
      if (a != 0 && b != 0) c[2] = 0;
      else if (a != 1 && b != 1) c[2] = 1;
      else c[2] = 26;
    }
    if (prev) return c[mpm];
    if (c[0] > c[1]) std::swap(c[0], c[1]);
    if (c[0] > c[2]) std::swap(c[0], c[2]);
    if (c[1] > c[2]) std::swap(c[1], c[2]);
    int m = rem;
    for (int i = 0; i < 3; ++i)
      if (m >= c[i]) ++m;
    return m;
  }

  // ======================================================================== prediction unit (7.3.8.6)
  void prediction_unit(int xp, int yp, int w, int h, int part_idx, bool skip) {
    MvField mf{{{0, 0}, {0, 0}}, {-1, -1}, 0, 0};
    bool merge = skip;
    int merge_idx = 0;
    if (!skip) merge = eng.decode(ctx[C_MERGE_FLAG]);
    if (merge) {
      if (sh.max_merge > 1) {
        if (eng.decode(ctx[C_MERGE_IDX])) {
          merge_idx = 1;
          while (merge_idx < sh.max_merge - 1 && eng.bypass()) ++merge_idx;
        }
      }
      if (part_idx == 0 && w == (1 << cu_log2) && h == (1 << cu_log2)) merge_2nx2n = true;
      merge_mode(xp, yp, w, h, part_idx, merge_idx, mf);
    } else {
      int idc = 0;  // 0 L0, 1 L1, 2 BI
      if (sh.slice_type == 0) {
        if (w + h != 12) {
          const int d = ct_depth[g4(cu_x, cu_y)];
          if (eng.decode(ctx[C_INTER_PRED + d])) idc = 2;
          else idc = eng.decode(ctx[C_INTER_PRED + 4]);
        } else {
          idc = eng.decode(ctx[C_INTER_PRED + 4]);
        }
      }
      int mvd[2][2] = {{0, 0}, {0, 0}}, ref[2] = {-1, -1}, mvp[2] = {0, 0};
      for (int l = 0; l < 2; ++l) {
        if ((l == 0 && idc == 1) || (l == 1 && idc == 0)) continue;
        ref[l] = 0;
        if (sh.num_ref[l] > 1) ref[l] = parse_ref_idx(sh.num_ref[l] - 1);
        if (l == 1 && sh.mvd_l1_zero && idc == 2) {
          mvd[1][0] = mvd[1][1] = 0;
        } else {
          parse_mvd(mvd[l]);
        }
        mvp[l] = eng.decode(ctx[C_MVP]);
      }
      for (int l = 0; l < 2; ++l) {
        if (ref[l] < 0) continue;
        int px, py;
        amvp(xp, yp, w, h, part_idx, l, ref[l], mvp[l], &px, &py);
        const int ux = (px + mvd[l][0] + 65536) & 0xFFFF, uy = (py + mvd[l][1] + 65536) & 0xFFFF;
        mf.mv[l][0] = static_cast<int16_t>(ux >= 32768 ? ux - 65536 : ux);
        mf.mv[l][1] = static_cast<int16_t>(uy >= 32768 ? uy - 65536 : uy);
        mf.ref[l] = static_cast<int8_t>(ref[l]);
        mf.pred |= static_cast<uint8_t>(1 << l);
      }
    }
    // store the PU's motion, mark its boundary as a prediction edge
    for (int y = yp; y < yp + h; y += 4)
      for (int x = xp; x < xp + w; x += 4) cur->mvf[g4(x, y)] = mf;
    for (int k = 0; k < h; k += 4) edge[g4(xp, yp + k)] |= E_PU_V;
    for (int k = 0; k < w; k += 4) edge[g4(xp + k, yp)] |= E_PU_H;
    if (opt.recon) predict_inter(xp, yp, w, h, mf);
  }

  int parse_ref_idx(int cmax) {
    int i = 0;
    while (i < cmax) {
      const int b = i < 2 ? eng.decode(ctx[C_REF_IDX + i]) : eng.bypass();
      if (!b) break;
      ++i;
    }
    return i;
  }

  void parse_mvd(int* d) {
    const int g0x = eng.decode(ctx[C_MVD_G0]), g0y = eng.decode(ctx[C_MVD_G0]);
    const int g1x = g0x ? eng.decode(ctx[C_MVD_G1]) : 0, g1y = g0y ? eng.decode(ctx[C_MVD_G1]) : 0;
    const int g0[2] = {g0x, g0y}, g1[2] = {g1x, g1y};
    for (int c = 0; c < 2; ++c) {
      d[c] = 0;
      if (!g0[c]) continue;
      int a = 1;
      if (g1[c]) {  // abs_mvd_minus2: EG1
        int k = 1, v = 0;
        while (eng.bypass()) {
          v += 1 << k;
          if (++k > 31) fail("abs_mvd_minus2 prefix too long");
        }
        v += static_cast<int>(eng.bypass_bits(k));
        a = v + 2;
      }
      d[c] = eng.bypass() ? -a : a;
    }
  }

  // ---------------------------------------------------------------- merge (8.5.3.2.2 - 8.5.3.2.5)
  void merge_mode(int xp, int yp, int w, int h, int part_idx, int merge_idx, MvField& out) {
    const int ncbs = 1 << cu_log2;
    const int w0 = w, h0 = h;
    int xpb = xp, ypb = yp, pidx = part_idx, pw = w, ph = h;
    const int par = pps->log2_par_mrg_level;
    if (par > 2 && ncbs == 8) {  // singleMCLFlag: one merge list for every PU of an 8x8 CU
      xpb = cu_x;
      ypb = cu_y;
      pw = ph = ncbs;
      pidx = 0;
    }
    MvField cand[6];
    int nc = 0;
    auto nbmv = [&](int x, int y) -> const MvField& { return cur->mvf[g4(x, y)]; };
    auto par_same = [&](int xn, int yn) { return (xpb >> par) == (xn >> par) && (ypb >> par) == (yn >> par); };
    const int part = (par > 2 && ncbs == 8) ? P_2Nx2N : cu_part;
    // the chosen candidate; 8x4 / 4x8 PUs are uni-predicted.  Spatial candidates only depend on
    // the ones before them, so the list stops as soon as it holds merge_idx + 1 entries
    auto done = [&](const MvField& m) {
      out = m;
      if (out.pred == 3 && w0 + h0 == 12) {
        out.pred = 1;
        out.ref[1] = -1;
        out.mv[1][0] = out.mv[1][1] = 0;
      }
    };
    // A1
    const int xa1 = xpb - 1, ya1 = ypb + ph - 1;
    bool a1 = !par_same(xa1, ya1) && !((part == P_Nx2N || part == P_nLx2N || part == P_nRx2N) && pidx == 1) &&
              avail_pb(cu_x, cu_y, ncbs, xpb, ypb, pw, ph, pidx, xa1, ya1);
    if (a1) cand[nc++] = nbmv(xa1, ya1);
    if (merge_idx < nc) return done(cand[merge_idx]);
    // B1
    const int xb1 = xpb + pw - 1, yb1 = ypb - 1;
    bool b1 = !par_same(xb1, yb1) && !((part == P_2NxN || part == P_2NxnU || part == P_2NxnD) && pidx == 1) &&
              avail_pb(cu_x, cu_y, ncbs, xpb, ypb, pw, ph, pidx, xb1, yb1);
    // pruning compares against availableA1 / availableB1 (before their own pruning)
    const bool av_b1 = b1;
    if (b1 && a1 && same_motion(nbmv(xa1, ya1), nbmv(xb1, yb1))) b1 = false;
    if (b1) cand[nc++] = nbmv(xb1, yb1);
    if (merge_idx < nc) return done(cand[merge_idx]);
    // B0
    const int xb0 = xpb + pw, yb0 = ypb - 1;
    bool b0 = !par_same(xb0, yb0) && avail_pb(cu_x, cu_y, ncbs, xpb, ypb, pw, ph, pidx, xb0, yb0);
    if (b0 && av_b1 && same_motion(nbmv(xb1, yb1), nbmv(xb0, yb0))) b0 = false;
    if (b0) cand[nc++] = nbmv(xb0, yb0);
    if (merge_idx < nc) return done(cand[merge_idx]);
    // A0
    const int xa0 = xpb - 1, ya0 = ypb + ph;
    bool a0 = !par_same(xa0, ya0) && avail_pb(cu_x, cu_y, ncbs, xpb, ypb, pw, ph, pidx, xa0, ya0);
    if (a0 && a1 && same_motion(nbmv(xa1, ya1), nbmv(xa0, ya0))) a0 = false;
    if (a0) cand[nc++] = nbmv(xa0, ya0);
    if (merge_idx < nc) return done(cand[merge_idx]);
    // B2
    const int xb2 = xpb - 1, yb2 = ypb - 1;
    bool b2 = !par_same(xb2, yb2) && avail_pb(cu_x, cu_y, ncbs, xpb, ypb, pw, ph, pidx, xb2, yb2);
    if (b2 && a1 && same_motion(nbmv(xa1, ya1), nbmv(xb2, yb2))) b2 = false;
    if (b2 && av_b1 && same_motion(nbmv(xb1, yb1), nbmv(xb2, yb2))) b2 = false;
    if (a0 + a1 + b0 + b1 == 4) b2 = false;
    if (b2) cand[nc++] = nbmv(xb2, yb2);
    if (merge_idx < nc) {
      out = cand[merge_idx];
    } else {
      // temporal candidate (refIdxLXCol = 0)
      if (sh.tmvp && nc < sh.max_merge) {
        MvField t{{{0, 0}, {0, 0}}, {-1, -1}, 0, 0};
        int mvx, mvy;
        if (temporal_mv(xpb, ypb, pw, ph, 0, 0, &mvx, &mvy)) {
          t.pred |= 1;
          t.ref[0] = 0;
          t.mv[0][0] = static_cast<int16_t>(mvx);
          t.mv[0][1] = static_cast<int16_t>(mvy);
        }
        if (sh.slice_type == 0 && temporal_mv(xpb, ypb, pw, ph, 1, 0, &mvx, &mvy)) {
          t.pred |= 2;
          t.ref[1] = 0;
          t.mv[1][0] = static_cast<int16_t>(mvx);
          t.mv[1][1] = static_cast<int16_t>(mvy);
        }
        if (t.pred) cand[nc++] = t;
      }
      // combined bi-predictive candidates (B slices)
      const int num_orig = nc;
      if (sh.slice_type == 0 && num_orig > 1 && num_orig < sh.max_merge) {
        static const int l0i[12] = {0, 1, 0, 2, 1, 2, 0, 3, 1, 3, 2, 3};
        static const int l1i[12] = {1, 0, 2, 0, 2, 1, 3, 0, 3, 1, 3, 2};
        int comb = 0;
        while (comb < num_orig * (num_orig - 1) && nc < sh.max_merge) {
          const MvField& c0 = cand[l0i[comb]];
          const MvField& c1 = cand[l1i[comb]];
          if ((c0.pred & 1) && (c1.pred & 2) &&
              (ref_poc[0][c0.ref[0]] != ref_poc[1][c1.ref[1]] || ref_list[0][c0.ref[0]] != ref_list[1][c1.ref[1]] ||
               c0.mv[0][0] != c1.mv[1][0] || c0.mv[0][1] != c1.mv[1][1])) {
            MvField m{{{c0.mv[0][0], c0.mv[0][1]}, {c1.mv[1][0], c1.mv[1][1]}}, {c0.ref[0], c1.ref[1]}, 3, 0};
            cand[nc++] = m;
          }
          ++comb;
        }
      }
      // zero candidates
      const int nref = sh.slice_type == 1 ? sh.num_ref[0] : std::min(sh.num_ref[0], sh.num_ref[1]);
      int zero = 0;
      while (nc <= merge_idx) {
        const int r = zero < nref ? zero : 0;
        MvField m{{{0, 0}, {0, 0}}, {static_cast<int8_t>(r), static_cast<int8_t>(sh.slice_type == 0 ? r : -1)},
                  static_cast<uint8_t>(sh.slice_type == 0 ? 3 : 1), 0};
        cand[nc++] = m;
        ++zero;
      }
      out = cand[merge_idx];
    }
    // 8x4 / 4x8 PUs are uni-predicted
    if (out.pred == 3 && w0 + h0 == 12) {
      out.pred = 1;
      out.ref[1] = -1;
      out.mv[1][0] = out.mv[1][1] = 0;
    }
  }

  // ---------------------------------------------------------------- TMVP (8.5.3.2.8 / 8.5.3.2.9)
  bool temporal_mv(int xp, int yp, int w, int h, int X, int ref_idx, int* mvx, int* mvy) {
    if (!sh.tmvp) return false;
    const int cl = (sh.slice_type == 0 && !sh.col_from_l0) ? 1 : 0;
    StoredPic* col = ref_list[cl][sh.col_ref_idx];
    if (!col) return false;
    const int xbr = xp + w, ybr = yp + h;
    if ((yp >> log2_ctb) == (ybr >> log2_ctb) && ybr < H && xbr < W) {
      if (col_mv(col, (xbr >> 4) << 4, (ybr >> 4) << 4, X, ref_idx, mvx, mvy)) return true;
    }
    const int xc = xp + (w >> 1), yc = yp + (h >> 1);
    return col_mv(col, (xc >> 4) << 4, (yc >> 4) << 4, X, ref_idx, mvx, mvy);
  }
  bool col_mv(StoredPic* col, int x, int y, int X, int ref_idx, int* mvx, int* mvy) {
    if (x >= col->W || y >= col->H) return false;
    const MvField& m = col->mvf[static_cast<size_t>(y >> 2) * col->w4 + (x >> 2)];
    if (!m.pred) return false;
    int list;
    if (!(m.pred & 1)) list = 1;
    else if (m.pred == 1) list = 0;
    else list = nobackward ? X : (sh.col_from_l0 ? 1 : 0);
    const int cs = col->ctb_slice[static_cast<size_t>(y >> col->log2_ctb) * col->wctb + (x >> col->log2_ctb)];
    const SliceRefs& sr = col->slices[cs];
    const int rc = m.ref[list];
    const bool col_lt = sr.lt[list][rc] != 0;
    const bool cur_lt = ref_lt[X][ref_idx];
    if (col_lt != cur_lt) return false;
    int vx = m.mv[list][0], vy = m.mv[list][1];
    const int col_diff = col->poc - sr.poc[list][rc];
    const int cur_diff = poc - ref_poc[X][ref_idx];
    if (!cur_lt && col_diff != cur_diff && col_diff != 0) {
      scale_mv(col_diff, cur_diff, &vx, &vy);
    }
    *mvx = vx;
    *mvy = vy;
    return true;
  }
  static void scale_mv(int td0, int tb0, int* vx, int* vy) {
    const int td = clip3(-128, 127, td0), tb = clip3(-128, 127, tb0);
    const int tx = (16384 + (std::abs(td) >> 1)) / td;
    const int dsf = clip3(-4096, 4095, (tb * tx + 32) >> 6);
    auto sc = [&](int v) {
      const int p = dsf * v;
      return clip3(-32768, 32767, sgn(p) * ((std::abs(p) + 127) >> 8));
    };
    *vx = sc(*vx);
    *vy = sc(*vy);
  }

  // ---------------------------------------------------------------- AMVP (8.5.3.2.6 / 8.5.3.2.7)
  void amvp(int xp, int yp, int w, int h, int part_idx, int X, int ref_idx, int mvp_flag, int* mx, int* my) {
    const int ncbs = 1 << cu_log2;
    const int Y = 1 - X;
    const int target_poc = ref_poc[X][ref_idx];
    StoredPic* target = ref_list[X][ref_idx];
    const bool target_lt = ref_lt[X][ref_idx];
    auto av = [&](int xn, int yn) { return avail_pb(cu_x, cu_y, ncbs, xp, yp, w, h, part_idx, xn, yn); };
    // same reference picture, no scaling
    auto try_same = [&](int xn, int yn, int* vx, int* vy) {
      const MvField& m = cur->mvf[g4(xn, yn)];
      if ((m.pred & (1 << X)) && ref_list[X][m.ref[X]] == target) {
        *vx = m.mv[X][0];
        *vy = m.mv[X][1];
        return true;
      }
      if ((m.pred & (1 << Y)) && ref_list[Y][m.ref[Y]] == target) {
        *vx = m.mv[Y][0];
        *vy = m.mv[Y][1];
        return true;
      }
      return false;
    };
    // any reference of the same long-term-ness, scaled when both are short-term
    auto try_scaled = [&](int xn, int yn, int* vx, int* vy) {
      const MvField& m = cur->mvf[g4(xn, yn)];
      for (int k = 0; k < 2; ++k) {
        const int L = k == 0 ? X : Y;
        if (!(m.pred & (1 << L))) continue;
        const bool nlt = ref_lt[L][m.ref[L]];
        if (nlt != target_lt) continue;
        *vx = m.mv[L][0];
        *vy = m.mv[L][1];
        if (!nlt && !target_lt) {
          const int td = poc - ref_poc[L][m.ref[L]], tb = poc - target_poc;
          if (td != tb && td != 0) scale_mv(td, tb, vx, vy);
        }
        return true;
      }
      return false;
    };
    const int xa[2] = {xp - 1, xp - 1}, ya[2] = {yp + h, yp + h - 1};
    const bool ava[2] = {av(xa[0], ya[0]), av(xa[1], ya[1])};
    const bool is_scaled = ava[0] || ava[1];
    bool fa = false, fb = false;
    int ax = 0, ay = 0, bx = 0, by = 0;
    for (int k = 0; k < 2 && !fa; ++k)
      if (ava[k]) fa = try_same(xa[k], ya[k], &ax, &ay);
    for (int k = 0; k < 2 && !fa; ++k)
      if (ava[k]) fa = try_scaled(xa[k], ya[k], &ax, &ay);
    const int xb[3] = {xp + w, xp + w - 1, xp - 1}, yb = yp - 1;
    const bool avb[3] = {av(xb[0], yb), av(xb[1], yb), av(xb[2], yb)};
    for (int k = 0; k < 3 && !fb; ++k)
      if (avb[k]) fb = try_same(xb[k], yb, &bx, &by);
    if (!is_scaled && fb) {
      fa = true;
      ax = bx;
      ay = by;
    }
    if (!is_scaled) {
      fb = false;
      for (int k = 0; k < 3 && !fb; ++k)
        if (avb[k]) fb = try_scaled(xb[k], yb, &bx, &by);
    }
    int lx[3], ly[3], n = 0;
    if (fa) {
      lx[n] = ax;
      ly[n++] = ay;
    }
    if (fb && !(fa && ax == bx && ay == by)) {
      lx[n] = bx;
      ly[n++] = by;
    }
    if (n < 2) {
      int tx, ty;
      if (temporal_mv(xp, yp, w, h, X, ref_idx, &tx, &ty)) {
        lx[n] = tx;
        ly[n++] = ty;
      }
    }
    while (n < 2) {
      lx[n] = 0;
      ly[n++] = 0;
    }
    *mx = lx[mvp_flag];
    *my = ly[mvp_flag];
  }

  // ======================================================================== transform tree (7.3.8.8)
  void transform_tree(int x0, int y0, int xb, int yb, int log2, int depth, int blk, int max_depth, int intra_split,
                      int pcb, int pcr) {
    int split;
    if (log2 <= log2_max_tb && log2 > log2_min_tb && depth < max_depth && !(intra_split && depth == 0)) {
      split = eng.decode(ctx[C_SPLIT_TF + 5 - log2]);
    } else {
      const bool inter_split = sps->depth_inter == 0 && !cu_intra && cu_part != P_2Nx2N && depth == 0;
      split = log2 > log2_max_tb || (intra_split && depth == 0) || inter_split;
    }
    int cb = 0, cr = 0;
    if (log2 > 2) {
      if (depth == 0 || pcb) cb = eng.decode(ctx[C_CBF_CHROMA + depth]);
      if (depth == 0 || pcr) cr = eng.decode(ctx[C_CBF_CHROMA + depth]);
    } else {
      cb = pcb;  // 4x4 luma TUs: chroma coded at blkIdx 3 with the parent's flags
      cr = pcr;
    }
    if (split) {
      const int h = 1 << (log2 - 1);
      for (int k = 0; k < 4; ++k)
        transform_tree(x0 + (k & 1) * h, y0 + (k >> 1) * h, x0, y0, log2 - 1, depth + 1, k, max_depth, intra_split, cb, cr);
      return;
    }
    int cbf_luma = 1;
    if (cu_intra || depth != 0 || cb || cr) cbf_luma = eng.decode(ctx[C_CBF_LUMA + (depth == 0 ? 1 : 0)]);
    transform_unit(x0, y0, xb, yb, log2, depth, blk, cbf_luma, cb, cr);
  }

  // 7.3.8.10 transform_unit() + reconstruction of the TU
  void transform_unit(int x0, int y0, int xb, int yb, int log2, int depth, int blk, int cbf_luma, int cb, int cr) {
    const int n = 1 << log2;
    (void)depth;
    // transform edges
    for (int k = 0; k < n; k += 4) {
      edge[g4(x0, y0 + k)] |= E_TU_V;
      edge[g4(x0 + k, y0)] |= E_TU_H;
    }
    if (cbf_luma)
      for (int y = y0; y < y0 + n; y += 4)
        for (int x = x0; x < x0 + n; x += 4) cbf_y[g4(x, y)] = 1;
    const bool chroma_here = log2 > 2;
    const bool chroma_blk3 = log2 == 2 && blk == 3;
    if (cbf_luma || cb || cr) {
      if (pps->cu_qp_delta && !qp_delta_coded) parse_qp_delta(x0, y0);
    }
    const int mode_y = cu_intra ? static_cast<int>(ipm[g4(x0, y0)]) : -1;
    const int mode_c = cu_intra ? cu_chroma_mode : -1;
    // luma
    residual_and_recon(x0, y0, log2, 0, cbf_luma, mode_y);
    if (enc_rec && log2 > 2 && depth > 0 && !cu_intra) {
      for (int gy = y0; gy < y0 + n; gy += 8)
        for (int gx = x0; gx < x0 + n; gx += 8) enc_cu_at(gx, gy).flags |= 16;
    }
    if (chroma_here) {
      residual_and_recon(x0 / 2, y0 / 2, log2 - 1, 1, cb, mode_c);
      residual_and_recon(x0 / 2, y0 / 2, log2 - 1, 2, cr, mode_c);
    } else if (chroma_blk3) {
      residual_and_recon(xb / 2, yb / 2, 2, 1, cb, mode_c);
      residual_and_recon(xb / 2, yb / 2, 2, 2, cr, mode_c);
    }
  }

  // cu_qp_delta_abs / sign (7.3.8.14, 9.3.3.10) -> QpY (8.6.1)
  void parse_qp_delta(int x0, int y0) {
    int a = 0;
    while (a < 5 && eng.decode(ctx[C_QP_DELTA + (a > 0)])) ++a;
    if (a == 5) {
      int k = 0;
      while (eng.bypass()) {
        a += 1 << k;
        if (++k > 30) fail("cu_qp_delta_abs suffix too long");
      }
      while (k--) a += eng.bypass() << k;
    }
    const int d = a && eng.bypass() ? -a : a;
    if (d < -(26 + qp_bd / 2) || d > 25 + qp_bd / 2) fail("CuQpDeltaVal out of range");
    qp_delta_coded = true;
    cu_qp = ((qg_pred + d + 52 + 2 * qp_bd) % (52 + qp_bd)) - qp_bd;
    if (enc_rec)
      for_qg_blocks([&](CtuInfo& t) {
        t.qp = static_cast<int8_t>(cu_qp);
        t.qp_first = static_cast<uint8_t>(zorder8((x0 & 31) >> 3, (y0 & 31) >> 3));
      });
  }

  int qp_prime(int cidx) const {
    if (cidx == 0) return cu_qp + qp_bd;
    const int off = cidx == 1 ? pps->cb_qp_off + sh.cb_qp_off : pps->cr_qp_off + sh.cr_qp_off;
    const int qpi = clip3(-qp_bd_c, 57, cu_qp + off);
    return chroma_qp_map(qpi) + qp_bd_c;
  }

  // residual_coding() (when coded), then the CPU reconstruction and the GPU records of the TB
  int16_t lev[32 * 32];
  void residual_and_recon(int x0, int y0, int log2, int cidx, int cbf, int intra_mode) {
    const int n = 1 << log2;
    bool tskip = false;
    if (cbf) {
      std::memset(lev, 0, sizeof(int16_t) * n * n);
      tskip = residual_coding(x0, y0, log2, cidx, intra_mode);
    }
    const bool intra = intra_mode >= 0;
    uint32_t tu = 0xFFFFFFFFu;
    if (cbf && opt.gpu_records) {
      uint8_t fl = 0;
      if (intra && cidx == 0 && log2 == 2) fl |= DT_DST;
      if (tskip) fl |= DT_TSKIP;
      if (cu_bypass) fl |= DT_BYPASS;
      if (intra) fl |= DT_INTRA;
      if (sps->scaling_enabled) fl |= DT_SCALING;
      tu = push_tu(x0, y0, log2, cidx, qp_prime(cidx), fl, lev);
    }
    if (enc_rec && cbf) {
      std::vector<int16_t>& pl = cidx == 0 ? dp->coef_y : (cidx == 1 ? dp->coef_cb : dp->coef_cr);
      const int stride = cidx ? W / 2 : W;
      for (int y = 0; y < n; ++y)
        for (int x = 0; x < n; ++x) pl[static_cast<size_t>(y0 + y) * stride + x0 + x] = lev[y * n + x];
    }
    if (intra && opt.gpu_records) push_op(x0, y0, log2, cidx, static_cast<uint8_t>(intra_mode), tu);
    if (opt.recon) {
      if (intra) predict_intra(x0, y0, log2, cidx, intra_mode);
      if (cbf) add_residual(x0, y0, log2, cidx, intra, tskip);
    }
  }

  uint32_t push_tu(int x, int y, int log2, int cidx, int qp, uint8_t flags, const int16_t* c) {
    DecPicture& d = *dp;
    const int n = 1 << log2;
    DecTu t;
    t.x = static_cast<uint16_t>(x);
    t.y = static_cast<uint16_t>(y);
    t.log2 = static_cast<uint8_t>(log2);
    t.cidx = static_cast<uint8_t>(cidx);
    t.qp = static_cast<uint8_t>(qp);
    t.flags = flags;
    // sparse levels: a 64-bit mask of the coded 4x4 coefficient groups (raster over the
    // block, as 4 uint16 words), then the 16 levels (raster) of each coded group
    t.coef = static_cast<uint32_t>(d.coefs.size());
    const int g = n >> 2;
    uint64_t mask = 0;
    for (int cg = 0; cg < g * g; ++cg) {
      const int16_t* p = c + (cg / g) * 4 * n + (cg % g) * 4;
      uint64_t any = 0;
      for (int r = 0; r < 4; ++r) {
        uint64_t w;
        std::memcpy(&w, p + r * n, 8);
        any |= w;
      }
      if (any) mask |= 1ull << cg;
    }
    const size_t at = d.coefs.size();
    d.coefs.resize(at + 4 + 16 * static_cast<size_t>(__builtin_popcountll(mask)));
    int16_t* o = d.coefs.data() + at;
    for (int k = 0; k < 4; ++k) o[k] = static_cast<int16_t>(static_cast<uint16_t>(mask >> (16 * k)));
    o += 4;
    for (int cg = 0; cg < g * g; ++cg) {
      if (!((mask >> cg) & 1)) continue;
      const int16_t* p = c + (cg / g) * 4 * n + (cg % g) * 4;
      for (int r = 0; r < 4; ++r) std::memcpy(o + r * 4, p + r * n, 8);
      o += 16;
    }
    d.tus.push_back(t);
    return static_cast<uint32_t>(d.tus.size() - 1);
  }
  void push_op(int x, int y, int log2, int cidx, uint8_t mode, uint32_t tu) {
    DecIntraOp o;
    o.x = static_cast<uint16_t>(x);
    o.y = static_cast<uint16_t>(y);
    o.log2 = static_cast<uint8_t>(log2);
    o.cidx = static_cast<uint8_t>(cidx);
    o.mode = mode;
    o.flags = 0;
    o.tu = tu;
    ctb_ops[ctb_addr_rs].push_back(o);
  }

  // ---------------------------------------------------------------- residual_coding (7.3.8.11)
  // returns transform_skip_flag
  bool residual_coding(int x0, int y0, int log2, int cidx, int intra_mode) {
    (void)x0;
    (void)y0;
    const int n = 1 << log2;
    bool tskip = false;
    if (pps->transform_skip && !cu_bypass && log2 <= 2) tskip = eng.decode(ctx[C_TSKIP + (cidx ? 1 : 0)]);
    int scan = 0;
    if (intra_mode >= 0 && (log2 == 2 || (log2 == 3 && cidx == 0))) {
      if (intra_mode >= 6 && intra_mode <= 14) scan = 2;
      else if (intra_mode >= 22 && intra_mode <= 30) scan = 1;
    }
    int lx = last_prefix(log2, cidx, C_LAST_X);
    int ly = last_prefix(log2, cidx, C_LAST_Y);
    lx = last_suffix(lx);
    ly = last_suffix(ly);
    if (lx >= n || ly >= n) fail("last significant position outside the block");
    if (scan == 2) std::swap(lx, ly);
    const int log2sb = log2 - 2, nsb = 1 << log2sb;
    const uint8_t *sbx = kScan.x[scan][log2sb], *sby = kScan.y[scan][log2sb];
    const uint8_t *px = kScan.x[scan][2], *py = kScan.y[scan][2];
    const int last_sb = kScan.inv[scan][log2sb][((ly >> 2) << log2sb) + (lx >> 2)];
    const int last_pos = kScan.inv[scan][2][((ly & 3) << 2) + (lx & 3)];
    uint8_t csbf[8][8] = {};
    int g1ctx_prev = 1;
    bool first_sb = true;
    const bool sdh = pps->sign_hiding && !cu_bypass;
    for (int i = last_sb; i >= 0; --i) {
      const int xs = sbx[i], ys = sby[i];
      bool infer_dc = false;
      if (i < last_sb && i > 0) {
        int cs = 0;
        if (xs < nsb - 1) cs += csbf[xs + 1][ys];
        if (ys < nsb - 1) cs += csbf[xs][ys + 1];
        csbf[xs][ys] = static_cast<uint8_t>(eng.decode(ctx[C_CSBF + std::min(cs, 1) + (cidx ? 2 : 0)]));
        infer_dc = true;
      } else {
        csbf[xs][ys] = 1;
      }
      int prev_csbf = 0;
      if (xs < nsb - 1) prev_csbf += csbf[xs + 1][ys];
      if (ys < nsb - 1) prev_csbf += csbf[xs][ys + 1] << 1;
      const uint8_t* sig_row = kSigCtx.t[cidx ? 1 : 0][log2 - 2][scan][prev_csbf][(xs | ys) ? 1 : 0];
      int sig[16] = {};
      if (i == last_sb) sig[last_pos] = 1;
      for (int p = (i == last_sb ? last_pos - 1 : 15); p >= 0; --p) {
        if (csbf[xs][ys] && (p > 0 || !infer_dc)) {
          sig[p] = eng.decode(ctx[C_SIG + sig_row[(py[p] << 2) + px[p]]]);
          if (sig[p]) infer_dc = false;
        } else if (p == 0 && infer_dc && csbf[xs][ys]) {
          sig[p] = 1;
        }
      }
      if (!csbf[xs][ys]) continue;
      int ctx_set = (i == 0 || cidx > 0) ? 0 : 2;
      if (!first_sb && g1ctx_prev == 0) ++ctx_set;
      int g1ctx = 1;
      int g1[16] = {}, g2[16] = {};
      int num_g1 = 0, last_g1 = -1;
      bool any = false;
      for (int p = 15; p >= 0; --p) {
        if (!sig[p]) continue;
        any = true;
        if (num_g1 < 8) {
          g1[p] = eng.decode(ctx[C_GT1 + (cidx ? 16 : 0) + ctx_set * 4 + g1ctx]);
          ++num_g1;
          if (g1[p]) {
            g1ctx = 0;
            if (last_g1 < 0) last_g1 = p;
          } else if (g1ctx > 0 && g1ctx < 3) {
            ++g1ctx;
          }
        }
      }
      if (any) {
        first_sb = false;
        g1ctx_prev = g1ctx;
      }
      if (last_g1 >= 0) g2[last_g1] = eng.decode(ctx[C_GT2 + (cidx ? 4 : 0) + ctx_set]);
      int first_sig = -1, last_sig = -1;
      for (int p = 0; p < 16; ++p)
        if (sig[p]) {
          if (first_sig < 0) first_sig = p;
          last_sig = p;
        }
      const bool hidden = sdh && first_sig >= 0 && last_sig - first_sig > 3;
      int sign[16] = {};
      for (int p = 15; p >= 0; --p)
        if (sig[p] && !(hidden && p == first_sig)) sign[p] = eng.bypass();
      int num_sig = 0, rice = 0, sum = 0;
      for (int p = 15; p >= 0; --p) {
        if (!sig[p]) continue;
        const int base = 1 + g1[p] + g2[p];
        int a = base;
        const int thr = num_sig < 8 ? (p == last_g1 ? 3 : 2) : 1;
        if (base == thr) {
          a = base + remaining(rice);
          if (a > 3 * (1 << rice)) rice = std::min(rice + 1, 4);
        }
        ++num_sig;
        sum += a;
        if (hidden && p == first_sig) sign[p] = sum & 1;
        lev[(ys * 4 + py[p]) * n + xs * 4 + px[p]] = static_cast<int16_t>(clip3(-32768, 32767, sign[p] ? -a : a));
      }
    }
    return tskip;
  }
  int last_prefix(int log2, int cidx, int base) {
    int off, shift;
    if (cidx == 0) {
      off = 3 * (log2 - 2) + ((log2 - 1) >> 2);
      shift = (log2 + 1) >> 2;
    } else {
      off = 15;
      shift = log2 - 2;
    }
    const int cmax = (log2 << 1) - 1;
    int v = 0;
    while (v < cmax && eng.decode(ctx[base + off + (v >> shift)])) ++v;
    return v;
  }
  int last_suffix(int prefix) {
    if (prefix <= 3) return prefix;
    const int nb = (prefix >> 1) - 1;
    return (1 << nb) * (2 + (prefix & 1)) + static_cast<int>(eng.bypass_bits(nb));
  }
  int remaining(int rice) {
    int prefix = 0;
    while (prefix < 32 && eng.bypass()) ++prefix;
    if (prefix <= 3) return (prefix << rice) + static_cast<int>(eng.bypass_bits(rice));
    const int k = prefix - 3 + rice;
    if (k > 31) fail("coeff_abs_level_remaining too long");
    return (((1 << (prefix - 3)) + 2) << rice) + static_cast<int>(eng.bypass_bits(k));
  }
  static int sig_ctx(int xc, int yc, int log2, int cidx, int scan, int prev_csbf, int xs, int ys) {
    static const int map4[15] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8};
    int s;
    if (log2 == 2) {
      s = map4[(yc << 2) + xc];
    } else if (xc + yc == 0) {
      s = 0;
    } else {
      const int xp = xc & 3, yp = yc & 3;
      switch (prev_csbf) {
        case 0: s = (xp + yp == 0) ? 2 : (xp + yp < 3) ? 1 : 0; break;
        case 1: s = yp == 0 ? 2 : (yp == 1 ? 1 : 0); break;
        case 2: s = xp == 0 ? 2 : (xp == 1 ? 1 : 0); break;
        default: s = 2;
      }
      if (cidx == 0) {
        if (xs > 0 || ys > 0) s += 3;
        if (log2 == 3) s += scan == 0 ? 9 : 15;
        else s += 21;
      } else {
        s += log2 == 3 ? 9 : 12;
      }
    }
    return cidx == 0 ? s : 27 + s;
  }
  // sig_coeff_flag ctxInc (9.3.4.2.5) of every (chroma, log2 - 2, scanIdx, prevCsbf, sub-block
  // not the first, raster position in the sub-block), from sig_ctx once
  struct SigCtxTable {
    uint8_t t[2][4][3][4][2][16];
    SigCtxTable() : t() {
      for (int c = 0; c < 2; ++c)
        for (int l = 0; l < 4; ++l)
          for (int sc = 0; sc < 3; ++sc)
            for (int pc = 0; pc < 4; ++pc)
              for (int nf = 0; nf < 2; ++nf)
                for (int q = 0; q < 16; ++q) {
                  if (l == 0 && (nf || q == 15)) continue;  // one sub-block; (3, 3) is never a sig_coeff_flag
                  const int xs = nf, ys = 0;
                  t[c][l][sc][pc][nf][q] =
                      static_cast<uint8_t>(sig_ctx(xs * 4 + (q & 3), ys * 4 + (q >> 2), l + 2, c, sc, pc, xs, ys));
                }
    }
  };
  inline static const SigCtxTable kSigCtx;

  // ======================================================================== CPU reconstruction
  // 8.6.2 - 8.6.4: scaling, transform (or skip / bypass), residual added to the prediction
  void add_residual(int x0, int y0, int log2, int cidx, bool intra, bool tskip) {
    const int n = 1 << log2;
    const int bdv = cidx ? bdc : bd, mx = cidx ? maxvc : maxv;
    const int stride = cidx ? W / 2 : W;
    int r[32 * 32];
    if (cu_bypass) {
      for (int i = 0; i < n * n; ++i) r[i] = lev[i];
    } else {
      const int qp = qp_prime(cidx);
      const int bdshift = bdv + log2 - 5;
      const bool use_sl = sps->scaling_enabled && !(tskip && log2 > 2);
      const uint8_t* sl = nullptr;
      if (use_sl) {
        const ScalingList& L = pps->scaling_present ? pps->scaling : sps->scaling;
        sl = L.f.data() + kScalingOff[log2 - 2] + ((intra ? 0 : 3) + cidx) * n * n;
      }
      int d[32 * 32];
      for (int i = 0; i < n * n; ++i) {
        const int m = sl ? sl[i] : 16;
        const int64_t v = (static_cast<int64_t>(lev[i]) * m * kLevelScale[qp % 6] << (qp / 6)) + (1LL << (bdshift - 1));
        d[i] = clip3(-32768, 32767, static_cast<int>(v >> bdshift));
      }
      const int sh2 = 20 - bdv;
      if (tskip) {
        const int ts = 5 + log2;
        for (int i = 0; i < n * n; ++i) r[i] = ((d[i] << ts) + (1 << (sh2 - 1))) >> sh2;
      } else {
        const bool dst = intra && cidx == 0 && log2 == 2;
        const int step = 32 >> log2;
        auto c = [&](int k, int m) { return dst ? static_cast<int>(kDst4[k][m]) : dct_coef(k * step, m); };
        int e[32 * 32];
        for (int x = 0; x < n; ++x)
          for (int y = 0; y < n; ++y) {
            int64_t s = 0;
            for (int k = 0; k < n; ++k) s += static_cast<int64_t>(c(k, y)) * d[k * n + x];
            e[y * n + x] = clip3(-32768, 32767, static_cast<int>((s + 64) >> 7));
          }
        for (int y = 0; y < n; ++y)
          for (int x = 0; x < n; ++x) {
            int64_t s = 0;
            for (int k = 0; k < n; ++k) s += static_cast<int64_t>(c(k, x)) * e[y * n + k];
            r[y * n + x] = static_cast<int>((s + (1LL << (sh2 - 1))) >> sh2);
          }
      }
    }
    uint16_t* pl = cur->pl[cidx].data() + static_cast<size_t>(y0) * stride + x0;
    for (int y = 0; y < n; ++y)
      for (int x = 0; x < n; ++x) pl[y * stride + x] = static_cast<uint16_t>(clip3(0, mx, pl[y * stride + x] + r[y * n + x]));
  }

  // 8.4.4.2 intra sample prediction of one transform block
  void predict_intra(int x0, int y0, int log2, int cidx, int mode) {
    const int n = 1 << log2;
    const int stride = cidx ? W / 2 : W;
    const int sc = cidx ? 1 : 0;
    const int bdv = cidx ? bdc : bd, mx = cidx ? maxvc : maxv;
    uint16_t* pl = cur->pl[cidx].data();
    const int total = 4 * n + 1;
    int p[129], av[129];
    const int xl = x0 << sc, yl = y0 << sc;  // luma location of the block
    int navail = 0;
    for (int i = 0; i < total; ++i) {
      int xc, yc;
      if (i < 2 * n) {
        xc = x0 - 1;
        yc = y0 + 2 * n - 1 - i;
      } else if (i == 2 * n) {
        xc = x0 - 1;
        yc = y0 - 1;
      } else {
        xc = x0 + (i - 2 * n - 1);
        yc = y0 - 1;
      }
      const int xn = xc << sc, yn = yc << sc;
      bool a = avail_z(xl, yl, xn, yn);
      if (a && pps->constrained_intra && !(cu_flags[g4(xn, yn)] & CF_INTRA)) a = false;
      av[i] = a;
      if (a) {
        p[i] = pl[static_cast<size_t>(yc) * stride + xc];
        ++navail;
      }
    }
    if (navail == 0) {
      for (int i = 0; i < total; ++i) p[i] = 1 << (bdv - 1);
    } else {
      if (!av[0])
        for (int i = 1; i < total; ++i)
          if (av[i]) {
            p[0] = p[i];
            break;
          }
      for (int i = 1; i < total; ++i)
        if (!av[i]) p[i] = p[i - 1];
    }
    auto L = [&](int y) { return p[2 * n - 1 - y]; };
    auto T = [&](int x) { return p[2 * n + 1 + x]; };
    if (cidx == 0 && mode != 1 && n != 4) {
      const int md = std::min(std::abs(mode - 26), std::abs(mode - 10));
      const int thr = n == 8 ? 7 : (n == 16 ? 1 : 0);
      if (md > thr) {
        int f[129];
        const int tl = T(-1), bl = L(2 * n - 1), tr = T(2 * n - 1);
        const bool bi = sps->strong_intra && n == 32 && std::abs(tl + tr - 2 * T(n - 1)) < (1 << (bdv - 5)) &&
                        std::abs(tl + bl - 2 * L(n - 1)) < (1 << (bdv - 5));
        if (bi) {
          f[2 * n] = tl;
          for (int y = 0; y < 63; ++y) f[2 * n - 1 - y] = ((63 - y) * tl + (y + 1) * bl + 32) >> 6;
          f[0] = bl;
          for (int x = 0; x < 63; ++x) f[2 * n + 1 + x] = ((63 - x) * tl + (x + 1) * tr + 32) >> 6;
          f[total - 1] = tr;
        } else {
          f[0] = p[0];
          f[total - 1] = p[total - 1];
          for (int i = 1; i < total - 1; ++i) f[i] = (p[i - 1] + 2 * p[i] + p[i + 1] + 2) >> 2;
        }
        std::memcpy(p, f, sizeof(int) * total);
      }
    }
    uint16_t* dst = pl + static_cast<size_t>(y0) * stride + x0;
    if (mode == 0) {
      for (int y = 0; y < n; ++y)
        for (int x = 0; x < n; ++x)
          dst[y * stride + x] =
              static_cast<uint16_t>(((n - 1 - x) * L(y) + (x + 1) * T(n) + (n - 1 - y) * T(x) + (y + 1) * L(n) + n) >> (log2 + 1));
      return;
    }
    if (mode == 1) {
      int s = n;
      for (int i = 0; i < n; ++i) s += T(i) + L(i);
      const int dc = s >> (log2 + 1);
      for (int y = 0; y < n; ++y)
        for (int x = 0; x < n; ++x) dst[y * stride + x] = static_cast<uint16_t>(dc);
      if (cidx == 0 && n < 32) {
        dst[0] = static_cast<uint16_t>((L(0) + 2 * dc + T(0) + 2) >> 2);
        for (int x = 1; x < n; ++x) dst[x] = static_cast<uint16_t>((T(x) + 3 * dc + 2) >> 2);
        for (int y = 1; y < n; ++y) dst[y * stride] = static_cast<uint16_t>((L(y) + 3 * dc + 2) >> 2);
      }
      return;
    }
    const int ang = kIntraPredAngle[mode];
    int refa[3 * 32 + 2];
    int* ref = refa + n;
    if (mode >= 18) {
      for (int x = 0; x <= n; ++x) ref[x] = T(x - 1);
      if (ang < 0) {
        if ((n * ang) >> 5 < -1)
          for (int x = (n * ang) >> 5; x <= -1; ++x) ref[x] = L(-1 + ((x * kInvAngle[mode - 11] + 128) >> 8));
      } else {
        for (int x = n + 1; x <= 2 * n; ++x) ref[x] = T(x - 1);
      }
      for (int y = 0; y < n; ++y) {
        const int idx = ((y + 1) * ang) >> 5, fact = ((y + 1) * ang) & 31;
        for (int x = 0; x < n; ++x)
          dst[y * stride + x] = static_cast<uint16_t>(
              fact ? ((32 - fact) * ref[x + idx + 1] + fact * ref[x + idx + 2] + 16) >> 5 : ref[x + idx + 1]);
      }
      if (mode == 26 && cidx == 0 && n < 32)
        for (int y = 0; y < n; ++y) dst[y * stride] = static_cast<uint16_t>(clip3(0, mx, T(0) + ((L(y) - L(-1)) >> 1)));
    } else {
      for (int x = 0; x <= n; ++x) ref[x] = L(x - 1);
      if (ang < 0) {
        if ((n * ang) >> 5 < -1)
          for (int x = (n * ang) >> 5; x <= -1; ++x) ref[x] = T(-1 + ((x * kInvAngle[mode - 11] + 128) >> 8));
      } else {
        for (int x = n + 1; x <= 2 * n; ++x) ref[x] = L(x - 1);
      }
      for (int x = 0; x < n; ++x) {
        const int idx = ((x + 1) * ang) >> 5, fact = ((x + 1) * ang) & 31;
        for (int y = 0; y < n; ++y)
          dst[y * stride + x] = static_cast<uint16_t>(
              fact ? ((32 - fact) * ref[y + idx + 1] + fact * ref[y + idx + 2] + 16) >> 5 : ref[y + idx + 1]);
      }
      if (mode == 10 && cidx == 0 && n < 32)
        for (int x = 0; x < n; ++x) dst[x] = static_cast<uint16_t>(clip3(0, mx, L(0) + ((T(x) - T(-1)) >> 1)));
    }
  }

  // 8.5.3.3 fractional sample interpolation + weighted sample prediction of one PU
  void predict_inter(int xp, int yp, int w, int h, const MvField& mf) {
    for (int c = 0; c < 3; ++c) {
      const int bdv = c ? bdc : bd, mx = c ? maxvc : maxv;
      const int pw = c ? W / 2 : W, ph = c ? H / 2 : H;
      const int bw = c ? w / 2 : w, bh = c ? h / 2 : h;
      const int bx = c ? xp / 2 : xp, by = c ? yp / 2 : yp;
      int pred[2][64 * 64];
      for (int l = 0; l < 2; ++l) {
        if (!(mf.pred & (1 << l))) continue;
        const StoredPic* rp = ref_list[l][mf.ref[l]];
        if (!rp || rp->pl[c].empty()) fail("reference picture without samples");
        mc_block(rp->pl[c].data(), pw, ph, bx, by, bw, bh, mf.mv[l][0], mf.mv[l][1], c, bdv, pred[l]);
      }
      uint16_t* dst = cur->pl[c].data();
      const int shift1 = 14 - bdv;
      const bool bi = mf.pred == 3;
      const int l0 = (mf.pred & 1) ? 0 : 1;
      if (!sh.weighted) {
        for (int y = 0; y < bh; ++y)
          for (int x = 0; x < bw; ++x) {
            int v;
            if (bi) {
              const int sh2 = 15 - bdv;
              v = (pred[0][y * bw + x] + pred[1][y * bw + x] + (1 << (sh2 - 1))) >> sh2;
            } else {
              v = (pred[l0][y * bw + x] + (shift1 > 0 ? 1 << (shift1 - 1) : 0)) >> shift1;
            }
            dst[static_cast<size_t>(by + y) * pw + bx + x] = static_cast<uint16_t>(clip3(0, mx, v));
          }
      } else {
        const int log2wd = (c ? sh.pw.log2_denom_c : sh.pw.log2_denom_y) + shift1;
        const int ofs = 1 << (bdv - 8);
        for (int y = 0; y < bh; ++y)
          for (int x = 0; x < bw; ++x) {
            int v;
            if (bi) {
              const int w0 = sh.pw.w[0][mf.ref[0]][c], w1 = sh.pw.w[1][mf.ref[1]][c];
              const int o0 = sh.pw.o[0][mf.ref[0]][c] * ofs, o1 = sh.pw.o[1][mf.ref[1]][c] * ofs;
              v = (pred[0][y * bw + x] * w0 + pred[1][y * bw + x] * w1 + ((o0 + o1 + 1) << log2wd)) >> (log2wd + 1);
            } else {
              const int w0 = sh.pw.w[l0][mf.ref[l0]][c], o0 = sh.pw.o[l0][mf.ref[l0]][c] * ofs;
              if (log2wd >= 1) v = ((pred[l0][y * bw + x] * w0 + (1 << (log2wd - 1))) >> log2wd) + o0;
              else v = pred[l0][y * bw + x] * w0 + o0;
            }
            dst[static_cast<size_t>(by + y) * pw + bx + x] = static_cast<uint16_t>(clip3(0, mx, v));
          }
      }
    }
  }
  static void mc_block(const uint16_t* rp, int pw, int ph, int bx, int by, int bw, int bh, int mvx, int mvy, int c, int bdv,
                       int* out) {
    const int fx = c ? (mvx & 7) : (mvx & 3), fy = c ? (mvy & 7) : (mvy & 3);
    const int ix = c ? (mvx >> 3) : (mvx >> 2), iy = c ? (mvy >> 3) : (mvy >> 2);
    const int sh1 = std::min(4, bdv - 8), sh3 = 14 - bdv;
    auto R = [&](int x, int y) { return static_cast<int>(rp[static_cast<size_t>(clip3(0, ph - 1, y)) * pw + clip3(0, pw - 1, x)]); };
    const int ntap = c ? 4 : 8, half = c ? 1 : 3;
    auto tap = [&](int f, int i) { return c ? kChromaTaps[f][i] : kLumaTaps[f][i]; };
    for (int y = 0; y < bh; ++y)
      for (int x = 0; x < bw; ++x) {
        const int xi = bx + x + ix, yi = by + y + iy;
        int v;
        if (fx == 0 && fy == 0) {
          v = R(xi, yi) << sh3;
        } else if (fy == 0) {
          int s = 0;
          for (int i = 0; i < ntap; ++i) s += tap(fx, i) * R(xi + i - half, yi);
          v = s >> sh1;
        } else if (fx == 0) {
          int s = 0;
          for (int i = 0; i < ntap; ++i) s += tap(fy, i) * R(xi, yi + i - half);
          v = s >> sh1;
        } else {
          int s = 0;
          for (int j = 0; j < ntap; ++j) {
            int t = 0;
            for (int i = 0; i < ntap; ++i) t += tap(fx, i) * R(xi + i - half, yi + j - half);
            s += tap(fy, j) * (t >> sh1);
          }
          v = s >> 6;
        }
        out[y * bw + x] = v;
      }
  }

  // ======================================================================== picture end
  void finish_picture() {
    if (!pic_open) return;
    pic_open = false;
    for (int r = 0; r < nctb; ++r)
      if (ctb_slice[r] < 0) fail("picture has undecoded CTBs");
    if (sao_params.size() != static_cast<size_t>(nctb)) sao_params.assign(nctb, DecSao{});
    DecPicture& d = *dp;
    // deblocking boundary strengths (8.7.2.4), shared by the CPU filter and the GPU records
    std::vector<uint8_t> bsv(static_cast<size_t>(w4) * h4, 0);
    compute_bs(bsv);
    bool any_deblock = false, any_sao = false;
    for (const SliceHeader& s : slices) {
      any_deblock |= !s.deblock_disabled;
      any_sao |= s.sao_luma || s.sao_chroma;
    }
    d.deblock_any = any_deblock;
    d.sao_any = any_sao && sps->sao;
    d.slice_qp = pps->init_qp + slices[0].qp_delta;
    if (opt.gpu_records) {
      d.bs = bsv;
      std::vector<int> ref_base(2 * slices.size());  // slice_ref_base of every (slice, list)
      for (size_t s = 0; s < slices.size(); ++s)
        for (int l = 0; l < 2; ++l) ref_base[2 * s + l] = slice_ref_base(static_cast<int>(s), l);
      // the GPU record of 4x4 block k (slice segment sidx)
      auto rec4 = [&](size_t k, int sidx, DecMv4& m) {
        const MvField& f = cur->mvf[k];
        m.qp = qp_y[k];
        m.flags = 0;
        if (cu_flags[k] & CF_INTRA) m.flags |= DM_INTRA;
        if (no_filter(k)) m.flags |= DM_NOFILTER;
        m.ref[0] = m.ref[1] = 0xFF;
        if (f.pred) {
          m.flags |= DM_INTER;
          for (int l = 0; l < 2; ++l)
            if (f.pred & (1 << l)) {
              m.ref[l] = static_cast<uint8_t>(ref_base[2 * sidx + l] + f.ref[l]);
              m.mv[l][0] = f.mv[l][0];
              m.mv[l][1] = f.mv[l][1];
            } else {
              m.mv[l][0] = m.mv[l][1] = 0;
            }
        } else {
          m.mv[0][0] = m.mv[0][1] = m.mv[1][0] = m.mv[1][1] = 0;
        }
      };
      // 8x8 records: a coding block is >= 8x8, so flags and QpY are uniform per 8x8; only
      // 8x4 / 4x8 prediction blocks differ inside one -- those become DM_SPLIT records whose
      // first 4 bytes index 4 per-4x4 records (raster) in mvf_sub.  Built straight from the
      // 4x4 motion field (an 8x8 block lies in one CTB, so in one slice segment)
      const int w8 = w4 / 2, h8 = h4 / 2;
      d.mvf.resize(static_cast<size_t>(w8) * h8);
      for (int by = 0; by < h8; ++by)
        for (int bx = 0; bx < w8; ++bx) {
          const int sidx = ctb_slice[((by * 8) >> log2_ctb) * wctb + ((bx * 8) >> log2_ctb)];
          const size_t k0 = static_cast<size_t>(2 * by) * w4 + 2 * bx;
          DecMv4 c[4] = {};
          rec4(k0, sidx, c[0]);
          rec4(k0 + 1, sidx, c[1]);
          rec4(k0 + w4, sidx, c[2]);
          rec4(k0 + w4 + 1, sidx, c[3]);
          DecMv4& o = d.mvf[static_cast<size_t>(by) * w8 + bx];
          o = c[0];
          bool same = true;
          for (int i = 1; i < 4; ++i) same = same && std::memcmp(&c[i], &c[0], sizeof(DecMv4)) == 0;
          if (same) continue;
          const uint32_t idx = static_cast<uint32_t>(d.mvf_sub.size() / 4);
          std::memcpy(o.mv, &idx, 4);
          o.flags |= DM_SPLIT;
          for (int i = 0; i < 4; ++i) d.mvf_sub.push_back(c[i]);
        }
      uint32_t off = 0;
      for (int r = 0; r < nctb; ++r) {
        d.ops_off[r] = off;
        d.ops.insert(d.ops.end(), ctb_ops[r].begin(), ctb_ops[r].end());
        off += static_cast<uint32_t>(ctb_ops[r].size());
      }
      d.ops_off[nctb] = off;
    }
    if (opt.recon && !opt.skip_filters) {
      if (any_deblock) deblock(bsv);
      if (d.sao_any) apply_sao();
    }
    if (opt.recon) {
      d.y = cur->pl[0];
      d.u = cur->pl[1];
      d.v = cur->pl[2];
    }
    sao_params.clear();
    // the picture enters the DPB as a short-term reference
    cur->is_ref = true;
    dpb.push_back(cur);
    cur.reset();
    dp = nullptr;
  }

  int slice_ref_base(int sidx, int l) const {
    // GPU reference entries were appended per slice segment: L0 entries then L1 entries
    int base = 0;
    for (int s = 0; s < sidx; ++s) base += slices[s].num_ref[0] + slices[s].num_ref[1];
    return base + (l == 1 ? slices[sidx].num_ref[0] : 0);
  }

  bool no_filter(size_t k) const {
    const uint8_t f = cu_flags[k];
    return (f & CF_BYPASS) || ((f & CF_PCM) && sps->pcm_loop_filter_disabled);
  }

  // ---------------------------------------------------------------- deblocking (8.7.2)
  int slice_of(int x, int y) const { return ctb_slice[(y >> log2_ctb) * wctb + (x >> log2_ctb)]; }
  int tile_of(int x, int y) const { return tile_id[rs2ts[(y >> log2_ctb) * wctb + (x >> log2_ctb)]]; }

  // reference picture identity of list entry (slice, list, idx)
  const StoredPic* ref_pic_of(int sidx, int l, int idx) const;

  // compute_bs: the DPB picture of every (slice segment, list, ref_idx) of the current picture,
  // resolved once per picture (ref_pic_of walks the DPB)
  std::vector<std::array<const StoredPic*, 32>> bs_refs_;
  void compute_bs(std::vector<uint8_t>& bsv) {
    bs_refs_.assign(cur->slices.size(), {});
    for (size_t s = 0; s < cur->slices.size(); ++s)
      for (int l = 0; l < 2; ++l)
        for (int i = 0; i < 16; ++i) bs_refs_[s][l * 16 + i] = ref_pic_of(static_cast<int>(s), l, i);
    const bool one_slice = slices.size() == 1;  // no slice lookups per edge
    for (int y = 0; y < H; y += 4)
      for (int x = 0; x < W; x += 4) {
        uint8_t v = 0;
        for (int dir = 0; dir < 2; ++dir) {
          const bool on_grid = dir == 0 ? (x % 8 == 0 && x > 0) : (y % 8 == 0 && y > 0);
          if (!on_grid) continue;
          const uint8_t e = edge[g4(x, y)];
          const bool tu = dir == 0 ? (e & E_TU_V) : (e & E_TU_H);
          const bool pu = dir == 0 ? (e & E_PU_V) : (e & E_PU_H);
          if (!tu && !pu) continue;
          const int xp = dir == 0 ? x - 1 : x, yp = dir == 0 ? y : y - 1;
          // edge filtering restrictions of the q-side (current) coding block's slice
          const int sq = one_slice ? 0 : slice_of(x, y), sp = one_slice ? 0 : slice_of(xp, yp);
          const SliceHeader& S = slices[sq];
          if (S.deblock_disabled) continue;
          if (sq != sp && slice_addr_of(sq) != slice_addr_of(sp) && !S.lf_across_slices) continue;
          if (!pps->lf_across_tiles && tile_of(x, y) != tile_of(xp, yp)) continue;
          const int b = bs_value(xp, yp, x, y, tu, sp, sq);
          v |= static_cast<uint8_t>(b << (dir * 2));
        }
        bsv[g4(x, y)] = v;
      }
  }
  // sa / sb: slice segments of the p / q blocks
  int bs_value(int xp, int yp, int xq, int yq, bool tu_edge, int sa, int sb) const {
    const size_t p = g4(xp, yp), q = g4(xq, yq);
    if ((cu_flags[p] & CF_INTRA) || (cu_flags[q] & CF_INTRA)) return 2;
    if (tu_edge && (cbf_y[p] || cbf_y[q])) return 1;
    const MvField& A = cur->mvf[p];
    const MvField& B = cur->mvf[q];
    auto pic = [&](int s, const MvField& m, int l) -> const void* {
      return m.pred & (1 << l) ? static_cast<const void*>(bs_refs_[s][l * 16 + (m.ref[l] & 15)]) : nullptr;
    };
    const int na = __builtin_popcount(A.pred), nb = __builtin_popcount(B.pred);
    if (na != nb) return 1;
    auto far = [](const int16_t* a, const int16_t* b) { return std::abs(a[0] - b[0]) >= 4 || std::abs(a[1] - b[1]) >= 4; };
    if (na == 1) {
      const int la = (A.pred & 1) ? 0 : 1, lb = (B.pred & 1) ? 0 : 1;
      if (pic(sa, A, la) != pic(sb, B, lb)) return 1;
      return far(A.mv[la], B.mv[lb]) ? 1 : 0;
    }
    const void* a0 = pic(sa, A, 0);
    const void* a1 = pic(sa, A, 1);
    const void* b0 = pic(sb, B, 0);
    const void* b1 = pic(sb, B, 1);
    if (!((a0 == b0 && a1 == b1) || (a0 == b1 && a1 == b0))) return 1;
    if (a0 != a1) {
      if (a0 == b0) return (far(A.mv[0], B.mv[0]) || far(A.mv[1], B.mv[1])) ? 1 : 0;
      return (far(A.mv[0], B.mv[1]) || far(A.mv[1], B.mv[0])) ? 1 : 0;
    }
    // both vectors of each block refer to the same picture
    const bool c1 = far(A.mv[0], B.mv[0]) || far(A.mv[1], B.mv[1]);
    const bool c2 = far(A.mv[0], B.mv[1]) || far(A.mv[1], B.mv[0]);
    return (c1 && c2) ? 1 : 0;
  }

  void deblock(const std::vector<uint8_t>& bsv) {
    for (int dir = 0; dir < 2; ++dir) {
      for (int y = 0; y < H; y += 4)
        for (int x = 0; x < W; x += 4) {
          const int b = (bsv[g4(x, y)] >> (dir * 2)) & 3;
          if (!b) continue;
          const int xp = dir == 0 ? x - 1 : x, yp = dir == 0 ? y : y - 1;
          const int qpl = (qp_y[g4(xp, yp)] + qp_y[g4(x, y)] + 1) >> 1;
          const SliceHeader& S = slices[slice_of(x, y)];
          const bool np = no_filter(g4(xp, yp)), nq = no_filter(g4(x, y));
          uint16_t* s = cur->pl[0].data() + static_cast<size_t>(y) * W + x;
          filter_luma(s, dir == 0 ? W : 1, dir == 0 ? 1 : W, b, qpl, S.beta_off, S.tc_off, np, nq);
        }
      for (int c = 1; c < 3; ++c)
        for (int y = 0; y < H; y += 4)
          for (int x = 0; x < W; x += 4) {
            const int b = (bsv[g4(x, y)] >> (dir * 2)) & 3;
            if (b != 2 || (dir == 0 ? (x % 16) : (y % 16))) continue;
            const int xp = dir == 0 ? x - 1 : x, yp = dir == 0 ? y : y - 1;
            const int qpl = (qp_y[g4(xp, yp)] + qp_y[g4(x, y)] + 1) >> 1;
            const SliceHeader& S = slices[slice_of(x, y)];
            const bool np = no_filter(g4(xp, yp)), nq = no_filter(g4(x, y));
            const int cw = W / 2;
            uint16_t* s = cur->pl[c].data() + static_cast<size_t>(y / 2) * cw + x / 2;
            filter_chroma(s, dir == 0 ? cw : 1, dir == 0 ? 1 : cw, qpl, c == 1 ? pps->cb_qp_off : pps->cr_qp_off, S.tc_off,
                          np, nq);
          }
    }
  }
  void filter_luma(uint16_t* s, int step, int across, int b, int qpl, int beta_off, int tc_off, bool np, bool nq) const {
    const int qb = clip3(0, 51, qpl + beta_off);
    const int qt = clip3(0, 53, qpl + 2 * (b - 1) + tc_off);
    const int beta = kBetaTable[qb] * (1 << (bd - 8)), tc = kTcTable[qt] * (1 << (bd - 8));
    auto P = [&](int l, int i) -> uint16_t& { return s[l * step - (i + 1) * across]; };
    auto Q = [&](int l, int i) -> uint16_t& { return s[l * step + i * across]; };
    const int dp0 = std::abs(P(0, 2) - 2 * P(0, 1) + P(0, 0)), dp3 = std::abs(P(3, 2) - 2 * P(3, 1) + P(3, 0));
    const int dq0 = std::abs(Q(0, 2) - 2 * Q(0, 1) + Q(0, 0)), dq3 = std::abs(Q(3, 2) - 2 * Q(3, 1) + Q(3, 0));
    const int dpq0 = dp0 + dq0, dpq3 = dp3 + dq3, dpv = dp0 + dp3, dqv = dq0 + dq3, d = dpq0 + dpq3;
    if (d >= beta) return;
    auto dsam = [&](int l, int dpq) {
      return 2 * dpq < (beta >> 2) && std::abs(P(l, 3) - P(l, 0)) + std::abs(Q(l, 0) - Q(l, 3)) < (beta >> 3) &&
             std::abs(P(l, 0) - Q(l, 0)) < ((5 * tc + 1) >> 1);
    };
    const bool strong = dsam(0, dpq0) && dsam(3, dpq3);
    const bool dep = dpv < ((beta + (beta >> 1)) >> 3), deq = dqv < ((beta + (beta >> 1)) >> 3);
    for (int l = 0; l < 4; ++l) {
      const int p0 = P(l, 0), p1 = P(l, 1), p2 = P(l, 2), p3 = P(l, 3);
      const int q0 = Q(l, 0), q1 = Q(l, 1), q2 = Q(l, 2), q3 = Q(l, 3);
      if (strong) {
        if (!np) {
          P(l, 0) = static_cast<uint16_t>(clip3(p0 - 2 * tc, p0 + 2 * tc, (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3));
          P(l, 1) = static_cast<uint16_t>(clip3(p1 - 2 * tc, p1 + 2 * tc, (p2 + p1 + p0 + q0 + 2) >> 2));
          P(l, 2) = static_cast<uint16_t>(clip3(p2 - 2 * tc, p2 + 2 * tc, (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3));
        }
        if (!nq) {
          Q(l, 0) = static_cast<uint16_t>(clip3(q0 - 2 * tc, q0 + 2 * tc, (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3));
          Q(l, 1) = static_cast<uint16_t>(clip3(q1 - 2 * tc, q1 + 2 * tc, (p0 + q0 + q1 + q2 + 2) >> 2));
          Q(l, 2) = static_cast<uint16_t>(clip3(q2 - 2 * tc, q2 + 2 * tc, (p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3));
        }
      } else {
        int delta = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4;
        if (std::abs(delta) >= tc * 10) continue;
        delta = clip3(-tc, tc, delta);
        if (!np) P(l, 0) = static_cast<uint16_t>(clip3(0, maxv, p0 + delta));
        if (!nq) Q(l, 0) = static_cast<uint16_t>(clip3(0, maxv, q0 - delta));
        if (dep && !np) P(l, 1) = static_cast<uint16_t>(clip3(0, maxv, p1 + clip3(-(tc >> 1), tc >> 1, (((p2 + p0 + 1) >> 1) - p1 + delta) >> 1)));
        if (deq && !nq) Q(l, 1) = static_cast<uint16_t>(clip3(0, maxv, q1 + clip3(-(tc >> 1), tc >> 1, (((q2 + q0 + 1) >> 1) - q1 - delta) >> 1)));
      }
    }
  }
  void filter_chroma(uint16_t* s, int step, int across, int qpl, int cqp_off, int tc_off, bool np, bool nq) const {
    const int qpc = chroma_qp_map(qpl + cqp_off);  // 8.7.2.5.5: QpC from qPi = QpL + cQpPicOffset (Table 8-10)
    const int qt = clip3(0, 53, qpc + 2 + tc_off);
    const int tc = kTcTable[qt] * (1 << (bdc - 8));
    for (int l = 0; l < 2; ++l) {  // a 4-row luma segment covers 2 chroma rows
      uint16_t* q = s + l * step;
      const int p0 = q[-across], p1 = q[-2 * across], q0 = q[0], q1 = q[across];
      const int delta = clip3(-tc, tc, ((((q0 - p0) << 2) + p1 - q1 + 4) >> 3));
      if (!np) q[-across] = static_cast<uint16_t>(clip3(0, maxvc, p0 + delta));
      if (!nq) q[0] = static_cast<uint16_t>(clip3(0, maxvc, q0 - delta));
    }
  }

  // ---------------------------------------------------------------- SAO (8.7.3)
  void apply_sao() {
    for (int c = 0; c < 3; ++c) {
      const int pw = c ? W / 2 : W, ph = c ? H / 2 : H, cs = c ? ctb / 2 : ctb, sc = c ? 1 : 0;
      const int mx = c ? maxvc : maxv, bdv = c ? bdc : bd;
      const std::vector<uint16_t> src = cur->pl[c];
      uint16_t* dst = cur->pl[c].data();
      for (int ry = 0; ry < hctb; ++ry)
        for (int rx = 0; rx < wctb; ++rx) {
          const DecSao& t = sao_params[ry * wctb + rx];
          const int type = t.type[c];
          if (!type) continue;
          const int x0 = rx * cs, y0 = ry * cs;
          const int sidx = ctb_slice[ry * wctb + rx];
          int table[32] = {};
          if (type == 1)
            for (int k = 0; k < 4; ++k) table[(k + t.band[c]) & 31] = k + 1;
          static const int hp[4][2] = {{-1, 1}, {0, 0}, {-1, 1}, {1, -1}};
          static const int vp[4][2] = {{0, 0}, {-1, 1}, {-1, 1}, {-1, 1}};
          const int cl = t.eo[c];
          for (int y = y0; y < std::min(y0 + cs, ph); ++y)
            for (int x = x0; x < std::min(x0 + cs, pw); ++x) {
              if (no_filter(g4(x << sc, y << sc))) continue;
              const int v = src[static_cast<size_t>(y) * pw + x];
              int off = 0;
              if (type == 1) {
                const int b = table[v >> (bdv - 5)];
                if (b) off = t.off[c][b - 1];
              } else {
                bool skip = false;
                int e = 2;
                for (int k = 0; k < 2 && !skip; ++k) {
                  const int xa = x + hp[cl][k], ya = y + vp[cl][k];
                  if (xa < 0 || ya < 0 || xa >= pw || ya >= ph) {
                    skip = true;
                    break;
                  }
                  const int xl = xa << sc, yl = ya << sc;
                  const int sn = slice_of(xl, yl);
                  if (sn != sidx && slice_addr_of(sn) != slice_addr_of(sidx)) {
                    const int rsn = (yl >> log2_ctb) * wctb + (xl >> log2_ctb), rsc = ry * wctb + rx;
                    const bool nb_first = rs2ts[rsn] < rs2ts[rsc];
                    if (nb_first && !slices[sidx].lf_across_slices) skip = true;
                    if (!nb_first && !slices[sn].lf_across_slices) skip = true;
                  }
                  if (!pps->lf_across_tiles && tile_of(xl, yl) != tile_of(x << sc, y << sc)) skip = true;
                  if (!skip) e += sgn(v - src[static_cast<size_t>(ya) * pw + xa]);
                }
                if (skip) continue;
                if (e <= 2) e = (e == 2) ? 0 : e + 1;
                if (e) off = t.off[c][e - 1];
              }
              if (off) dst[static_cast<size_t>(y) * pw + x] = static_cast<uint16_t>(clip3(0, mx, v + off));
            }
        }
    }
  }

  // ---------------------------------------------------------------- encoder records (32x32 blocks)
  CtuInfo& enc_blk(int x, int y) { return dp->ctu[static_cast<size_t>(y >> 5) * (W / 32) + (x >> 5)]; }
  CuInfo& enc_cu_at(int x, int y) {
    return dp->cu[(static_cast<size_t>(y >> 5) * (W / 32) + (x >> 5)) * kCusPerCtb + zorder8((x & 31) >> 3, (y & 31) >> 3)];
  }
  void enc_cu(int x0, int y0, int n, int pred, int pcm) {
    (void)pcm;
    for (int y = y0; y < y0 + n; y += 8)
      for (int x = x0; x < x0 + n; x += 8) {
        CuInfo& c = enc_cu_at(x, y);
        c.pred = static_cast<uint8_t>(pred);
        c.flags = static_cast<uint8_t>(c.flags & ~6);
        c.flags |= static_cast<uint8_t>(((cu_log2 - 3) & 3) << 1);
        if (pred == CU_INTRA) {
          c.mode = ipm[g4(x0, y0)];
          c.mv[0] = c.mv[1] = 0;
          if (cu_part == P_NxN) {
            c.flags |= 8;
            for (int k = 0; k < 4; ++k) reinterpret_cast<uint8_t*>(c.mv)[k] = static_cast<uint8_t>(pu_modes[k]);
          }
        } else {
          const MvField& m = cur->mvf[g4(x, y)];
          c.mode = 0;
          c.mv[0] = (m.pred & 1) ? m.mv[0][0] : 0;
          c.mv[1] = (m.pred & 1) ? m.mv[0][1] : 0;
          c.mv1[0] = (m.pred & 2) ? m.mv[1][0] : 0;
          c.mv1[1] = (m.pred & 2) ? m.mv[1][1] : 0;
          c.dir = m.pred;
          c.pad[0] = static_cast<uint8_t>((m.pred & 1) ? m.ref[0] : 0);  // refIdx L0 / L1
          c.pad[1] = static_cast<uint8_t>((m.pred & 2) ? m.ref[1] : 0);
        }
      }
  }
};

// picture identity of a reference list entry, for boundary strengths (any list / slice)
const StoredPic* HevcStreamDecoder::Impl::ref_pic_of(int sidx, int l, int idx) const {
  const SliceRefs& sr = cur->slices[sidx];
  const int id = sr.pic[l][idx];
  for (const auto& p : dpb)
    if (p->decode_idx == id) return p.get();
  return nullptr;
}

// ======================================================================================
HevcStreamDecoder::HevcStreamDecoder(const DecodeOptions& o) : impl_(new Impl) {
  impl_->opt = o;
  impl_->out = &pics_;
}
HevcStreamDecoder::~HevcStreamDecoder() = default;

void HevcStreamDecoder::decode(const uint8_t* data, size_t n) {
  const std::vector<NalUnit> nals = parse_annexb(data, n);
  for (const NalUnit& u : nals) impl_->decode_nal(u, data);
  impl_->finish_picture();
}

std::vector<int> HevcStreamDecoder::output_order() const {
  std::vector<int> idx;
  for (size_t i = 0; i < pics_.size(); ++i)
    if (pics_[i].output) idx.push_back(static_cast<int>(i));
  std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) {
    if (pics_[a].cvs != pics_[b].cvs) return pics_[a].cvs < pics_[b].cvs;
    return pics_[a].poc < pics_[b].poc;
  });
  return idx;
}

// ======================================================================================
// Compatibility facade: the encoder-subset oracle API (hevc_codec.h) on the general decoder
struct HevcDecoder::Impl {};
HevcDecoder::HevcDecoder() : impl_(new Impl) {}
HevcDecoder::~HevcDecoder() = default;
void HevcDecoder::decode(const uint8_t* data, size_t n) {
  DecodeOptions o;
  o.recon = true;
  o.skip_filters = skip_filters_;
  o.enc_records = true;
  HevcStreamDecoder d(o);
  d.decode(data, n);
  for (int i : d.output_order()) {
    DecPicture& s = d.pictures()[i];
    HevcPicture p;
    p.coded_width = s.W;
    p.coded_height = s.H;
    p.width = s.width;
    p.height = s.height;
    p.bit_depth = s.bit_depth;
    p.poc = s.poc;
    p.idr = s.idr;
    p.slice_type = s.slice_type;
    p.qp = s.slice_qp;
    p.y = std::move(s.y);
    p.u = std::move(s.u);
    p.v = std::move(s.v);
    p.ctu = std::move(s.ctu);
    p.cu = std::move(s.cu);
    p.coef_y = std::move(s.coef_y);
    p.coef_cb = std::move(s.coef_cb);
    p.coef_cr = std::move(s.coef_cr);
    out_.push_back(std::move(p));
  }
}

}  // namespace hevc
}  // namespace mivc
