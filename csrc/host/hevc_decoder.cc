// Independent HEVC decoder for the coding-tool subset of hevc_codec.h: the
// conformance oracle of the HEVC encoder (SURVEY.md 4.2 tier T2 -- "encoder
// reconstruction == our decoder output, bit-exact").  Written from ITU-T H.265
// clauses 7-9 separately from the encoder-side writer (hevc_writer.cc) and the HIP
// kernels; only constant tables are shared.  Streams outside the subset raise.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "bitstream.h"
#include "hevc_cabac.h"
#include "hevc_codec.h"

namespace mivc {
namespace hevc {

namespace {

inline int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
inline int sgn(int v) { return (v > 0) - (v < 0); }

struct Sps {
  bool valid = false;
  int chroma_format = 1, W = 0, H = 0, bit_depth = 8, bit_depth_c = 8;
  int crop[4] = {0, 0, 0, 0};
  int log2_poc = 8, log2_min_cb = 3, log2_ctb = 5, log2_min_tb = 2, log2_max_tb = 5;
  int depth_inter = 0, depth_intra = 0;
  bool amp = false, sao = false, pcm = false, strong = false, tmvp = false, scaling = false, long_term = false;
  int num_st_rps = 0;
  int st_neg[64] = {};     // number of negative pictures per set (only delta -1 sets supported)
};

struct Pps {
  bool valid = false;
  int sps_id = 0, init_qp = 26, cb_off = 0, cr_off = 0, num_ref_l0 = 1, log2_pml = 2, diff_qp_depth = 0;
  bool sign_hiding = false, cabac_init_present = false, cu_qp_delta = false, tskip = false, bypass = false;
  bool tiles = false, wpp = false, deblock_disabled = false, deblock_override = false, lists_mod = false;
  bool slice_chroma_offsets = false, constrained_intra = false, weighted = false, output_flag = false;
  bool dep_slices = false, lf_across_slices = false, ext_header = false;
  int extra_bits = 0, beta_off = 0, tc_off = 0;
};

struct Picture {
  int W = 0, H = 0;
  std::vector<uint16_t> pl[3];
};

void skip_ptl(BitReader& br, int max_sub_layers_minus1) {
  br.get(8);   // profile space, tier, idc
  br.get(32);  // compatibility flags
  br.get(4);   // source flags
  br.get(32);
  br.get(11);
  br.get(1);
  br.get(8);   // level
  std::vector<int> pp(max_sub_layers_minus1), lp(max_sub_layers_minus1);
  for (int i = 0; i < max_sub_layers_minus1; ++i) {
    pp[i] = br.get(1);
    lp[i] = br.get(1);
  }
  if (max_sub_layers_minus1 > 0)
    for (int i = max_sub_layers_minus1; i < 8; ++i) br.get(2);
  for (int i = 0; i < max_sub_layers_minus1; ++i) {
    if (pp[i]) {
      br.get(32);
      br.get(32);
      br.get(24);
    }
    if (lp[i]) br.get(8);
  }
}

// luma / chroma interpolation filters (8.5.3.3.3)
const int kLumaTaps[4][8] = {{0, 0, 0, 64, 0, 0, 0, 0},
                             {-1, 4, -10, 58, 17, -5, 1, 0},
                             {-1, 4, -11, 40, 40, -11, 4, -1},
                             {0, 1, -5, 17, 58, -10, 4, -1}};
const int kChromaTaps[8][4] = {{0, 64, 0, 0},     {-2, 58, 10, -2}, {-4, 54, 16, -2}, {-6, 46, 28, -4},
                               {-4, 36, 36, -4},  {-4, 28, 46, -6}, {-2, 16, 54, -4}, {-2, 10, 58, -2}};

}  // namespace

struct HevcDecoder::Impl {
  Sps sps;
  Pps pps;
  bool skip_filters = false;
  Picture ref;
  bool have_ref = false;
  int poc_prev = 0;

  // ---- per-picture state
  int W = 0, H = 0, bd = 8, maxv = 255, wctb = 0, hctb = 0, slice_type = 2, qp = 26, poc = 0;
  bool idr = false, sao_luma = false, sao_chroma = false, deblock = true;
  int max_merge = 5;
  // quantization parameters (8.6.1): QpY of the current CU, the quantization group's
  // prediction and CuQpDeltaVal, QpY of the last CU decoded (qPY_PREV of the next group)
  int cu_qp = 26, qg_pred = 26, qp_delta_val = 0, last_cu_qp = 26, log2_min_qg = 6;
  bool qp_delta_coded = false;
  Picture cur;
  std::vector<int8_t> g_pred, g_skip, g_depth, g_mode, g_qp, g_cbf, g_done;  // per 4x4 luma block
  std::vector<int16_t> g_mvx, g_mvy;
  int w4 = 0, h4 = 0;
  std::vector<uint8_t> edge_v, edge_h;  // per 4x4: 1 if the left / top edge is a TU/PU edge
  std::vector<CtuInfo> rec_ctu;
  std::vector<CuInfo> rec_cu;
  std::vector<int16_t> rec_coef[3];
  CtxState ctx[kNumCtx];
  CabacDecoder* cd = nullptr;

  // ------------------------------------------------------------ parameter sets
  void parse_sps(BitReader& br) {
    Sps s;
    br.get(4);
    const int msl = br.get(3);
    br.get(1);
    skip_ptl(br, msl);
    if (br.get_ue() != 0) throw std::runtime_error("HEVC: only sps id 0");
    s.chroma_format = br.get_ue();
    if (s.chroma_format != 1) throw std::runtime_error("HEVC: only 4:2:0");
    s.W = br.get_ue();
    s.H = br.get_ue();
    if (br.get(1))
      for (int i = 0; i < 4; ++i) s.crop[i] = br.get_ue();
    s.bit_depth = 8 + br.get_ue();
    s.bit_depth_c = 8 + br.get_ue();
    if (s.bit_depth != s.bit_depth_c || s.bit_depth > 10) throw std::runtime_error("HEVC: bit depth");
    s.log2_poc = br.get_ue() + 4;
    const int sub = br.get(1);
    for (int i = sub ? 0 : msl; i <= msl; ++i) {
      br.get_ue();
      br.get_ue();
      br.get_ue();
    }
    s.log2_min_cb = br.get_ue() + 3;
    s.log2_ctb = s.log2_min_cb + br.get_ue();
    s.log2_min_tb = br.get_ue() + 2;
    s.log2_max_tb = s.log2_min_tb + br.get_ue();
    s.depth_inter = br.get_ue();
    s.depth_intra = br.get_ue();
    s.scaling = br.get(1);
    if (s.scaling) throw std::runtime_error("HEVC: scaling lists unsupported");
    s.amp = br.get(1);
    s.sao = br.get(1);
    s.pcm = br.get(1);
    if (s.pcm) throw std::runtime_error("HEVC: PCM unsupported");
    s.num_st_rps = br.get_ue();
    for (int i = 0; i < s.num_st_rps; ++i) {
      if (i > 0 && br.get(1)) throw std::runtime_error("HEVC: inter RPS prediction unsupported");
      const int nneg = br.get_ue(), npos = br.get_ue();
      if (npos) throw std::runtime_error("HEVC: positive reference pictures unsupported");
      for (int k = 0; k < nneg; ++k) {
        br.get_ue();
        br.get(1);
      }
      s.st_neg[i] = nneg;
    }
    s.long_term = br.get(1);
    if (s.long_term) throw std::runtime_error("HEVC: long-term references unsupported");
    s.tmvp = br.get(1);
    s.strong = br.get(1);
    s.valid = true;
    sps = s;
  }

  void parse_pps(BitReader& br) {
    Pps p;
    if (br.get_ue() != 0 || br.get_ue() != 0) throw std::runtime_error("HEVC: only pps/sps id 0");
    p.dep_slices = br.get(1);
    p.output_flag = br.get(1);
    p.extra_bits = br.get(3);
    p.sign_hiding = br.get(1);
    p.cabac_init_present = br.get(1);
    p.num_ref_l0 = br.get_ue() + 1;
    br.get_ue();
    p.init_qp = 26 + br.get_se();
    p.constrained_intra = br.get(1);
    p.tskip = br.get(1);
    p.cu_qp_delta = br.get(1);
    if (p.cu_qp_delta) p.diff_qp_depth = br.get_ue();
    p.cb_off = br.get_se();
    p.cr_off = br.get_se();
    p.slice_chroma_offsets = br.get(1);
    p.weighted = br.get(1) | br.get(1);
    p.bypass = br.get(1);
    p.tiles = br.get(1);
    p.wpp = br.get(1);
    if (p.tskip || p.bypass || p.tiles || p.weighted || p.constrained_intra ||
        p.slice_chroma_offsets || p.dep_slices || p.output_flag || p.extra_bits)
      throw std::runtime_error("HEVC: PPS tool outside the supported subset");
    p.lf_across_slices = br.get(1);
    if (br.get(1)) {  // deblocking_filter_control_present_flag
      p.deblock_override = br.get(1);
      p.deblock_disabled = br.get(1);
      if (!p.deblock_disabled) {
        p.beta_off = br.get_se() * 2;
        p.tc_off = br.get_se() * 2;
      }
    }
    if (br.get(1)) throw std::runtime_error("HEVC: PPS scaling lists unsupported");
    p.lists_mod = br.get(1);
    p.log2_pml = br.get_ue() + 2;
    p.ext_header = br.get(1);
    p.valid = true;
    pps = p;
  }

  // ------------------------------------------------------------ picture buffers
  void start_picture() {
    W = sps.W;
    H = sps.H;
    bd = sps.bit_depth;
    maxv = (1 << bd) - 1;
    const int ctb = 1 << sps.log2_ctb;
    wctb = (W + ctb - 1) / ctb;
    hctb = (H + ctb - 1) / ctb;
    cur.W = W;
    cur.H = H;
    cur.pl[0].assign(static_cast<size_t>(W) * H, 0);
    cur.pl[1].assign(static_cast<size_t>(W / 2) * (H / 2), 0);
    cur.pl[2].assign(cur.pl[1].size(), 0);
    w4 = W / 4;
    h4 = H / 4;
    const size_t n4 = static_cast<size_t>(w4) * h4;
    g_pred.assign(n4, 0);
    g_skip.assign(n4, 0);
    g_depth.assign(n4, 0);
    g_mode.assign(n4, 1);
    g_qp.assign(n4, 0);
    g_cbf.assign(n4, 0);
    g_done.assign(n4, 0);
    g_mvx.assign(n4, 0);
    g_mvy.assign(n4, 0);
    edge_v.assign(n4, 0);
    edge_h.assign(n4, 0);
    rec_ctu.assign(static_cast<size_t>(wctb) * hctb, CtuInfo{});
    rec_cu.assign(static_cast<size_t>(wctb) * hctb * kCusPerCtb, CuInfo{});
    rec_coef[0].assign(static_cast<size_t>(W) * H, 0);
    rec_coef[1].assign(static_cast<size_t>(W / 2) * (H / 2), 0);
    rec_coef[2].assign(rec_coef[1].size(), 0);
  }

  size_t g4(int x, int y) const { return static_cast<size_t>(y >> 2) * w4 + (x >> 2); }
  bool in_pic(int x, int y) const { return x >= 0 && y >= 0 && x < W && y < H; }
  bool done(int x, int y) const { return in_pic(x, y) && g_done[g4(x, y)]; }

  // ------------------------------------------------------------ slice
  void decode_slice(const NalUnit& nal, int type, std::vector<HevcPicture>& out) {
    // rbsp[0] is the second NAL header byte
    BitReader br(nal.rbsp.data() + 1, nal.rbsp.size() - 1);
    if (!sps.valid || !pps.valid) throw std::runtime_error("HEVC: slice before parameter sets");
    if (!br.get(1)) throw std::runtime_error("HEVC: multiple slices per picture unsupported");
    idr = type == 19 || type == 20;
    if (type >= 16 && type <= 23) br.get(1);  // no_output_of_prior_pics_flag
    br.get_ue();                              // pps id
    slice_type = br.get_ue();
    if (slice_type == 0) throw std::runtime_error("HEVC: B slices unsupported");
    poc = 0;
    if (!idr) {
      const int lsb = br.get(sps.log2_poc);
      const int maxlsb = 1 << sps.log2_poc;
      const int prev_lsb = poc_prev & (maxlsb - 1), prev_msb = poc_prev - prev_lsb;
      int msb = prev_msb;
      if (lsb < prev_lsb && prev_lsb - lsb >= maxlsb / 2) msb += maxlsb;
      else if (lsb > prev_lsb && lsb - prev_lsb > maxlsb / 2) msb -= maxlsb;
      poc = msb + lsb;
      if (br.get(1)) {  // short_term_ref_pic_set_sps_flag
        int bits = 0;
        while ((1 << bits) < sps.num_st_rps) ++bits;
        if (bits) br.get(bits);
      } else {
        throw std::runtime_error("HEVC: slice-level RPS unsupported");
      }
    }
    sao_luma = sao_chroma = false;
    if (sps.sao) {
      sao_luma = br.get(1);
      sao_chroma = br.get(1);
    }
    if (slice_type == 1) {
      if (br.get(1)) {  // num_ref_idx_active_override_flag
        if (br.get_ue() != 0) throw std::runtime_error("HEVC: more than one reference");
      } else if (pps.num_ref_l0 != 1) {
        throw std::runtime_error("HEVC: more than one reference");
      }
      if (pps.lists_mod) throw std::runtime_error("HEVC: list modification unsupported");
      if (pps.cabac_init_present) br.get(1);
      max_merge = 5 - br.get_ue();
    }
    qp = pps.init_qp + br.get_se();
    deblock = !pps.deblock_disabled;
    if (pps.deblock_override && br.get(1)) throw std::runtime_error("HEVC: deblocking override unsupported");
    if (pps.lf_across_slices && (sao_luma || sao_chroma || deblock)) br.get(1);
    std::vector<uint32_t> entry;  // entry_point_offset_minus1 + 1 (escaped bytes, 7.4.7.1)
    if (pps.wpp) {
      const uint32_t ne = br.get_ue();
      const int ctb = 1 << sps.log2_ctb;
      if (ne != static_cast<uint32_t>((sps.H + ctb - 1) / ctb - 1)) throw std::runtime_error("HEVC: WPP entry points != CTB rows - 1");
      if (ne > 0) {
        const int len = br.get_ue() + 1;
        if (len > 32) throw std::runtime_error("HEVC: offset_len_minus1 out of range");
        for (uint32_t k = 0; k < ne; ++k) entry.push_back(br.get(len) + 1);
      }
    }
    if (pps.ext_header) {
      const int n = br.get_ue();
      for (int i = 0; i < n; ++i) br.get(8);
    }
    // byte_alignment()
    if (br.get(1) != 1) throw std::runtime_error("HEVC: slice header alignment");
    while (!br.byte_aligned()) br.get(1);
    if (slice_type == 1 && !have_ref) throw std::runtime_error("HEVC: P slice without a reference picture");

    start_picture();
    CabacDecoder dec(nal.rbsp.data() + 1, nal.rbsp.size() - 1, br.pos() / 8);
    cd = &dec;
    dec.start();
    init_contexts(ctx, slice_type == 2 ? 0 : 1, qp);
    cu_qp = qg_pred = last_cu_qp = qp;
    qp_delta_val = 0;
    log2_min_qg = sps.log2_ctb - pps.diff_qp_depth;
    if (pps.cu_qp_delta && log2_min_qg < sps.log2_min_cb) throw std::runtime_error("HEVC: diff_cu_qp_delta_depth out of range");
    const int nctb = wctb * hctb;
    const size_t data0 = 1 + br.pos() / 8;  // rbsp index of the slice data
    auto escaped = [&](size_t r) {  // rbsp index -> byte offset in the escaped NAL payload
      size_t k = 0;
      while (k < nal.epb.size() && nal.epb[k] < r) ++k;
      return r + k;
    };
    size_t sub_start = data0;
    CtxState wpp_ctx[kNumCtx];
    for (int i = 0; i < nctb; ++i) {
      const int rx = i % wctb, ry = i / wctb;
      if (pps.wpp && rx == 0 && ry > 0) {
        // 9.3.1: new substream, contexts synchronised from CTB (1, ry-1) when it exists
        const size_t at = 1 + dec.byte_pos();
        if (escaped(at) - escaped(sub_start) != entry[ry - 1])
          throw std::runtime_error("HEVC: WPP entry point offset mismatch");
        sub_start = at;
        dec.start();
        if (wctb >= 2) std::copy(wpp_ctx, wpp_ctx + kNumCtx, ctx);
        else init_contexts(ctx, slice_type == 2 ? 0 : 1, qp);
        last_cu_qp = qp;  // 8.6.1: first quantization group of a CTB row with WPP
      }
      if (sps.sao && (sao_luma || sao_chroma)) parse_sao(rx, ry);
      coding_quadtree(rx << sps.log2_ctb, ry << sps.log2_ctb, sps.log2_ctb, 0, rx, ry);
      const int end = dec.terminate();
      if (end != (i == nctb - 1)) throw std::runtime_error("HEVC: end_of_slice_segment_flag mismatch");
      if (pps.wpp && rx == 1) std::copy(ctx, ctx + kNumCtx, wpp_ctx);
      if (pps.wpp && rx == wctb - 1 && i != nctb - 1) {
        if (dec.terminate() != 1) throw std::runtime_error("HEVC: end_of_subset_one_bit != 1");
        dec.align();  // byte_alignment(): the flush's final 1 bit is alignment_bit_equal_to_one
      }
    }
    cd = nullptr;
    if (!skip_filters) {
      if (deblock) deblocking();
      if (sps.sao && (sao_luma || sao_chroma)) apply_sao();
    }
    // output
    HevcPicture p;
    p.coded_width = W;
    p.coded_height = H;
    p.width = W - 2 * (sps.crop[0] + sps.crop[1]);
    p.height = H - 2 * (sps.crop[2] + sps.crop[3]);
    p.bit_depth = bd;
    p.poc = poc;
    p.idr = idr;
    p.slice_type = slice_type;
    p.qp = qp;
    p.y = cur.pl[0];
    p.u = cur.pl[1];
    p.v = cur.pl[2];
    p.ctu = rec_ctu;
    p.cu = rec_cu;
    p.coef_y = rec_coef[0];
    p.coef_cb = rec_coef[1];
    p.coef_cr = rec_coef[2];
    out.push_back(std::move(p));
    ref = cur;
    have_ref = true;
    poc_prev = poc;
  }

  // ------------------------------------------------------------ SAO syntax (7.3.8.3)
  void parse_sao(int rx, int ry) {
    CtuInfo& t = rec_ctu[ry * wctb + rx];
    if (rx > 0 && cd->decode(ctx[CTX_SAO_MERGE])) {
      copy_sao(t, rec_ctu[ry * wctb + rx - 1]);
      return;
    }
    if (ry > 0 && cd->decode(ctx[CTX_SAO_MERGE])) {
      copy_sao(t, rec_ctu[(ry - 1) * wctb + rx]);
      return;
    }
    const int cmax = (1 << (std::min(bd, 10) - 5)) - 1;
    for (int ci = 0; ci < 3; ++ci) {
      if ((ci == 0 && !sao_luma) || (ci > 0 && !sao_chroma)) {
        if (ci < 2) t.sao_type[ci] = 0;
        continue;
      }
      if (ci < 2) {
        int type = 0;
        if (cd->decode(ctx[CTX_SAO_TYPE])) type = cd->bypass() ? 2 : 1;
        t.sao_type[ci] = static_cast<uint8_t>(type);
      }
      const int type = t.sao_type[ci ? 1 : 0];
      if (type == 0) continue;
      int abs_[4];
      for (int i = 0; i < 4; ++i) {
        int a = 0;
        while (a < cmax && cd->bypass()) ++a;
        abs_[i] = a;
      }
      if (type == 1) {
        for (int i = 0; i < 4; ++i) t.sao_off[ci][i] = static_cast<int8_t>(abs_[i] && cd->bypass() ? -abs_[i] : abs_[i]);
        t.sao_band[ci] = static_cast<uint8_t>(cd->bypass_bits(5));
      } else {
        t.sao_off[ci][0] = static_cast<int8_t>(abs_[0]);
        t.sao_off[ci][1] = static_cast<int8_t>(abs_[1]);
        t.sao_off[ci][2] = static_cast<int8_t>(-abs_[2]);
        t.sao_off[ci][3] = static_cast<int8_t>(-abs_[3]);
        if (ci == 0) t.sao_class[0] = static_cast<uint8_t>(cd->bypass_bits(2));
        if (ci == 1) t.sao_class[1] = static_cast<uint8_t>(cd->bypass_bits(2));
      }
    }
  }
  static void copy_sao(CtuInfo& d, const CtuInfo& s) {
    const uint8_t split = d.split;
    const int8_t q = d.qp;
    d = s;
    d.split = split;
    d.qp = q;
  }

  // ------------------------------------------------------------ coding quadtree (7.3.8.4)
  void coding_quadtree(int x0, int y0, int log2, int depth, int rx, int ry) {
    const int n = 1 << log2;
    if (pps.cu_qp_delta && log2 >= log2_min_qg) start_qg(x0, y0);
    bool split;
    if (x0 + n <= W && y0 + n <= H && log2 > sps.log2_min_cb) {
      int c = 0;
      if (done(x0 - 1, y0) && g_depth[g4(x0 - 1, y0)] > depth) ++c;
      if (done(x0, y0 - 1) && g_depth[g4(x0, y0 - 1)] > depth) ++c;
      split = cd->decode(ctx[CTX_SPLIT_CU + c]);
    } else {
      split = log2 > sps.log2_min_cb;
    }
    if (split) {
      CtuInfo& t = rec_ctu[ry * wctb + rx];
      if (log2 == sps.log2_ctb) t.split |= 1;
      else if (log2 == sps.log2_ctb - 1) t.split |= static_cast<uint8_t>(1 << (1 + quadrant(x0, y0)));
      const int h = n >> 1;
      for (int q = 0; q < 4; ++q) {
        const int x1 = x0 + (q & 1) * h, y1 = y0 + (q >> 1) * h;
        if (x1 < W && y1 < H) coding_quadtree(x1, y1, log2 - 1, depth + 1, rx, ry);
      }
      return;
    }
    coding_unit(x0, y0, log2, depth, rx, ry);
  }
  int quadrant(int x, int y) const {
    const int m = (1 << sps.log2_ctb) - 1, h = 1 << (sps.log2_ctb - 1);
    return ((x & m) >= h) + 2 * ((y & m) >= h);
  }

  void set_cu(int x0, int y0, int n, int pred, int skip, int depth, int mode, int mvx, int mvy) {
    for (int y = y0; y < y0 + n; y += 4)
      for (int x = x0; x < x0 + n; x += 4) {
        const size_t k = g4(x, y);
        g_pred[k] = static_cast<int8_t>(pred);
        g_skip[k] = static_cast<int8_t>(skip);
        g_depth[k] = static_cast<int8_t>(depth);
        g_mode[k] = static_cast<int8_t>(mode);
        g_mvx[k] = static_cast<int16_t>(mvx);
        g_mvy[k] = static_cast<int16_t>(mvy);
        g_qp[k] = static_cast<int8_t>(cu_qp);
      }
    const int ctb = 1 << sps.log2_ctb;
    for (int y = y0; y < y0 + n; y += 8)
      for (int x = x0; x < x0 + n; x += 8) {
        const int rx = x / ctb, ry = y / ctb;
        if (ctb != kCtb) continue;  // records are defined for 32x32 CTBs only
        CuInfo& c = rec_cu[static_cast<size_t>(ry * wctb + rx) * kCusPerCtb + zorder8((x & 31) >> 3, (y & 31) >> 3)];
        c.pred = static_cast<uint8_t>(pred);
        c.mode = static_cast<uint8_t>(pred == CU_INTRA ? mode : 0);
        c.mv[0] = static_cast<int16_t>(mvx);
        c.mv[1] = static_cast<int16_t>(mvy);
      }
    // TU = PU = CU: its boundary is a transform and prediction edge
    for (int k = 0; k < n; k += 4) {
      edge_v[g4(x0, y0 + k)] = 1;
      edge_h[g4(x0 + k, y0)] = 1;
    }
  }
  void mark_done(int x0, int y0, int n) {
    for (int y = y0; y < y0 + n; y += 4)
      for (int x = x0; x < x0 + n; x += 4) g_done[g4(x, y)] = 1;
  }

  // 8.6.1 start of a quantization group: IsCuQpDeltaCoded = 0, CuQpDeltaVal = 0 and
  // qPY_PRED from the left / above groups when they lie in the same CTB, else qPY_PREV
  void start_qg(int x0, int y0) {
    qp_delta_coded = false;
    qp_delta_val = 0;
    const int prev = last_cu_qp;
    const int cm = ~((1 << sps.log2_ctb) - 1);
    auto nb = [&](int x, int y) {
      if (!done(x, y) || (x & cm) != (x0 & cm) || (y & cm) != (y0 & cm)) return prev;
      return static_cast<int>(g_qp[g4(x, y)]);
    };
    qg_pred = (nb(x0 - 1, y0) + nb(x0, y0 - 1) + 1) >> 1;
    if (!pps.cu_qp_delta) qg_pred = qp;
    cu_qp = qg_pred;
    if (x0 % (1 << sps.log2_ctb) == 0 && y0 % (1 << sps.log2_ctb) == 0 && sps.log2_ctb == kCtbLog2) {
      CtuInfo& t = rec_ctu[(y0 >> kCtbLog2) * wctb + (x0 >> kCtbLog2)];
      t.qp = static_cast<int8_t>(qg_pred);
      t.qp_pred = static_cast<int8_t>(qg_pred);
      t.qp_first = 16;
    }
  }
  // cu_qp_delta_abs / _sign_flag (7.3.8.10, 9.3.3.10) -> QpY of the CU (8.6.1)
  void parse_qp_delta(int x0, int y0) {
    int a = 0;
    while (a < 5 && cd->decode(ctx[CTX_CU_QP_DELTA + (a > 0)])) ++a;
    if (a == 5) {
      int k = 0;
      while (cd->bypass()) {
        a += 1 << k;
        if (++k > 30) throw std::runtime_error("HEVC: cu_qp_delta_abs suffix too long");
      }
      while (k--) a += cd->bypass() << k;
    }
    const int d = a && cd->bypass() ? -a : a;
    const int off = 6 * (bd - 8);
    if (d < -(26 + off / 2) || d > 25 + off / 2) throw std::runtime_error("HEVC: CuQpDeltaVal out of range");
    qp_delta_coded = true;
    qp_delta_val = d;
    cu_qp = ((qg_pred + d + 52 + 2 * off) % (52 + off)) - off;
    if (sps.log2_ctb == kCtbLog2) {
      CtuInfo& t = rec_ctu[(y0 >> kCtbLog2) * wctb + (x0 >> kCtbLog2)];
      t.qp = static_cast<int8_t>(cu_qp);
      t.qp_first = static_cast<uint8_t>(zorder8((x0 & 31) >> 3, (y0 & 31) >> 3));
    }
  }

  // ------------------------------------------------------------ coding unit (7.3.8.5)
  void coding_unit(int x0, int y0, int log2, int depth, int rx, int ry) {
    coding_unit_syntax(x0, y0, log2, depth, rx, ry);
    // the CU's QpY (deblocking, and qPY_PREV of the next quantization group)
    const int n = 1 << log2;
    for (int y = y0; y < y0 + n; y += 4)
      for (int x = x0; x < x0 + n; x += 4) g_qp[g4(x, y)] = static_cast<int8_t>(cu_qp);
    last_cu_qp = cu_qp;
  }
  void coding_unit_syntax(int x0, int y0, int log2, int depth, int rx, int ry) {
    (void)rx;
    (void)ry;
    const int n = 1 << log2;
    bool skip = false;
    if (slice_type != 2) {
      int c = 0;
      if (done(x0 - 1, y0) && g_skip[g4(x0 - 1, y0)]) ++c;
      if (done(x0, y0 - 1) && g_skip[g4(x0, y0 - 1)]) ++c;
      skip = cd->decode(ctx[CTX_CU_SKIP + c]);
    }
    if (skip) {
      const int idx = parse_merge_idx();
      int mx, my;
      merge_candidate(x0, y0, n, idx, &mx, &my);
      set_cu(x0, y0, n, CU_INTER, 1, depth, 1, mx, my);
      predict_inter(x0, y0, n, mx, my);
      mark_done(x0, y0, n);
      return;
    }
    bool intra = true;
    if (slice_type != 2) intra = cd->decode(ctx[CTX_PRED_MODE]);
    bool nxn = false;
    if (!intra || log2 == sps.log2_min_cb) {
      // part_mode (9.3.3.7): intra at the minimum CB size: 1 = PART_2Nx2N, 0 = PART_NxN
      if (!cd->decode(ctx[CTX_PART_MODE])) {
        if (!intra) throw std::runtime_error("HEVC: only PART_2Nx2N inter PUs supported");
        if (log2 <= sps.log2_min_tb) throw std::runtime_error("HEVC: PART_NxN below the minimum TB size");
        nxn = true;
      }
    }
    if (intra) {
      const int npu = nxn ? 4 : 1, h = nxn ? n / 2 : n;
      int prev[4], mpm[4] = {}, rem[4] = {}, m[4];
      for (int k = 0; k < npu; ++k) prev[k] = cd->decode(ctx[CTX_PREV_INTRA]);
      for (int k = 0; k < npu; ++k) {
        if (prev[k]) {
          mpm[k] = cd->bypass();
          if (mpm[k]) mpm[k] += cd->bypass();
        } else {
          rem[k] = static_cast<int>(cd->bypass_bits(5));
        }
      }
      // chroma mode: 4 = DM
      int cm = 4;
      if (cd->decode(ctx[CTX_CHROMA_MODE])) cm = static_cast<int>(cd->bypass_bits(2));
      const int cu_rect[3] = {x0, y0, n};
      for (int k = 0; k < npu; ++k)
        m[k] = derive_luma_mode(x0 + (k & 1) * h, y0 + (k >> 1) * h, prev[k], mpm[k], rem[k], cu_rect, m);
      int mc = m[0];  // 8.4.3: chroma from IntraPredModeY[xCb][yCb]
      if (cm != 4) {
        const int tab[4] = {0, 26, 10, 1};
        mc = tab[cm] == m[0] ? 34 : tab[cm];
      }
      set_cu(x0, y0, n, CU_INTRA, 0, depth, m[0], 0, 0);
      if (nxn) {
        for (int k = 1; k < 4; ++k)
          for (int y = 0; y < h; y += 4)
            for (int x = 0; x < h; x += 4) g_mode[g4(x0 + (k & 1) * h + x, y0 + (k >> 1) * h + y)] = static_cast<int8_t>(m[k]);
        if (sps.log2_ctb == kCtbLog2) {
          CuInfo& c = rec_cu[static_cast<size_t>((y0 >> kCtbLog2) * wctb + (x0 >> kCtbLog2)) * kCusPerCtb +
                             zorder8((x0 & 31) >> 3, (y0 & 31) >> 3)];
          c.flags |= 8;
          for (int k = 0; k < 4; ++k) reinterpret_cast<uint8_t*>(c.mv)[k] = static_cast<uint8_t>(m[k]);
        }
        transform_tree_nxn(x0, y0, log2, m, mc);
      } else {
        transform_tree(x0, y0, log2, true, m[0], mc);
      }
      mark_done(x0, y0, n);
      return;
    }
    // inter 2Nx2N
    const bool merge = cd->decode(ctx[CTX_MERGE_FLAG]);
    int mx, my;
    if (merge) {
      merge_candidate(x0, y0, n, parse_merge_idx(), &mx, &my);
    } else {
      int d[2];
      parse_mvd(d);
      const int pidx = cd->decode(ctx[CTX_MVP_IDX]);
      int px, py;
      amvp_candidate(x0, y0, n, pidx, &px, &py);
      mx = static_cast<int16_t>(px + d[0]);
      my = static_cast<int16_t>(py + d[1]);
    }
    set_cu(x0, y0, n, CU_INTER, 0, depth, 1, mx, my);
    predict_inter(x0, y0, n, mx, my);
    bool root = true;
    if (!merge) root = cd->decode(ctx[CTX_RQT_ROOT_CBF]);
    if (root) transform_tree(x0, y0, log2, false, 0, 0);
    mark_done(x0, y0, n);
  }

  int parse_merge_idx() {
    if (max_merge <= 1) return 0;
    int i = 0;
    if (cd->decode(ctx[CTX_MERGE_IDX])) {
      i = 1;
      while (i < max_merge - 1 && cd->bypass()) ++i;
    }
    return i;
  }

  void parse_mvd(int* d) {
    const int g0x = cd->decode(ctx[CTX_MVD_G0]), g0y = cd->decode(ctx[CTX_MVD_G0]);
    const int g1x = g0x ? cd->decode(ctx[CTX_MVD_G1]) : 0, g1y = g0y ? cd->decode(ctx[CTX_MVD_G1]) : 0;
    int v[2] = {0, 0};
    const int g0[2] = {g0x, g0y}, g1[2] = {g1x, g1y};
    for (int c = 0; c < 2; ++c) {
      if (!g0[c]) continue;
      int a = 1;
      if (g1[c]) {  // EG1
        int k = 1, val = 0;
        while (cd->bypass()) {
          val += 1 << k;
          ++k;
        }
        val += static_cast<int>(cd->bypass_bits(k));
        a = val + 2;
      }
      v[c] = cd->bypass() ? -a : a;
    }
    d[0] = v[0];
    d[1] = v[1];
  }

  // 8.4.2 luma intra mode from the MPM syntax
  // cu: (x, y, n) of the current CU and the modes of its earlier PUs (NxN: the left / above
  // neighbour of a PU may be an earlier PU of the same CU, available in z-scan order)
  int derive_luma_mode(int x0, int y0, int prev, int mpm, int rem, const int* cu = nullptr, const int* pu_modes = nullptr) {
    auto cand_of = [&](int x, int y, bool above) {
      if (cu && x >= cu[0] && y >= cu[1] && x < cu[0] + cu[2] && y < cu[1] + cu[2]) {
        const int h = cu[2] / 2;
        return pu_modes[(x - cu[0] >= h) + 2 * (y - cu[1] >= h)];
      }
      if (!done(x, y)) return 1;
      if (g_pred[g4(x, y)] != CU_INTRA) return 1;
      if (above && (y >> sps.log2_ctb) != (y0 >> sps.log2_ctb)) return 1;
      return static_cast<int>(g_mode[g4(x, y)]);
    };
    const int a = cand_of(x0 - 1, y0, false), b = cand_of(x0, y0 - 1, true);
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

  // 6.4.2 prediction block availability (+ not intra)
  bool pb_avail(int xn, int yn) const { return done(xn, yn) && g_pred[g4(xn, yn)] == CU_INTER; }

  // 8.5.3.2.2-5 merge candidate idx of a 2Nx2N PU in a P slice (no temporal candidate)
  void merge_candidate(int xp, int yp, int n, int idx, int* mx, int* my) {
    int lx[5], ly[5], k = 0;
    struct N {
      int x, y;
      bool a;
    };
    const N a1{xp - 1, yp + n - 1, pb_avail(xp - 1, yp + n - 1)};
    const N b1{xp + n - 1, yp - 1, pb_avail(xp + n - 1, yp - 1)};
    const N b0{xp + n, yp - 1, pb_avail(xp + n, yp - 1)};
    const N a0{xp - 1, yp + n, pb_avail(xp - 1, yp + n)};
    const N b2{xp - 1, yp - 1, pb_avail(xp - 1, yp - 1)};
    auto same = [&](const N& p, const N& q) {
      return g_mvx[g4(p.x, p.y)] == g_mvx[g4(q.x, q.y)] && g_mvy[g4(p.x, p.y)] == g_mvy[g4(q.x, q.y)];
    };
    auto add = [&](const N& p) {
      lx[k] = g_mvx[g4(p.x, p.y)];
      ly[k] = g_mvy[g4(p.x, p.y)];
      ++k;
    };
    const bool fa1 = a1.a;
    const bool fb1 = b1.a && !(a1.a && same(a1, b1));
    const bool fb0 = b0.a && !(b1.a && same(b1, b0));
    const bool fa0 = a0.a && !(a1.a && same(a1, a0));
    const bool fb2 = b2.a && !(a1.a && same(a1, b2)) && !(b1.a && same(b1, b2)) && (fa0 + fa1 + fb0 + fb1) != 4;
    if (fa1) add(a1);
    if (fb1) add(b1);
    if (fb0) add(b0);
    if (fa0) add(a0);
    if (fb2) add(b2);
    while (k < 5) {
      lx[k] = 0;
      ly[k] = 0;
      ++k;
    }
    if (idx >= max_merge) throw std::runtime_error("HEVC: merge_idx out of range");
    *mx = lx[idx];
    *my = ly[idx];
  }

  // 8.5.3.2.6-7 luma motion vector predictor (single reference picture)
  void amvp_candidate(int xp, int yp, int n, int idx, int* mx, int* my) {
    const int xa[2] = {xp - 1, xp - 1}, ya[2] = {yp + n, yp + n - 1};
    const bool av0 = pb_avail(xa[0], ya[0]), av1 = pb_avail(xa[1], ya[1]);
    const bool is_scaled = av0 || av1;
    bool fa = false, fb = false;
    int ax = 0, ay = 0, bx = 0, by = 0;
    for (int k = 0; k < 2 && !fa; ++k)
      if (pb_avail(xa[k], ya[k])) {
        ax = g_mvx[g4(xa[k], ya[k])];
        ay = g_mvy[g4(xa[k], ya[k])];
        fa = true;
      }
    const int xb[3] = {xp + n, xp + n - 1, xp - 1};
    for (int k = 0; k < 3 && !fb; ++k)
      if (pb_avail(xb[k], yp - 1)) {
        bx = g_mvx[g4(xb[k], yp - 1)];
        by = g_mvy[g4(xb[k], yp - 1)];
        fb = true;
      }
    if (!is_scaled && fb) {
      fa = true;
      ax = bx;
      ay = by;
    }
    if (!is_scaled) {  // re-derivation of B (scaled path): with one reference it repeats the first available B
      fb = false;
      for (int k = 0; k < 3 && !fb; ++k)
        if (pb_avail(xb[k], yp - 1)) {
          bx = g_mvx[g4(xb[k], yp - 1)];
          by = g_mvy[g4(xb[k], yp - 1)];
          fb = true;
        }
    }
    int lx[2] = {0, 0}, ly[2] = {0, 0}, k = 0;
    if (fa) {
      lx[k] = ax;
      ly[k] = ay;
      ++k;
    }
    if (fb && !(fa && ax == bx && ay == by)) {
      lx[k] = bx;
      ly[k] = by;
      ++k;
    }
    *mx = lx[idx];
    *my = ly[idx];
  }

  // ------------------------------------------------------------ transform tree (7.3.8.8)
  // 7.3.8.8 (2Nx2N CUs): an explicit split_transform_flag where the depth allows it (inter
  // CUs with max_transform_hierarchy_depth_inter 1), chroma cbfs at each level with a set
  // parent cbf, cbf_luma coded below depth 0 or whenever chroma is coded
  void transform_tree(int x0, int y0, int log2, bool intra, int mode_y, int mode_c, int depth = 0, int pcb = 1,
                      int pcr = 1) {
    const int max_depth = intra ? sps.depth_intra : sps.depth_inter;
    if (log2 > sps.log2_max_tb) throw std::runtime_error("HEVC: implicit TU split unsupported");
    int split = 0;
    if (log2 <= sps.log2_max_tb && log2 > sps.log2_min_tb && depth < max_depth)
      split = cd->decode(ctx[CTX_SPLIT_TRANSFORM + 5 - log2]);
    int cbf_cb = 0, cbf_cr = 0;
    if (depth == 0 || pcb) cbf_cb = cd->decode(ctx[CTX_CBF_CHROMA + depth]);
    if (depth == 0 || pcr) cbf_cr = cd->decode(ctx[CTX_CBF_CHROMA + depth]);
    if (split) {
      if (intra || log2 - 1 < 3) throw std::runtime_error("HEVC: transform split below 8x8 / intra unsupported");
      const int h = 1 << (log2 - 1);
      for (int k = 0; k < 4; ++k) {
        const int xc = x0 + (k & 1) * h, yc = y0 + (k >> 1) * h;
        for (int j = 0; j < h; j += 4) {  // the child's boundary is a transform edge
          edge_v[g4(xc, yc + j)] = 1;
          edge_h[g4(xc + j, yc)] = 1;
        }
        if (sps.log2_ctb == kCtbLog2)
          for (int gy = yc; gy < yc + h; gy += 8)
            for (int gx = xc; gx < xc + h; gx += 8)
              rec_cu[static_cast<size_t>((gy >> kCtbLog2) * wctb + (gx >> kCtbLog2)) * kCusPerCtb +
                     zorder8((gx & 31) >> 3, (gy & 31) >> 3)].flags |= 16;
        transform_tree(xc, yc, log2 - 1, intra, mode_y, mode_c, depth + 1, cbf_cb, cbf_cr);
      }
      return;
    }
    int cbf_y = 1;
    if (intra || depth != 0 || cbf_cb || cbf_cr) cbf_y = cd->decode(ctx[CTX_CBF_LUMA + (depth == 0 ? 1 : 0)]);
    if (pps.cu_qp_delta && !qp_delta_coded && (cbf_y || cbf_cb || cbf_cr)) parse_qp_delta(x0, y0);
    if (log2 == 2) throw std::runtime_error("HEVC: 4x4 luma TUs unsupported");
    const int n = 1 << log2;
    for (int y = y0; y < y0 + n; y += 4)
      for (int x = x0; x < x0 + n; x += 4) g_cbf[g4(x, y)] = static_cast<int8_t>(cbf_y);
    if (cbf_y) residual(x0, y0, log2, 0, intra ? mode_y : -1);
    if (cbf_cb) residual(x0 / 2, y0 / 2, log2 - 1, 1, intra ? mode_c : -1);
    if (cbf_cr) residual(x0 / 2, y0 / 2, log2 - 1, 2, intra ? mode_c : -1);
    // reconstruction: prediction (intra) + residual
    if (intra) {
      predict_intra(x0, y0, log2, 0, mode_y);
      add_residual(x0, y0, log2, 0, cbf_y);
      predict_intra(x0 / 2, y0 / 2, log2 - 1, 1, mode_c);
      add_residual(x0 / 2, y0 / 2, log2 - 1, 1, cbf_cb);
      predict_intra(x0 / 2, y0 / 2, log2 - 1, 2, mode_c);
      add_residual(x0 / 2, y0 / 2, log2 - 1, 2, cbf_cr);
    } else {
      add_residual(x0, y0, log2, 0, cbf_y);
      add_residual(x0 / 2, y0 / 2, log2 - 1, 1, cbf_cb);
      add_residual(x0 / 2, y0 / 2, log2 - 1, 2, cbf_cr);
    }
  }

  // transform_tree of an intra PART_NxN CU (7.3.8.8): split_transform_flag inferred 1 at
  // depth 0 (IntraSplitFlag), chroma cbfs at depth 0, four 4x4 luma TUs (DST, z-order, each
  // predicted from the reconstruction of the previous ones), the 4x4 chroma blocks of the
  // CU after the last luma TU (blkIdx 3)
  void transform_tree_nxn(int x0, int y0, int log2, const int* m, int mode_c) {
    if (log2 - 1 != 2 || sps.depth_intra != 0) throw std::runtime_error("HEVC: NxN transform tree unsupported");
    const int cbf_cb = cd->decode(ctx[CTX_CBF_CHROMA + 0]);
    const int cbf_cr = cd->decode(ctx[CTX_CBF_CHROMA + 0]);
    const int h = 1 << (log2 - 1);
    for (int k = 0; k < 4; ++k) {
      const int xk = x0 + (k & 1) * h, yk = y0 + (k >> 1) * h;
      const int cbf_y = cd->decode(ctx[CTX_CBF_LUMA + 0]);  // trafoDepth 1
      for (int y = yk; y < yk + h; y += 4)
        for (int x = xk; x < xk + h; x += 4) g_cbf[g4(x, y)] = static_cast<int8_t>(cbf_y);
      if (pps.cu_qp_delta && !qp_delta_coded && (cbf_y || cbf_cb || cbf_cr)) parse_qp_delta(x0, y0);
      if (cbf_y) residual(xk, yk, 2, 0, m[k]);
      if (k == 3) {
        if (cbf_cb) residual(x0 / 2, y0 / 2, 2, 1, mode_c);
        if (cbf_cr) residual(x0 / 2, y0 / 2, 2, 2, mode_c);
      }
      predict_intra(xk, yk, 2, 0, m[k]);
      add_residual(xk, yk, 2, 0, cbf_y, true);
      mark_done(xk, yk, h);
    }
    predict_intra(x0 / 2, y0 / 2, 2, 1, mode_c);
    add_residual(x0 / 2, y0 / 2, 2, 1, cbf_cb);
    predict_intra(x0 / 2, y0 / 2, 2, 2, mode_c);
    add_residual(x0 / 2, y0 / 2, 2, 2, cbf_cr);
  }

  // ------------------------------------------------------------ residual_coding (7.3.8.11)
  int16_t tu_levels[32 * 32];

  void residual(int x0, int y0, int log2, int cidx, int intra_mode) {
    const int n = 1 << log2;
    int scan = 0;
    if (intra_mode >= 0 && (log2 == 2 || (log2 == 3 && cidx == 0))) {
      if (intra_mode >= 6 && intra_mode <= 14) scan = 2;
      else if (intra_mode >= 22 && intra_mode <= 30) scan = 1;
    }
    // last significant position
    int lx = parse_last_prefix(log2, cidx, CTX_LAST_X);
    int ly = parse_last_prefix(log2, cidx, CTX_LAST_Y);
    lx = parse_last_suffix(lx);
    ly = parse_last_suffix(ly);
    if (scan == 2) std::swap(lx, ly);
    std::vector<int> lev(n * n, 0);
    const int log2sb = log2 - 2, nsb = 1 << log2sb;
    // ScanOrder tables
    int sbx[64], sby[64], px[16], py[16];
    for (int i = 0; i < nsb * nsb; ++i) {
      const int p = scan_pos(scan, log2sb, i);
      sbx[i] = p & 255;
      sby[i] = p >> 8;
    }
    for (int i = 0; i < 16; ++i) {
      const int p = scan_pos(scan, 2, i);
      px[i] = p & 255;
      py[i] = p >> 8;
    }
    int last_sb = -1, last_pos = -1;
    for (int i = 0; i < nsb * nsb && last_sb < 0; ++i)
      for (int p = 0; p < 16; ++p)
        if (sbx[i] * 4 + px[p] == lx && sby[i] * 4 + py[p] == ly) {
          last_sb = i;
          last_pos = p;
          break;
        }
    if (last_sb < 0) throw std::runtime_error("HEVC: last position outside the block");
    uint8_t csbf[8][8] = {};
    int greater1_ctx_prev = 1;
    bool first_invocation = true;
    for (int i = last_sb; i >= 0; --i) {
      const int xs = sbx[i], ys = sby[i];
      bool infer_dc = false;
      if (i < last_sb && i > 0) {
        int cs = 0;
        if (xs < nsb - 1) cs += csbf[xs + 1][ys];
        if (ys < nsb - 1) cs += csbf[xs][ys + 1];
        csbf[xs][ys] = static_cast<uint8_t>(cd->decode(ctx[CTX_CSBF + std::min(cs, 1) + (cidx ? 2 : 0)]));
        infer_dc = true;
      } else {
        csbf[xs][ys] = 1;
      }
      int prev_csbf = 0;
      if (xs < nsb - 1) prev_csbf += csbf[xs + 1][ys];
      if (ys < nsb - 1) prev_csbf += csbf[xs][ys + 1] << 1;
      int sig[16] = {};
      if (i == last_sb) sig[last_pos] = 1;
      for (int p = (i == last_sb ? last_pos - 1 : 15); p >= 0; --p) {
        const int xc = xs * 4 + px[p], yc = ys * 4 + py[p];
        if (csbf[xs][ys] && (p > 0 || !infer_dc)) {
          sig[p] = cd->decode(ctx[CTX_SIG + sig_ctx_inc(xc, yc, log2, cidx, scan, prev_csbf, xs, ys)]);
          if (sig[p]) infer_dc = false;
        } else if (p == 0 && infer_dc && csbf[xs][ys]) {
          sig[p] = 1;
        }
      }
      if (!csbf[xs][ys]) continue;
      // 9.3.4.2.6 / 9.3.4.2.7 context sets
      int ctx_set = (i == 0 || cidx > 0) ? 0 : 2;
      if (!first_invocation && greater1_ctx_prev == 0) ++ctx_set;
      int greater1_ctx = 1;
      int g1[16] = {}, g2[16] = {};
      int num_g1 = 0, last_g1_pos = -1;
      bool any_sig = false;
      for (int p = 15; p >= 0; --p) {
        if (!sig[p]) continue;
        any_sig = true;
        if (num_g1 < 8) {
          g1[p] = cd->decode(ctx[CTX_GT1 + (cidx ? 16 : 0) + ctx_set * 4 + greater1_ctx]);
          ++num_g1;
          if (g1[p]) {
            greater1_ctx = 0;
            if (last_g1_pos < 0) last_g1_pos = p;
          } else if (greater1_ctx > 0 && greater1_ctx < 3) {
            ++greater1_ctx;
          }
        }
      }
      if (any_sig) {
        first_invocation = false;
        greater1_ctx_prev = greater1_ctx;
      }
      if (last_g1_pos >= 0) g2[last_g1_pos] = cd->decode(ctx[CTX_GT2 + (cidx ? 4 : 0) + ctx_set]);
      // 7.3.8.11 / 7.4.9.11 sign data hiding: the sign of the first significant coefficient
      // in scan order is not coded when the group's significant span exceeds 3 positions;
      // an odd sum of absolute levels makes it negative
      int first_sig = -1, last_sig = -1;
      for (int p = 0; p < 16; ++p)
        if (sig[p]) {
          if (first_sig < 0) first_sig = p;
          last_sig = p;
        }
      const bool hidden = pps.sign_hiding && first_sig >= 0 && last_sig - first_sig > 3;
      int sign[16] = {};
      for (int p = 15; p >= 0; --p)
        if (sig[p] && !(hidden && p == first_sig)) sign[p] = cd->bypass();
      int num_sig = 0, rice = 0, sum_abs = 0;
      for (int p = 15; p >= 0; --p) {
        if (!sig[p]) continue;
        const int base = 1 + g1[p] + g2[p];
        int a = base;
        const int thr = num_sig < 8 ? (p == last_g1_pos ? 3 : 2) : 1;
        if (base == thr) {
          const int rem = parse_remaining(rice);
          a = base + rem;
          if (a > 3 * (1 << rice)) rice = std::min(rice + 1, 4);
        }
        ++num_sig;
        sum_abs += a;
        if (hidden && p == first_sig) sign[p] = sum_abs & 1;  // p == first_sig is the last one coded
        lev[(ys * 4 + py[p]) * n + xs * 4 + px[p]] = sign[p] ? -a : a;
      }
    }
    // keep the levels (record output) and the dequantised block for reconstruction
    const int stride = cidx ? W / 2 : W;
    int16_t* rc = rec_coef[cidx].data() + static_cast<size_t>(y0) * stride + x0;
    for (int y = 0; y < n; ++y)
      for (int x = 0; x < n; ++x) rc[y * stride + x] = static_cast<int16_t>(clip3(-32768, 32767, lev[y * n + x]));
  }

  int parse_last_prefix(int log2, int cidx, int base) {
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
    while (v < cmax && cd->decode(ctx[base + off + (v >> shift)])) ++v;
    return v;
  }
  int parse_last_suffix(int prefix) {
    if (prefix <= 3) return prefix;
    const int nb = (prefix >> 1) - 1;
    const int s = static_cast<int>(cd->bypass_bits(nb));
    return (1 << nb) * (2 + (prefix & 1)) + s;
  }

  int parse_remaining(int rice) {
    int prefix = 0;
    while (prefix < 32 && cd->bypass()) ++prefix;
    if (prefix <= 3) return (prefix << rice) + static_cast<int>(cd->bypass_bits(rice));
    // prefix > 3: EG(rice + 1) escape of the value minus (4 << rice); prefix - 4 leading ones
    const int k = prefix - 4 + rice + 1;
    int v = 0;
    for (int i = rice + 1; i < k; ++i) v += 1 << i;
    return (4 << rice) + v + static_cast<int>(cd->bypass_bits(k));
  }

  static int sig_ctx_inc(int xc, int yc, int log2, int cidx, int scan, int prev_csbf, int xs, int ys) {
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

  // ------------------------------------------------------------ scaling + inverse transform (8.6.2 - 8.6.4)
  void add_residual(int x0, int y0, int log2, int cidx, int cbf, bool dst = false) {
    if (!cbf) return;
    const int n = 1 << log2;
    const int stride = cidx ? W / 2 : W;
    const int qpy_off = 6 * (bd - 8);
    int qpp;
    if (cidx == 0) {
      qpp = cu_qp + qpy_off;
    } else {
      const int off = cidx == 1 ? pps.cb_off : pps.cr_off;
      const int qpi = clip3(-qpy_off, 57, cu_qp + off);
      qpp = chroma_qp_map(qpi) + qpy_off;
    }
    const int bdshift = bd + log2 - 5;
    std::vector<int> d(n * n), e(n * n), r(n * n);
    const int16_t* lv = rec_coef[cidx].data() + static_cast<size_t>(y0) * stride + x0;
    for (int y = 0; y < n; ++y)
      for (int x = 0; x < n; ++x) {
        const int64_t v = static_cast<int64_t>(lv[y * stride + x]) * 16 * kLevelScale[qpp % 6] * (1LL << (qpp / 6));
        d[y * n + x] = clip3(-32768, 32767, static_cast<int>((v + (1LL << (bdshift - 1))) >> bdshift));
      }
    const int step = 32 >> log2;
    // 8.6.4.2 transMatrix: DCT rows of the 32-point matrix, or DST-VII (trType 1: 4x4 intra luma)
    auto dct_coef = [&](int k, int m) { return dst ? static_cast<int>(kDst4[k / step][m]) : hevc::dct_coef(k, m); };
    // columns (vertical), then clip to 16 bits after >> 7
    for (int x = 0; x < n; ++x)
      for (int y = 0; y < n; ++y) {
        int64_t s = 0;
        for (int k = 0; k < n; ++k) s += static_cast<int64_t>(dct_coef(k * step, y)) * d[k * n + x];
        e[y * n + x] = clip3(-32768, 32767, static_cast<int>((s + 64) >> 7));
      }
    const int sh2 = 20 - bd;
    for (int y = 0; y < n; ++y)
      for (int x = 0; x < n; ++x) {
        int64_t s = 0;
        for (int k = 0; k < n; ++k) s += static_cast<int64_t>(dct_coef(k * step, x)) * e[y * n + k];
        r[y * n + x] = static_cast<int>((s + (1LL << (sh2 - 1))) >> sh2);
      }
    uint16_t* pl = cur.pl[cidx].data() + static_cast<size_t>(y0) * stride + x0;
    for (int y = 0; y < n; ++y)
      for (int x = 0; x < n; ++x) pl[y * stride + x] = static_cast<uint16_t>(clip3(0, maxv, pl[y * stride + x] + r[y * n + x]));
  }

  // ------------------------------------------------------------ intra prediction (8.4.4.2)
  void predict_intra(int x0, int y0, int log2, int cidx, int mode) {
    const int n = 1 << log2;
    const int stride = cidx ? W / 2 : W;
    const int pw = cidx ? W / 2 : W, ph = cidx ? H / 2 : H;
    const int sc = cidx ? 1 : 0;  // luma location = component location << sc
    uint16_t* pl = cur.pl[cidx].data();
    // reference samples: ref index 0 = p[-1][2n-1] (bottom) ... 2n-1 = p[-1][0], 2n = p[-1][-1], 2n+1.. = p[0..2n-1][-1]
    const int total = 4 * n + 1;
    std::vector<int> p(total), av(total);
    auto sample_avail = [&](int xc, int yc) {
      if (xc < 0 || yc < 0 || xc >= pw || yc >= ph) return false;
      return done(xc << sc, yc << sc);
    };
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
      av[i] = sample_avail(xc, yc);
      if (av[i]) {
        p[i] = pl[static_cast<size_t>(yc) * stride + xc];
        ++navail;
      }
    }
    if (navail == 0) {
      for (int i = 0; i < total; ++i) p[i] = 1 << (bd - 1);
    } else {
      if (!av[0]) {
        for (int i = 1; i < total; ++i)
          if (av[i]) {
            p[0] = p[i];
            break;
          }
      }
      for (int i = 1; i < total; ++i)
        if (!av[i]) p[i] = p[i - 1];
    }
    auto L = [&](int y) { return p[2 * n - 1 - y]; };  // p[-1][y], y = -1 .. 2n-1
    auto T = [&](int x) { return p[2 * n + 1 + x]; };  // p[x][-1], x = -1 .. 2n-1
    // 8.4.4.2.3 filtering (luma only for 4:2:0)
    if (cidx == 0 && mode != 1 && n != 4) {
      const int md = std::min(std::abs(mode - 26), std::abs(mode - 10));
      const int thr = n == 8 ? 7 : (n == 16 ? 1 : 0);
      if (md > thr) {
        std::vector<int> f(total);
        const int tl = T(-1), bl = L(2 * n - 1), tr = T(2 * n - 1);
        const bool bi = sps.strong && n == 32 && std::abs(tl + tr - 2 * T(n - 1)) < (1 << (bd - 5)) &&
                        std::abs(tl + bl - 2 * L(n - 1)) < (1 << (bd - 5));
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
        p = f;
      }
    }
    uint16_t* dst = pl + static_cast<size_t>(y0) * stride + x0;
    if (mode == 0) {  // planar
      for (int y = 0; y < n; ++y)
        for (int x = 0; x < n; ++x)
          dst[y * stride + x] = static_cast<uint16_t>(((n - 1 - x) * L(y) + (x + 1) * T(n) + (n - 1 - y) * T(x) + (y + 1) * L(n) + n) >> (log2 + 1));
      return;
    }
    if (mode == 1) {  // DC
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
    std::vector<int> refa(3 * n + 2);
    int* ref = refa.data() + n;  // ref[-n .. 2n]
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
        for (int x = 0; x < n; ++x) {
          const int v = fact ? ((32 - fact) * ref[x + idx + 1] + fact * ref[x + idx + 2] + 16) >> 5 : ref[x + idx + 1];
          dst[y * stride + x] = static_cast<uint16_t>(v);
        }
      }
      if (mode == 26 && cidx == 0 && n < 32)
        for (int y = 0; y < n; ++y) dst[y * stride] = static_cast<uint16_t>(clip3(0, maxv, T(0) + ((L(y) - L(-1)) >> 1)));
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
        for (int y = 0; y < n; ++y) {
          const int v = fact ? ((32 - fact) * ref[y + idx + 1] + fact * ref[y + idx + 2] + 16) >> 5 : ref[y + idx + 1];
          dst[y * stride + x] = static_cast<uint16_t>(v);
        }
      }
      if (mode == 10 && cidx == 0 && n < 32)
        for (int x = 0; x < n; ++x) dst[x] = static_cast<uint16_t>(clip3(0, maxv, L(0) + ((T(x) - T(-1)) >> 1)));
    }
  }

  // ------------------------------------------------------------ inter prediction (8.5.3.3)
  void predict_inter(int x0, int y0, int n, int mvx, int mvy) {
    const int sh1 = std::min(4, bd - 8), sh3 = std::max(2, 14 - bd);
    const int wsh = 14 - bd, woff = wsh > 0 ? 1 << (wsh - 1) : 0;
    for (int c = 0; c < 3; ++c) {
      const int pw = c ? W / 2 : W, ph = c ? H / 2 : H, bs = c ? n / 2 : n;
      const int bx = c ? x0 / 2 : x0, by = c ? y0 / 2 : y0;
      const int fx = c ? (mvx & 7) : (mvx & 3), fy = c ? (mvy & 7) : (mvy & 3);
      const int ix = c ? (mvx >> 3) : (mvx >> 2), iy = c ? (mvy >> 3) : (mvy >> 2);
      const uint16_t* rp = ref.pl[c].data();
      auto R = [&](int x, int y) { return static_cast<int>(rp[static_cast<size_t>(clip3(0, ph - 1, y)) * pw + clip3(0, pw - 1, x)]); };
      const int ntap = c ? 4 : 8, half = c ? 1 : 3;
      auto tap = [&](int f, int i) { return c ? kChromaTaps[f][i] : kLumaTaps[f][i]; };
      uint16_t* dst = cur.pl[c].data();
      for (int y = 0; y < bs; ++y)
        for (int x = 0; x < bs; ++x) {
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
          dst[static_cast<size_t>(by + y) * pw + bx + x] = static_cast<uint16_t>(clip3(0, maxv, (v + woff) >> wsh));
        }
    }
  }

  // ------------------------------------------------------------ deblocking (8.7.2)
  int bs_at(int xp, int yp, int xq, int yq, bool tu_edge) const {
    const size_t p = g4(xp, yp), q = g4(xq, yq);
    if (g_pred[p] == CU_INTRA || g_pred[q] == CU_INTRA) return 2;
    if (tu_edge && (g_cbf[p] || g_cbf[q])) return 1;
    if (std::abs(g_mvx[p] - g_mvx[q]) >= 4 || std::abs(g_mvy[p] - g_mvy[q]) >= 4) return 1;
    return 0;
  }

  void filter_luma(uint16_t* s, int step, int across, int bs, int qpl) {
    // s: first of 4 lines at q0; step: between lines; across: sample step across the edge
    const int qb = clip3(0, 51, qpl + pps.beta_off);
    const int qt = clip3(0, 53, qpl + 2 * (bs - 1) + pps.tc_off);
    const int beta = kBetaTable[qb] * (1 << (bd - 8)), tc = kTcTable[qt] * (1 << (bd - 8));
    auto P = [&](int line, int i) -> uint16_t& { return s[line * step - (i + 1) * across]; };
    auto Q = [&](int line, int i) -> uint16_t& { return s[line * step + i * across]; };
    const int dp0 = std::abs(P(0, 2) - 2 * P(0, 1) + P(0, 0)), dp3 = std::abs(P(3, 2) - 2 * P(3, 1) + P(3, 0));
    const int dq0 = std::abs(Q(0, 2) - 2 * Q(0, 1) + Q(0, 0)), dq3 = std::abs(Q(3, 2) - 2 * Q(3, 1) + Q(3, 0));
    const int dpq0 = dp0 + dq0, dpq3 = dp3 + dq3, dp = dp0 + dp3, dq = dq0 + dq3, d = dpq0 + dpq3;
    if (d >= beta) return;
    auto dsam = [&](int l, int dpq) {
      return 2 * dpq < (beta >> 2) && std::abs(P(l, 3) - P(l, 0)) + std::abs(Q(l, 0) - Q(l, 3)) < (beta >> 3) &&
             std::abs(P(l, 0) - Q(l, 0)) < ((5 * tc + 1) >> 1);
    };
    const bool strong = dsam(0, dpq0) && dsam(3, dpq3);
    const bool dep = dp < ((beta + (beta >> 1)) >> 3), deq = dq < ((beta + (beta >> 1)) >> 3);
    for (int l = 0; l < 4; ++l) {
      const int p0 = P(l, 0), p1 = P(l, 1), p2 = P(l, 2), p3 = P(l, 3);
      const int q0 = Q(l, 0), q1 = Q(l, 1), q2 = Q(l, 2), q3 = Q(l, 3);
      if (strong) {
        P(l, 0) = static_cast<uint16_t>(clip3(p0 - 2 * tc, p0 + 2 * tc, (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3));
        P(l, 1) = static_cast<uint16_t>(clip3(p1 - 2 * tc, p1 + 2 * tc, (p2 + p1 + p0 + q0 + 2) >> 2));
        P(l, 2) = static_cast<uint16_t>(clip3(p2 - 2 * tc, p2 + 2 * tc, (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3));
        Q(l, 0) = static_cast<uint16_t>(clip3(q0 - 2 * tc, q0 + 2 * tc, (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3));
        Q(l, 1) = static_cast<uint16_t>(clip3(q1 - 2 * tc, q1 + 2 * tc, (p0 + q0 + q1 + q2 + 2) >> 2));
        Q(l, 2) = static_cast<uint16_t>(clip3(q2 - 2 * tc, q2 + 2 * tc, (p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3));
      } else {
        int delta = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4;
        if (std::abs(delta) >= tc * 10) continue;
        delta = clip3(-tc, tc, delta);
        P(l, 0) = static_cast<uint16_t>(clip3(0, maxv, p0 + delta));
        Q(l, 0) = static_cast<uint16_t>(clip3(0, maxv, q0 - delta));
        if (dep) {
          const int dlt = clip3(-(tc >> 1), tc >> 1, (((p2 + p0 + 1) >> 1) - p1 + delta) >> 1);
          P(l, 1) = static_cast<uint16_t>(clip3(0, maxv, p1 + dlt));
        }
        if (deq) {
          const int dlt = clip3(-(tc >> 1), tc >> 1, (((q2 + q0 + 1) >> 1) - q1 - delta) >> 1);
          Q(l, 1) = static_cast<uint16_t>(clip3(0, maxv, q1 + dlt));
        }
      }
    }
  }

  void filter_chroma(uint16_t* s, int step, int across, int qpl_avg, int cidx) {
    const int off = cidx == 1 ? pps.cb_off : pps.cr_off;
    const int qpc = chroma_qp_map(qpl_avg + off);  // ChromaArrayType 1: Table 8-10 on qPi
    const int qt = clip3(0, 53, qpc + 2 + pps.tc_off);
    const int tc = kTcTable[qt] * (1 << (bd - 8));
    for (int l = 0; l < 2; ++l) {
      uint16_t* q = s + l * step;
      const int p0 = q[-across], p1 = q[-2 * across], q0 = q[0], q1 = q[across];
      const int delta = clip3(-tc, tc, ((((q0 - p0) << 2) + p1 - q1 + 4) >> 3));
      q[-across] = static_cast<uint16_t>(clip3(0, maxv, p0 + delta));
      q[0] = static_cast<uint16_t>(clip3(0, maxv, q0 - delta));
    }
  }

  void deblocking() {
    for (int dir = 0; dir < 2; ++dir) {
      // bS for every 4-sample segment of every 8x8-grid edge, from the unfiltered state
      std::vector<int8_t> bsv(static_cast<size_t>(w4) * h4, 0);
      for (int y = 0; y < H; y += 4)
        for (int x = 0; x < W; x += 4) {
          const bool on_grid = dir == 0 ? (x % 8 == 0 && x > 0) : (y % 8 == 0 && y > 0);
          if (!on_grid) continue;
          const bool edge = dir == 0 ? edge_v[g4(x, y)] : edge_h[g4(x, y)];
          if (!edge) continue;
          bsv[g4(x, y)] = static_cast<int8_t>(dir == 0 ? bs_at(x - 1, y, x, y, true) : bs_at(x, y - 1, x, y, true));
        }
      // luma
      for (int y = 0; y < H; y += 4)
        for (int x = 0; x < W; x += 4) {
          const int bs = bsv[g4(x, y)];
          if (!bs) continue;
          const size_t pq = dir == 0 ? g4(x - 1, y) : g4(x, y - 1);
          const int qpl = (g_qp[pq] + g_qp[g4(x, y)] + 1) >> 1;
          uint16_t* s = cur.pl[0].data() + static_cast<size_t>(y) * W + x;
          if (dir == 0) filter_luma(s, W, 1, bs, qpl);
          else filter_luma(s, 1, W, bs, qpl);
        }
      // chroma: edges on the 8x8 chroma grid (16 luma samples), bS == 2
      for (int c = 1; c < 3; ++c)
        for (int y = 0; y < H; y += 4)
          for (int x = 0; x < W; x += 4) {
            if (bsv[g4(x, y)] != 2) continue;
            if (dir == 0 ? (x % 16) : (y % 16)) continue;
            const size_t pq = dir == 0 ? g4(x - 1, y) : g4(x, y - 1);
            const int qpl = (g_qp[pq] + g_qp[g4(x, y)] + 1) >> 1;
            uint16_t* s = cur.pl[c].data() + static_cast<size_t>(y / 2) * (W / 2) + x / 2;
            if (dir == 0) filter_chroma(s, W / 2, 1, qpl, c);
            else filter_chroma(s, 1, W / 2, qpl, c);
          }
    }
  }

  // ------------------------------------------------------------ SAO (8.7.3)
  void apply_sao() {
    const int ctb = 1 << sps.log2_ctb;
    for (int c = 0; c < 3; ++c) {
      if ((c == 0 && !sao_luma) || (c > 0 && !sao_chroma)) continue;
      const int pw = c ? W / 2 : W, ph = c ? H / 2 : H, cs = c ? ctb / 2 : ctb;
      const std::vector<uint16_t> src = cur.pl[c];  // deblocked input
      uint16_t* dst = cur.pl[c].data();
      for (int ry = 0; ry < hctb; ++ry)
        for (int rx = 0; rx < wctb; ++rx) {
          const CtuInfo& t = rec_ctu[ry * wctb + rx];
          const int type = t.sao_type[c ? 1 : 0];
          if (!type) continue;
          const int x0 = rx * cs, y0 = ry * cs;
          if (type == 1) {
            int table[32] = {};
            for (int k = 0; k < 4; ++k) table[(k + t.sao_band[c]) & 31] = k + 1;
            const int sh = bd - 5;
            for (int y = y0; y < std::min(y0 + cs, ph); ++y)
              for (int x = x0; x < std::min(x0 + cs, pw); ++x) {
                const int v = src[static_cast<size_t>(y) * pw + x];
                const int b = table[v >> sh];
                if (b) dst[static_cast<size_t>(y) * pw + x] = static_cast<uint16_t>(clip3(0, maxv, v + t.sao_off[c][b - 1]));
              }
          } else {
            static const int hp[4][2] = {{-1, 1}, {0, 0}, {-1, 1}, {1, -1}};
            static const int vp[4][2] = {{0, 0}, {-1, 1}, {-1, 1}, {-1, 1}};
            const int cl = t.sao_class[c ? 1 : 0];
            for (int y = y0; y < std::min(y0 + cs, ph); ++y)
              for (int x = x0; x < std::min(x0 + cs, pw); ++x) {
                const int xa = x + hp[cl][0], ya = y + vp[cl][0], xb = x + hp[cl][1], yb = y + vp[cl][1];
                if (xa < 0 || ya < 0 || xb < 0 || yb < 0 || xa >= pw || xb >= pw || ya >= ph || yb >= ph) continue;
                const int v = src[static_cast<size_t>(y) * pw + x];
                int e = 2 + sgn(v - src[static_cast<size_t>(ya) * pw + xa]) + sgn(v - src[static_cast<size_t>(yb) * pw + xb]);
                if (e <= 2) e = (e == 2) ? 0 : e + 1;
                if (e) dst[static_cast<size_t>(y) * pw + x] = static_cast<uint16_t>(clip3(0, maxv, v + t.sao_off[c][e - 1]));
              }
          }
        }
    }
  }
};

HevcDecoder::HevcDecoder() : impl_(new Impl) {}
HevcDecoder::~HevcDecoder() = default;

void HevcDecoder::decode(const uint8_t* data, size_t n) {
  impl_->skip_filters = skip_filters_;
  std::vector<NalUnit> nals = parse_annexb(data, n);
  for (const NalUnit& u : nals) {
    if (u.rbsp.empty()) continue;
    // parse_annexb reads the first header byte as an H.264 header: recover the HEVC type
    const uint8_t h0 = data[u.offset + (data[u.offset + 2] == 1 ? 3 : 4)];
    const int type = (h0 >> 1) & 63;
    BitReader br(u.rbsp.data() + 1, u.rbsp.size() - 1);
    if (type == 32) continue;  // VPS
    if (type == 33) impl_->parse_sps(br);
    else if (type == 34) impl_->parse_pps(br);
    else if (type <= 21) impl_->decode_slice(u, type, out_);
  }
}

}  // namespace hevc
}  // namespace mivc
