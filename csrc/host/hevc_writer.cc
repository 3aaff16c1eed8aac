// HEVC parameter sets, slice header and CABAC slice data from decision records.
// Clause numbers refer to ITU-T H.265.  See hevc_codec.h for the coding-tool subset.
#include <algorithm>
#include <array>
#include <memory>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <exception>
#include <stdexcept>
#include <thread>

#include "bitstream.h"
#include "hevc_cabac.h"
#include "hevc_codec.h"

namespace mivc {
namespace hevc {

namespace {

enum NalType { NAL_TRAIL_N = 0, NAL_TRAIL_R = 1, NAL_IDR_W_RADL = 19, NAL_VPS = 32, NAL_SPS = 33, NAL_PPS = 34 };

void append_hevc_nal(std::vector<uint8_t>& out, int type, const std::vector<uint8_t>& rbsp) {
  static const uint8_t sc[4] = {0, 0, 0, 1};
  out.insert(out.end(), sc, sc + 4);
  out.push_back(static_cast<uint8_t>((type & 63) << 1));  // forbidden 0, type, layer id 0 (high bit)
  out.push_back(1);                                       // layer id low bits 0, temporal_id_plus1 = 1
  int zeros = 0;
  for (uint8_t b : rbsp) {
    if (zeros >= 2 && b <= 3) {
      out.push_back(3);
      zeros = 0;
    }
    out.push_back(b);
    zeros = (b == 0) ? zeros + 1 : 0;
  }
}

int auto_level_idc(const HevcConfig& c);

int level_idc(const HevcConfig& c) {
  const int need = auto_level_idc(c);
  if (c.level_idc <= 0) return need;
  if (c.level_idc < need)
    throw std::runtime_error("HEVC: picture size / frame rate exceed the requested level_idc " + std::to_string(c.level_idc));
  return c.level_idc;
}

int auto_level_idc(const HevcConfig& c) {
  const int64_t ps = static_cast<int64_t>(c.coded_width()) * c.coded_height();
  const double sps = ps * c.fps;
  // Table A.8 (MaxLumaPs, MaxLumaSr); level_idc = 30 * level
  if (ps <= 552960 && sps <= 16588800) return 93;      // 3.1
  if (ps <= 2228224 && sps <= 66846720) return 120;    // 4
  if (ps <= 2228224 && sps <= 133693440) return 123;   // 4.1
  if (ps <= 8912896 && sps <= 267386880) return 150;   // 5
  if (ps <= 8912896 && sps <= 534773760) return 153;   // 5.1
  if (ps <= 35651584 && sps <= 1069547520) return 180; // 6
  if (ps <= 35651584 && sps <= 2139095040) return 183; // 6.1
  return 186;                                          // 6.2
}

// DPB size / reordering of the GOP structures this encoder writes (models/gop.py): P only
// (1 reference + current), B pictures between two anchors (2 + current, 1 reordered),
// a pyramid with a reference B (3 + current, 2 reordered)
// (x265 --ref R: R list-0 pictures + the current one, one more with a reference B)
int dpb_minus1(const HevcConfig& c) {
  const int base = c.bframes <= 0 ? 1 : (c.pyramid && c.bframes > 1 ? 3 : 2);
  return std::max(base, c.refs + (c.pyramid && c.bframes > 1 ? 1 : 0));
}
int num_reorder(const HevcConfig& c) { return c.bframes <= 0 ? 0 : (c.pyramid && c.bframes > 1 ? 2 : 1); }

void profile_tier_level(BitWriter& bw, const HevcConfig& c) {
  const int profile = c.bit_depth > 8 ? 2 : 1;  // Main 10 / Main
  bw.put(0, 2);            // general_profile_space
  bw.put(0, 1);            // general_tier_flag
  bw.put(profile, 5);      // general_profile_idc
  for (int j = 0; j < 32; ++j) bw.put_bit(j == profile || (profile == 1 && j == 2));
  bw.put_bit(1);           // general_progressive_source_flag
  bw.put_bit(0);           // general_interlaced_source_flag
  bw.put_bit(0);           // general_non_packed_constraint_flag
  bw.put_bit(1);           // general_frame_only_constraint_flag
  bw.put(0, 32);           // general_reserved_zero_43bits (+ inbld flag)
  bw.put(0, 12);
  bw.put(level_idc(c), 8); // general_level_idc
}

}  // namespace

std::vector<uint8_t> hevc_parameter_sets(const HevcConfig& c) {
  std::vector<uint8_t> out;
  {  // 7.3.2.1 video_parameter_set_rbsp
    BitWriter bw;
    bw.put(0, 4);        // vps_video_parameter_set_id
    bw.put_bit(1);       // vps_base_layer_internal_flag
    bw.put_bit(1);       // vps_base_layer_available_flag
    bw.put(0, 6);        // vps_max_layers_minus1
    bw.put(0, 3);        // vps_max_sub_layers_minus1
    bw.put_bit(1);       // vps_temporal_id_nesting_flag
    bw.put(0xFFFF, 16);  // vps_reserved_0xffff_16bits
    profile_tier_level(bw, c);
    bw.put_bit(1);       // vps_sub_layer_ordering_info_present_flag
    bw.put_ue(dpb_minus1(c));  // vps_max_dec_pic_buffering_minus1
    bw.put_ue(num_reorder(c));  // vps_max_num_reorder_pics
    bw.put_ue(0);        // vps_max_latency_increase_plus1
    bw.put(0, 6);        // vps_max_layer_id
    bw.put_ue(0);        // vps_num_layer_sets_minus1
    bw.put_bit(0);       // vps_timing_info_present_flag
    bw.put_bit(0);       // vps_extension_flag
    bw.trailing();
    append_hevc_nal(out, NAL_VPS, bw.bytes());
  }
  {  // 7.3.2.2 seq_parameter_set_rbsp
    BitWriter bw;
    bw.put(0, 4);        // sps_video_parameter_set_id
    bw.put(0, 3);        // sps_max_sub_layers_minus1
    bw.put_bit(1);       // sps_temporal_id_nesting_flag
    profile_tier_level(bw, c);
    bw.put_ue(0);        // sps_seq_parameter_set_id
    bw.put_ue(1);        // chroma_format_idc 4:2:0
    bw.put_ue(c.coded_width());
    bw.put_ue(c.coded_height());
    const int crop_r = (c.coded_width() - c.width) / 2, crop_b = (c.coded_height() - c.height) / 2;
    bw.put_bit(crop_r || crop_b);  // conformance_window_flag
    if (crop_r || crop_b) {
      bw.put_ue(0);
      bw.put_ue(crop_r);
      bw.put_ue(0);
      bw.put_ue(crop_b);
    }
    bw.put_ue(c.bit_depth - 8);  // bit_depth_luma_minus8
    bw.put_ue(c.bit_depth - 8);  // bit_depth_chroma_minus8
    bw.put_ue(8 - 4);            // log2_max_pic_order_cnt_lsb_minus4 (8 bits)
    bw.put_bit(1);               // sps_sub_layer_ordering_info_present_flag
    bw.put_ue(dpb_minus1(c));    // sps_max_dec_pic_buffering_minus1
    bw.put_ue(num_reorder(c));   // sps_max_num_reorder_pics
    bw.put_ue(0);                // sps_max_latency_increase_plus1
    bw.put_ue(kMinCbLog2 - 3);   // log2_min_luma_coding_block_size_minus3
    bw.put_ue(c.ctb_log2() - kMinCbLog2);  // log2_diff_max_min_luma_coding_block_size
    bw.put_ue(0);                // log2_min_luma_transform_block_size_minus2 (4x4)
    bw.put_ue(3);                // log2_diff_max_min_luma_transform_block_size (32x32)
    bw.put_ue(c.tu_inter_depth);  // max_transform_hierarchy_depth_inter (x265 --tu-inter-depth)
    bw.put_ue(0);                // max_transform_hierarchy_depth_intra
    bw.put_bit(0);               // scaling_list_enabled_flag
    bw.put_bit(0);               // amp_enabled_flag
    bw.put_bit(c.sao ? 1 : 0);   // sample_adaptive_offset_enabled_flag
    bw.put_bit(0);               // pcm_enabled_flag
    bw.put_ue(1);                // num_short_term_ref_pic_sets
    // st_ref_pic_set(0): the previous picture
    bw.put_ue(1);                // num_negative_pics
    bw.put_ue(0);                // num_positive_pics
    bw.put_ue(0);                // delta_poc_s0_minus1
    bw.put_bit(1);               // used_by_curr_pic_s0_flag
    bw.put_bit(0);               // long_term_ref_pics_present_flag
    bw.put_bit(c.tmvp ? 1 : 0);  // sps_temporal_mvp_enabled_flag
    bw.put_bit(1);               // strong_intra_smoothing_enabled_flag
    bw.put_bit(0);               // vui_parameters_present_flag
    bw.put_bit(0);               // sps_extension_present_flag
    bw.trailing();
    append_hevc_nal(out, NAL_SPS, bw.bytes());
  }
  {  // 7.3.2.3 pic_parameter_set_rbsp
    BitWriter bw;
    bw.put_ue(0);   // pps_pic_parameter_set_id
    bw.put_ue(0);   // pps_seq_parameter_set_id
    bw.put_bit(0);  // dependent_slice_segments_enabled_flag
    bw.put_bit(0);  // output_flag_present_flag
    bw.put(0, 3);   // num_extra_slice_header_bits
    bw.put_bit(c.sdh ? 1 : 0);  // sign_data_hiding_enabled_flag
    bw.put_bit(0);  // cabac_init_present_flag
    bw.put_ue(0);   // num_ref_idx_l0_default_active_minus1
    bw.put_ue(0);   // num_ref_idx_l1_default_active_minus1
    bw.put_se(0);   // init_qp_minus26
    bw.put_bit(0);  // constrained_intra_pred_flag
    bw.put_bit(0);  // transform_skip_enabled_flag
    bw.put_bit(c.cu_qp_delta ? 1 : 0);  // cu_qp_delta_enabled_flag
    // diff_cu_qp_delta_depth: one quantization group per 32x32 block (per CTB, or 4 per 64x64 CTU)
    if (c.cu_qp_delta) bw.put_ue(c.ctu64 ? 1 : 0);
    bw.put_se(0);   // pps_cb_qp_offset
    bw.put_se(0);   // pps_cr_qp_offset
    bw.put_bit(0);  // pps_slice_chroma_qp_offsets_present_flag
    bw.put_bit(c.weightp ? 1 : 0);  // weighted_pred_flag
    bw.put_bit(0);  // weighted_bipred_flag
    bw.put_bit(0);  // transquant_bypass_enabled_flag
    bw.put_bit(0);  // tiles_enabled_flag
    bw.put_bit(c.wpp ? 1 : 0);  // entropy_coding_sync_enabled_flag
    bw.put_bit(0);  // pps_loop_filter_across_slices_enabled_flag
    bw.put_bit(c.deblock ? 0 : 1);  // deblocking_filter_control_present_flag
    if (!c.deblock) {
      bw.put_bit(0);  // deblocking_filter_override_enabled_flag
      bw.put_bit(1);  // pps_deblocking_filter_disabled_flag
    }
    bw.put_bit(0);  // pps_scaling_list_data_present_flag
    bw.put_bit(0);  // lists_modification_present_flag
    bw.put_ue(0);   // log2_parallel_merge_level_minus2
    bw.put_bit(0);  // slice_segment_header_extension_present_flag
    bw.put_bit(0);  // pps_extension_present_flag
    bw.trailing();
    append_hevc_nal(out, NAL_PPS, bw.bytes());
  }
  return out;
}

namespace {

// ------------------------------------------------------------------ slice writer state
struct Mv {
  int x, y;
  bool operator==(const Mv& o) const { return x == o.x && y == o.y; }
};
// motion of a PU: direction (bit 0 list 0, bit 1 list 1), refIdx and vector per used list
struct Motion {
  uint8_t dir = 0;
  int8_t r[2] = {0, 0};
  Mv m[2] = {{0, 0}, {0, 0}};
  bool operator==(const Motion& o) const {
    return dir == o.dir && (!(dir & 1) || (m[0] == o.m[0] && r[0] == o.r[0])) &&
           (!(dir & 2) || (m[1] == o.m[1] && r[1] == o.r[1]));
  }
};

struct PicState {
  std::vector<int8_t> depth, skip, pred, mode4;  // mode4: luma intra mode per 4x4 block (NxN PUs)
  std::vector<Motion> mot;
  std::vector<uint8_t> coded;
  std::vector<int8_t> qpy;  // QpY of the CU covering the granule (QP prediction inside a 64x64 CTU)
  explicit PicState(size_t n)
      : depth(n, 0), skip(n, 0), pred(n, 0), mode4(4 * n, 1), mot(n), coded(n, 0), qpy(n, 0) {}
};

struct Writer {
  const HevcConfig& c;
  const HevcFrameParams& fp;
  const CtuInfo* ctu;
  const CuInfo* cu;
  const int16_t* coef[3];
  CabacEncoder& e;
  CtxState ctx[kNumCtx];
  HevcSliceStats st;
  int W, H, wctb, hctb, w8, h8;
  bool inter_slice, bslice;
  bool tmvp;         // slice_temporal_mvp_enabled_flag
  bool col_l1;       // the collocated picture is RefPicList1[0] (B: collocated_from_l0_flag 0)
  bool no_backward;  // NoBackwardPredFlag: no reference picture follows the current one
  // per 8x8 granule of the picture (raster): state of already-coded CUs, shared by the
  // substream writers of one picture (WPP rows only read granules their 2-CTB lag
  // guarantees are final)
  std::vector<int8_t>&depth, &skip, &pred, &mode4;
  std::vector<Motion>& mot;
  std::vector<uint8_t>& coded;
  std::vector<int8_t>& qpy;
  // cu_qp_delta state (7.4.9.14, 8.6.1): qPY_PREV of the next quantization group (the
  // slice QP at the start of the slice and, with WPP, of every CTB row: a Writer codes
  // one row substream or the whole slice), and whether the current CTB coded its delta
  int qp_prev = 0, qp_ctb = 0;
  bool qp_coded = false;
  int qp_pred_cur = 0;  // qPY_PRED of the current quantization group (8.6.1)
  int L = kCtbLog2;     // CtbLog2SizeY

  // packed coefficient source (hevc_write_slice_packed): per CTB the sub-block maps
  // (nzmap[2 * ci]: luma bit by * 8 + bx; nzmap[2 * ci + 1]: Cb bits 0-15, Cr bits 16-31,
  // by * 4 + bx), the CTB's first block in `packed` and the non-zero 4x4 blocks (16 levels
  // each, raster) in luma, Cb, Cr, bit order
  const PackedLevels* pk = nullptr;
  uint32_t ctb_base = 0;

  Writer(const HevcConfig& cfg, const HevcFrameParams& f, const CtuInfo* ct, const CuInfo* cu_, const int16_t* cy,
         const int16_t* cb, const int16_t* cr, CabacEncoder& enc, PicState& ps)
      : c(cfg), fp(f), ctu(ct), cu(cu_), e(enc), depth(ps.depth), skip(ps.skip), pred(ps.pred), mode4(ps.mode4),
        mot(ps.mot), coded(ps.coded), qpy(ps.qpy) {
    coef[0] = cy;
    coef[1] = cb;
    coef[2] = cr;
    W = c.coded_width();
    H = c.coded_height();
    wctb = c.wctb();
    hctb = c.hctb();
    w8 = W / 8;
    h8 = H / 8;
    inter_slice = fp.slice_type != 2;
    bslice = fp.slice_type == 0;
    tmvp = inter_slice && c.tmvp;
    col_l1 = bslice;
    no_backward = true;  // NoBackwardPredFlag: no picture of either list follows the current one
    for (int l = 0; l < (bslice ? 2 : 1); ++l)
      for (int i = 0; i < nref(l); ++i) no_backward = no_backward && list_poc(l, i) <= fp.poc;
    L = c.ctb_log2();
    init_contexts(ctx, bslice ? 2 : (inter_slice ? 1 : 0), fp.qp);
    qp_prev = fp.qp;
  }

  size_t g(int x, int y) const { return static_cast<size_t>(y >> 3) * w8 + (x >> 3); }
  size_t g4(int x, int y) const { return static_cast<size_t>(y >> 2) * (2 * w8) + (x >> 2); }
  bool inside(int x, int y) const { return x >= 0 && y >= 0 && x < W && y < H; }
  // 6.4.1 z-scan availability at 8x8 granularity (the granule is coded iff already visited)
  bool avail(int x, int y) const { return inside(x, y) && coded[g(x, y)]; }

  const CuInfo& cu_at(int x, int y) const {
    const int ci = (y >> kCtbLog2) * wctb + (x >> kCtbLog2);
    return cu[static_cast<size_t>(ci) * kCusPerCtb + zorder8((x & (kCtb - 1)) >> 3, (y & (kCtb - 1)) >> 3)];
  }

  // ---------------------------------------------------------------- SAO (7.3.8.3)
  static bool same_sao(const CtuInfo& a, const CtuInfo& b) {
    for (int k = 0; k < 2; ++k)
      if (a.sao_type[k] != b.sao_type[k] || (a.sao_type[k] == 2 && a.sao_class[k] != b.sao_class[k])) return false;
    for (int ci = 0; ci < 3; ++ci) {
      const int t = a.sao_type[ci ? 1 : 0];
      if (t == 0) continue;
      if (t == 1 && a.sao_band[ci] != b.sao_band[ci]) return false;
      for (int i = 0; i < 4; ++i)
        if (a.sao_off[ci][i] != b.sao_off[ci][i]) return false;
    }
    return true;
  }

  // SAO parameters of CTU (cx, cy): those of its first 32x32 record block
  const CtuInfo& ctu_sao(int cx, int cy) const {
    const int k = c.ctu64 ? 1 : 0;
    return ctu[(cy << k) * wctb + (cx << k)];
  }
  void write_sao(int rx, int ry) {
    const CtuInfo& t = ctu_sao(rx, ry);
    if (rx > 0 && same_sao(t, ctu_sao(rx - 1, ry))) {
      e.encode(1, ctx[CTX_SAO_MERGE]);
      return;
    }
    if (rx > 0) e.encode(0, ctx[CTX_SAO_MERGE]);
    if (ry > 0 && same_sao(t, ctu_sao(rx, ry - 1))) {
      e.encode(1, ctx[CTX_SAO_MERGE]);
      return;
    }
    if (ry > 0) e.encode(0, ctx[CTX_SAO_MERGE]);
    const int cmax = (1 << (std::min(c.bit_depth, 10) - 5)) - 1;
    for (int ci = 0; ci < 3; ++ci) {
      const int type = t.sao_type[ci ? 1 : 0];
      if (ci < 2) {  // sao_type_idx_luma / _chroma: TR cMax 2, first bin context coded
        if (type == 0) {
          e.encode(0, ctx[CTX_SAO_TYPE]);
        } else {
          e.encode(1, ctx[CTX_SAO_TYPE]);
          e.bypass(type == 2);
        }
      }
      if (type == 0) continue;
      for (int i = 0; i < 4; ++i) {
        int a = std::abs(static_cast<int>(t.sao_off[ci][i]));
        if (a > cmax) throw std::runtime_error("SAO offset out of range");
        for (int k = 0; k < a; ++k) e.bypass(1);  // TR, bypass
        if (a < cmax) e.bypass(0);
      }
      if (type == 1) {
        for (int i = 0; i < 4; ++i)
          if (t.sao_off[ci][i] != 0) e.bypass(t.sao_off[ci][i] < 0);
        e.bypass_bits(t.sao_band[ci] & 31, 5);
      } else {
        if (t.sao_off[ci][0] < 0 || t.sao_off[ci][1] < 0 || t.sao_off[ci][2] > 0 || t.sao_off[ci][3] > 0)
          throw std::runtime_error("edge-offset signs violate 7.4.9.3.2");
        if (ci < 2) e.bypass_bits(t.sao_class[ci] & 3, 2);
      }
    }
  }

  // ---------------------------------------------------------------- residual coding (7.3.8.11)
  void write_last(int v, int log2, int cidx, int ctx_base) {
    static const int grp[32] = {0, 1, 2, 3, 4, 4, 5, 5, 6, 6, 6, 6, 7, 7, 7, 7,
                                8, 8, 8, 8, 8, 8, 8, 8, 9, 9, 9, 9, 9, 9, 9, 9};
    const int prefix = grp[v];
    const int cmax = (log2 << 1) - 1;
    int off, shift;
    if (cidx == 0) {
      off = 3 * (log2 - 2) + ((log2 - 1) >> 2);
      shift = (log2 + 1) >> 2;
    } else {
      off = 15;
      shift = log2 - 2;
    }
    for (int i = 0; i < prefix; ++i) e.encode(1, ctx[ctx_base + off + (i >> shift)]);
    if (prefix < cmax) e.encode(0, ctx[ctx_base + off + (prefix >> shift)]);
  }
  void write_last_suffix(int v) {
    static const int grp[32] = {0, 1, 2, 3, 4, 4, 5, 5, 6, 6, 6, 6, 7, 7, 7, 7,
                                8, 8, 8, 8, 8, 8, 8, 8, 9, 9, 9, 9, 9, 9, 9, 9};
    static const int mn[10] = {0, 1, 2, 3, 4, 6, 8, 12, 16, 24};
    const int prefix = grp[v];
    if (prefix > 3) e.bypass_bits(v - mn[prefix], (prefix >> 1) - 1);
  }

  void write_remaining(int v, int rice) {
    if (v < (3 << rice)) {
      const int len = v >> rice;
      e.bypass_bits((1u << (len + 1)) - 2, len + 1);
      e.bypass_bits(v & ((1 << rice) - 1), rice);
    } else {
      int len = rice;
      int s = v - (3 << rice);
      while (s >= (1 << len)) {
        s -= 1 << len;
        ++len;
      }
      const int ones = 3 + len + 1 - rice;
      // ones-1 ones and a zero, then len bits (may exceed 16 in total: split)
      for (int i = 0; i < ones - 1; ++i) e.bypass(1);
      e.bypass(0);
      e.bypass_bits(static_cast<uint32_t>(s), len);
    }
  }

  // scan orders (6.5.3-6.5.5) as tables: [scan_idx][log2 of the grid side 0..3][position] -> x | y << 4
  struct ScanTables {
    uint8_t t[3][4][64];
    ScanTables() {
      for (int s = 0; s < 3; ++s)
        for (int l = 0; l < 4; ++l)
          for (int i = 0; i < (1 << (2 * l)); ++i) {
            const int p = scan_pos(s, l, i);
            t[s][l][i] = static_cast<uint8_t>((p & 255) | ((p >> 8) << 4));
          }
    }
  };
  static const ScanTables& scans() {
    static const ScanTables tables;
    return tables;
  }

  // 7.3.8.11 residual_coding.  The coefficient groups are visited through the scan
  // tables; each group's 16 levels are gathered once (4 row loads) and an all-zero
  // group costs 4 loads, so sparse 32x32 blocks are cheap.
  // significance contexts (9.3.4.2.5) per (TU size, component, scan, neighbouring coded
  // sub-block flags, first sub-block or not, position in the sub-block's scan): a table
  // lookup per coefficient instead of the derivation
  struct SigTables {
    uint8_t t[4][2][3][4][2][16];
    SigTables() {
      for (int l = 0; l < 4; ++l)
        for (int c = 0; c < 2; ++c)
          for (int sc = 0; sc < 3; ++sc)
            for (int pc = 0; pc < 4; ++pc)
              for (int g0 = 0; g0 < 2; ++g0)
                for (int p = 0; p < 16; ++p) {
                  const int q = scans().t[sc][2][p];
                  // any sub-block other than the first (a 4x4 TU has only the first: the g0 = 0
                  // entries of l = 0 are never read, keep them in range)
                  const int xs = (g0 || l == 0) ? 0 : 1, ys = 0;
                  t[l][c][sc][pc][g0][p] = static_cast<uint8_t>(
                      sig_ctx(xs * 4 + (q & 15), ys * 4 + (q >> 4), l + 2, c, sc, pc, xs, ys));
                }
    }
  };
  static const SigTables& sig_tables() {
    static const SigTables tables;
    return tables;
  }

  // gmask: bit (ys * nsb + xs) set for every non-zero 4x4 sub-block of the TU (from the
  // CTB's sub-block map), so all-zero sub-blocks are never loaded
  // levels of the 4x4 block at plane position (px, py) of component cidx (in the current CTB)
  void load4x4(int cidx, int px, int py, int16_t (&rows)[4][4]) const {
    if (pk) {
      const int side = cidx ? 4 : 8, m = cidx ? 15 : 31;
      const int bit = ((py & m) >> 2) * side + ((px & m) >> 2);
      uint32_t rank;
      if (cidx == 0) {
        rank = static_cast<uint32_t>(__builtin_popcountll(nz_luma & ((1ull << bit) - 1ull)));
      } else {
        rank = static_cast<uint32_t>(__builtin_popcountll(nz_luma));
        if (cidx == 2) rank += static_cast<uint32_t>(__builtin_popcount(nz_chroma[0]));
        rank += static_cast<uint32_t>(__builtin_popcount(nz_chroma[cidx - 1] & ((1u << bit) - 1u)));
      }
      const size_t at = static_cast<size_t>(ctb_base) + rank;
      if (at >= pk->nblocks) throw std::runtime_error("HEVC packed levels: block index out of range");
      std::memcpy(rows, pk->levels + at * 16, 32);
      return;
    }
    const int stride = cidx ? W / 2 : W;
    const int16_t* b = coef[cidx] + static_cast<size_t>(py) * stride + px;
    for (int r = 0; r < 4; ++r) std::memcpy(rows[r], b + static_cast<size_t>(r) * stride, sizeof(rows[r]));
  }

  // residual_coding of the (1 << log2)^2 block of component cidx at plane position (bx0, by0)
  void write_residual(int cidx, int bx0, int by0, int log2, int scan_idx, uint64_t gmask) {
    const int log2sb = log2 - 2, nsb = 1 << log2sb, nsbsq = nsb * nsb;
    const uint8_t* sbs = scans().t[scan_idx][log2sb];
    const uint8_t* ps = scans().t[scan_idx][2];
    auto gbit = [&](int i) { return (gmask >> ((sbs[i] >> 4) * nsb + (sbs[i] & 15))) & 1u; };
    auto group_rows = [&](int i, int16_t (&rows)[4][4]) {
      const int xs = sbs[i] & 15, ys = sbs[i] >> 4;
      load4x4(cidx, bx0 + xs * 4, by0 + ys * 4, rows);
    };
    auto any_row = [](const int16_t (&rows)[4][4]) {
      uint64_t a = 0;
      for (int r = 0; r < 4; ++r) {
        uint64_t w;
        std::memcpy(&w, rows[r], 8);
        a |= w;
      }
      return a != 0;
    };
    // last significant group / position
    int last_i = -1, last_p = -1;
    int16_t lv[16];
    for (int i = nsbsq - 1; i >= 0 && last_i < 0; --i) {
      if (!gbit(i)) continue;
      int16_t rows[4][4];
      group_rows(i, rows);
      if (!any_row(rows)) continue;
      for (int p = 0; p < 16; ++p) lv[p] = rows[ps[p] >> 4][ps[p] & 15];
      for (int p = 15; p >= 0; --p)
        if (lv[p] != 0) {
          last_i = i;
          last_p = p;
          break;
        }
    }
    if (last_i < 0) throw std::runtime_error("residual_coding of an all-zero block");
    int lx = (sbs[last_i] & 15) * 4 + (ps[last_p] & 15), ly = (sbs[last_i] >> 4) * 4 + (ps[last_p] >> 4);
    if (scan_idx == 2) std::swap(lx, ly);
    write_last(lx, log2, cidx, CTX_LAST_X);
    write_last(ly, log2, cidx, CTX_LAST_Y);
    write_last_suffix(lx);
    write_last_suffix(ly);

    uint8_t csbf[8][8] = {};
    int c1 = 1;
    bool first_sb = true;
    for (int i = last_i; i >= 0; --i) {
      const int xs = sbs[i] & 15, ys = sbs[i] >> 4;
      int16_t lvl[16];
      bool nonzero;
      if (i == last_i) {
        std::memcpy(lvl, lv, sizeof(lvl));
        nonzero = true;
      } else if (!gbit(i)) {
        nonzero = false;
      } else {
        int16_t rows[4][4];
        group_rows(i, rows);
        nonzero = any_row(rows);
        if (nonzero)
          for (int p = 0; p < 16; ++p) lvl[p] = rows[ps[p] >> 4][ps[p] & 15];
      }
      bool infer_dc = false;
      if (i < last_i && i > 0) {
        int cs = 0;
        if (xs < nsb - 1) cs += csbf[xs + 1][ys];
        if (ys < nsb - 1) cs += csbf[xs][ys + 1];
        e.encode(nonzero, ctx[CTX_CSBF + std::min(cs, 1) + (cidx ? 2 : 0)]);
        csbf[xs][ys] = nonzero;
        infer_dc = true;
      } else {
        csbf[xs][ys] = 1;
        if (!nonzero) std::memset(lvl, 0, sizeof(lvl));  // DC group of a block: coded even if empty
      }
      if (!csbf[xs][ys]) continue;
      int prev_csbf = 0;
      if (xs < nsb - 1) prev_csbf += csbf[xs + 1][ys];
      if (ys < nsb - 1) prev_csbf += csbf[xs][ys + 1] << 1;
      // significance
      int vals[16], nsig = 0;
      if (i == last_i) vals[nsig++] = lvl[last_p];
      const uint8_t* sct = sig_tables().t[log2 - 2][cidx ? 1 : 0][scan_idx][prev_csbf][xs + ys == 0 ? 1 : 0];
      CtxState* sctx = ctx + CTX_SIG;
      for (int p = (i == last_i ? last_p - 1 : 15); p >= 0; --p) {
        const int v = lvl[p];
        if (p > 0 || !infer_dc) {
          e.encode(v != 0, sctx[sct[p]]);
          if (v != 0) infer_dc = false;
        }
        if (v != 0) vals[nsig++] = v;
      }
      // greater1 / greater2
      int ctx_set = (i == 0 || cidx > 0) ? 0 : 2;
      if (!first_sb && c1 == 0) ++ctx_set;
      first_sb = false;
      c1 = 1;
      int g1_first = -1;
      int g1[16] = {};
      for (int k = 0; k < nsig && k < 8; ++k) {
        const int a = std::abs(vals[k]);
        g1[k] = a > 1;
        e.encode(g1[k], ctx[CTX_GT1 + (cidx ? 16 : 0) + ctx_set * 4 + c1]);
        if (g1[k]) {
          c1 = 0;
          if (g1_first < 0) g1_first = k;
        } else if (c1 > 0 && c1 < 3) {
          ++c1;
        }
      }
      int g2 = 0;
      if (g1_first >= 0) {
        g2 = std::abs(vals[g1_first]) > 2;
        e.encode(g2, ctx[CTX_GT2 + (cidx ? 4 : 0) + ctx_set]);
      }
      uint32_t signs = 0;
      for (int k = 0; k < nsig; ++k) signs = (signs << 1) | (vals[k] < 0);
      // sign data hiding: vals[nsig - 1] is the first significant coefficient in scan order
      int first_p = -1, last_p_g = -1;
      for (int p = 0; p < 16; ++p)
        if (lvl[p] != 0) {
          if (first_p < 0) first_p = p;
          last_p_g = p;
        }
      if (c.sdh && first_p >= 0 && last_p_g - first_p > 3) {
        int sum = 0;
        for (int k = 0; k < nsig; ++k) sum += std::abs(vals[k]);
        if ((sum & 1) != (vals[nsig - 1] < 0 ? 1 : 0))
          throw std::runtime_error("HEVC: sign data hiding parity does not match the hidden sign");
        e.bypass_bits(signs >> 1, nsig - 1);
      } else {
        e.bypass_bits(signs, nsig);
      }
      int rice = 0;
      for (int k = 0; k < nsig; ++k) {
        const int a = std::abs(vals[k]);
        const int base = 1 + (k < 8 ? g1[k] : 0) + (k == g1_first ? g2 : 0);
        const int thr = k < 8 ? (k == g1_first ? 3 : 2) : 1;
        if (base == thr) {
          write_remaining(a - base, rice);
          if (a > 3 * (1 << rice)) rice = std::min(rice + 1, 4);
        }
      }
    }
  }

  static int sig_ctx(int xc, int yc, int log2, int cidx, int scan_idx, int prev_csbf, int xs, int ys) {
    static const uint8_t map4[16] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8};
    int s;
    if (log2 == 2) {
      s = map4[(yc << 2) + xc];
    } else if (xc + yc == 0) {
      s = 0;
    } else {
      const int xp = xc & 3, yp = yc & 3;
      if (prev_csbf == 0) s = (xp + yp == 0) ? 2 : (xp + yp < 3) ? 1 : 0;
      else if (prev_csbf == 1) s = (yp == 0) ? 2 : (yp == 1) ? 1 : 0;
      else if (prev_csbf == 2) s = (xp == 0) ? 2 : (xp == 1) ? 1 : 0;
      else s = 2;
      if (cidx == 0) {
        if (xs + ys > 0) s += 3;
        s += log2 == 3 ? (scan_idx == 0 ? 9 : 15) : 21;
      } else {
        s += log2 == 3 ? 9 : 12;
      }
    }
    return cidx == 0 ? s : 27 + s;
  }

  static int mdcs(int mode) { return (mode >= 6 && mode <= 14) ? 2 : ((mode >= 22 && mode <= 30) ? 1 : 0); }

  // non-zero 4x4 sub-blocks of the current CTB: luma bit (by * 8 + bx), chroma (by * 4 + bx)
  uint64_t nz_luma = 0;
  uint32_t nz_chroma[2] = {0, 0};
  void scan_ctb_nz(int x0, int y0) {
    if (pk) {
      const size_t ci = static_cast<size_t>(y0 / kCtb) * wctb + x0 / kCtb;
      nz_luma = pk->nzmap[2 * ci];
      nz_chroma[0] = static_cast<uint32_t>(pk->nzmap[2 * ci + 1] & 0xFFFFu);
      nz_chroma[1] = static_cast<uint32_t>((pk->nzmap[2 * ci + 1] >> 16) & 0xFFFFu);
      ctb_base = pk->ctb_off[ci];
      return;
    }
    nz_luma = 0;
    for (int by = 0; by < 8; ++by)
      for (int bx = 0; bx < 8; ++bx) {
        const int16_t* p = coef[0] + static_cast<size_t>(y0 + by * 4) * W + x0 + bx * 4;
        uint64_t a = 0;
        for (int r = 0; r < 4; ++r) {
          uint64_t w;
          std::memcpy(&w, p + static_cast<size_t>(r) * W, 8);
          a |= w;
        }
        nz_luma |= static_cast<uint64_t>(a != 0) << (by * 8 + bx);
      }
    const int cw = W / 2;
    for (int c = 0; c < 2; ++c) {
      nz_chroma[c] = 0;
      for (int by = 0; by < 4; ++by)
        for (int bx = 0; bx < 4; ++bx) {
          const int16_t* p = coef[1 + c] + static_cast<size_t>(y0 / 2 + by * 4) * cw + x0 / 2 + bx * 4;
          uint64_t a = 0;
          for (int r = 0; r < 4; ++r) {
            uint64_t w;
            std::memcpy(&w, p + static_cast<size_t>(r) * cw, 8);
            a |= w;
          }
          nz_chroma[c] |= static_cast<uint32_t>(a != 0) << (by * 4 + bx);
        }
    }
  }
  // sub-block mask of an n x n block at plane position (x, y) inside the current CTB, in
  // the block's own raster order (bit ys * (n / 4) + xs)
  uint64_t block_mask(int cidx, int x, int y, int n) const {
    const int side = cidx ? 4 : 8, m = cidx ? 15 : 31;
    const uint64_t src = cidx ? nz_chroma[cidx - 1] : nz_luma;
    const int bx0 = (x & m) >> 2, by0 = (y & m) >> 2, nb = n >> 2;
    uint64_t out = 0;
    for (int r = 0; r < nb; ++r)
      out |= ((src >> ((by0 + r) * side + bx0)) & ((1ull << nb) - 1ull)) << (r * nb);
    return out;
  }
  bool any_nonzero(int cidx, int x, int y, int n) const { return block_mask(cidx, x, y, n) != 0; }

  // ---------------------------------------------------------------- inter prediction helpers
  // A PU's motion is its direction (bit 0 list 0, bit 1 list 1) and a refIdx + vector per used
  // list; RefPicListX holds num_ref[X] pictures (POC list_poc(X, i)).
  bool inter_avail(int x, int y) const { return avail(x, y) && pred[g(x, y)] == CU_INTER; }
  const Motion& mot_at(int x, int y) const { return mot[g(x, y)]; }
  int ref_poc(int l) const { return l == 0 ? (fp.ref_poc[0] >= 0 ? fp.ref_poc[0] : fp.poc - 1) : fp.ref_poc[1]; }
  int nref(int l) const { return std::max(1, fp.num_ref[l]); }
  int list_poc(int l, int i) const { return i == 0 ? ref_poc(l) : fp.list_poc[l][i]; }

  static Mv scale_mv(Mv v, int td0, int tb0) {  // 8.5.3.2.8 (8-209 .. 8-213)
    const int td = std::clamp(td0, -128, 127), tb = std::clamp(tb0, -128, 127);
    const int tx = (16384 + (std::abs(td) >> 1)) / td;
    const int dsf = std::clamp((tb * tx + 32) >> 6, -4096, 4095);
    auto sc = [dsf](int m) {
      const int p = dsf * m;
      return std::clamp((p < 0 ? -1 : 1) * ((std::abs(p) + 127) >> 8), -32768, 32767);
    };
    return Mv{sc(v.x), sc(v.y)};
  }

  // 8.5.3.2.8 / 8.5.3.2.9 temporal vector of list X (target refIdx ri) for the PU (x, y, n x n)
  bool col_at(int xc, int yc, int X, int ri, Mv* out) const {
    if (!fp.col.cu || xc >= W || yc >= H) return false;
    const int ci = (yc >> kCtbLog2) * wctb + (xc >> kCtbLog2);
    const CuInfo& cc = fp.col.cu[static_cast<size_t>(ci) * kCusPerCtb + zorder8((xc & (kCtb - 1)) >> 3, (yc & (kCtb - 1)) >> 3)];
    if (cc.pred != CU_INTER) return false;
    const int dir = cu_dir(cc);
    int list;
    if (!(dir & 1)) list = 1;
    else if (dir == DIR_L0) list = 0;
    else list = no_backward ? X : (col_l1 ? 0 : 1);  // N = collocated_from_l0_flag
    Mv v = list == 0 ? Mv{cc.mv[0], cc.mv[1]} : Mv{cc.mv1[0], cc.mv1[1]};
    const int cr = cc.pad[list];
    if (cr >= kMaxRefs) throw std::runtime_error("HEVC: collocated refIdx out of range");
    const int col_diff = fp.col.poc - (cr == 0 ? fp.col.ref_poc[list] : fp.col.list_poc[list][cr]);
    const int cur_diff = fp.poc - list_poc(X, ri);
    if (col_diff != cur_diff && col_diff != 0) v = scale_mv(v, col_diff, cur_diff);
    *out = v;
    return true;
  }
  bool temporal(int x, int y, int n, int X, int ri, Mv* out) const {
    if (!tmvp) return false;
    const int xbr = x + n, ybr = y + n;
    if ((y >> L) == (ybr >> L) && ybr < H && xbr < W && col_at((xbr >> 4) << 4, (ybr >> 4) << 4, X, ri, out))
      return true;
    return col_at(((x + (n >> 1)) >> 4) << 4, ((y + (n >> 1)) >> 4) << 4, X, ri, out);
  }

  // 8.5.3.2.2-8.5.3.2.5 merge candidates of a 2Nx2N PU (MaxNumMergeCand entries)
  int merge_list(int x, int y, int n, Motion* out) const {
    Motion cand[8];
    int k = 0;
    const int xa1 = x - 1, ya1 = y + n - 1, xb1 = x + n - 1, yb1 = y - 1;
    const bool a1 = inter_avail(xa1, ya1), av_b1 = inter_avail(xb1, yb1);
    const Motion ma1 = a1 ? mot_at(xa1, ya1) : Motion{}, mb1 = av_b1 ? mot_at(xb1, yb1) : Motion{};
    const bool b1 = av_b1 && !(a1 && ma1 == mb1);
    bool b0 = inter_avail(x + n, y - 1), a0 = inter_avail(x - 1, y + n), b2 = inter_avail(x - 1, y - 1);
    const Motion mb0 = b0 ? mot_at(x + n, y - 1) : Motion{}, ma0 = a0 ? mot_at(x - 1, y + n) : Motion{};
    const Motion mb2 = b2 ? mot_at(x - 1, y - 1) : Motion{};
    if (b0 && av_b1 && mb1 == mb0) b0 = false;
    if (a0 && a1 && ma1 == ma0) a0 = false;
    if (b2 && ((a1 && ma1 == mb2) || (av_b1 && mb1 == mb2))) b2 = false;
    if (a0 + a1 + b0 + b1 == 4) b2 = false;
    if (a1) cand[k++] = ma1;
    if (b1) cand[k++] = mb1;
    if (b0) cand[k++] = mb0;
    if (a0) cand[k++] = ma0;
    if (b2) cand[k++] = mb2;
    if (k < c.max_merge && tmvp) {
      Motion t{};
      if (temporal(x, y, n, 0, 0, &t.m[0])) t.dir |= DIR_L0;  // refIdx 0 (8.5.3.2.8 merge: refIdxLXCol 0)
      if (bslice && temporal(x, y, n, 1, 0, &t.m[1])) t.dir |= DIR_L1;
      if (t.dir) cand[k++] = t;
    }
    const int orig = k;
    if (bslice && orig > 1 && orig < c.max_merge) {  // combined bi-predictive candidates
      static const int l0i[12] = {0, 1, 0, 2, 1, 2, 0, 3, 1, 3, 2, 3};
      static const int l1i[12] = {1, 0, 2, 0, 2, 1, 3, 0, 3, 1, 3, 2};
      for (int comb = 0; comb < orig * (orig - 1) && k < c.max_merge; ++comb) {
        const Motion &c0 = cand[l0i[comb]], &c1 = cand[l1i[comb]];
        if ((c0.dir & DIR_L0) && (c1.dir & DIR_L1) &&
            (list_poc(0, c0.r[0]) != list_poc(1, c1.r[1]) || !(c0.m[0] == c1.m[1])))
          cand[k++] = Motion{DIR_BI, {c0.r[0], c1.r[1]}, {c0.m[0], c1.m[1]}};
      }
    }
    // zero candidates (8.5.3.2.5): refIdx 0, 1, .. up to the active list size, then 0
    const int nzr = bslice ? std::min(nref(0), nref(1)) : nref(0);
    for (int zi = 0; k < c.max_merge; ++zi) {
      const int8_t r = static_cast<int8_t>(zi < nzr ? zi : 0);
      cand[k++] = Motion{static_cast<uint8_t>(bslice ? DIR_BI : DIR_L0), {r, r}, {{0, 0}, {0, 0}}};
    }
    const int nm = std::min(k, c.max_merge);
    std::copy(cand, cand + nm, out);
    return nm;
  }

  // 8.5.3.2.6-8.5.3.2.7 AMVP candidates of list X, refIdx ri
  void amvp_list(int x, int y, int n, int X, int ri, Mv* out) const {
    const int Y = 1 - X;
    const int tgt = list_poc(X, ri);
    auto same = [&](int xn, int yn, Mv* v) {  // a neighbour vector pointing at the target picture
      const Motion& m = mot_at(xn, yn);
      if ((m.dir >> X) & 1 && list_poc(X, m.r[X]) == tgt) {
        *v = m.m[X];
        return true;
      }
      if ((m.dir >> Y) & 1 && list_poc(Y, m.r[Y]) == tgt) {
        *v = m.m[Y];
        return true;
      }
      return false;
    };
    auto scaled = [&](int xn, int yn, Mv* v) {  // any vector, scaled by the POC distances
      const Motion& m = mot_at(xn, yn);
      for (int L : {X, Y}) {
        if (!((m.dir >> L) & 1)) continue;
        const int td = fp.poc - list_poc(L, m.r[L]), tb = fp.poc - tgt;
        *v = (td != tb && td != 0) ? scale_mv(m.m[L], td, tb) : m.m[L];
        return true;
      }
      return false;
    };
    const int xa[2] = {x - 1, x - 1}, ya[2] = {y + n, y + n - 1};
    const bool ava[2] = {inter_avail(xa[0], ya[0]), inter_avail(xa[1], ya[1])};
    const bool is_scaled = ava[0] || ava[1];
    bool fa = false, fb = false;
    Mv ma{0, 0}, mb{0, 0};
    for (int k = 0; k < 2 && !fa; ++k)
      if (ava[k]) fa = same(xa[k], ya[k], &ma);
    for (int k = 0; k < 2 && !fa; ++k)
      if (ava[k]) fa = scaled(xa[k], ya[k], &ma);
    const int xb[3] = {x + n, x + n - 1, x - 1}, yb = y - 1;
    const bool avb[3] = {inter_avail(xb[0], yb), inter_avail(xb[1], yb), inter_avail(xb[2], yb)};
    for (int k = 0; k < 3 && !fb; ++k)
      if (avb[k]) fb = same(xb[k], yb, &mb);
    if (!is_scaled && fb) {
      ma = mb;
      fa = true;
    }
    if (!is_scaled) {
      fb = false;
      for (int k = 0; k < 3 && !fb; ++k)
        if (avb[k]) fb = scaled(xb[k], yb, &mb);
    }
    int k = 0;
    if (fa) out[k++] = ma;
    if (fb && !(fa && ma == mb)) out[k++] = mb;
    if (k < 2) {
      Mv t;
      if (temporal(x, y, n, X, ri, &t)) out[k++] = t;
    }
    while (k < 2) out[k++] = Mv{0, 0};
  }

  // ---------------------------------------------------------------- coding unit (7.3.8.5)
  void mark(int x, int y, int n, int d, int sk, int pm, int md, const Motion& mv) {
    for (int yy = y; yy < y + n; yy += 8)
      for (int xx = x; xx < x + n; xx += 8) {
        const size_t k = g(xx, yy);
        depth[k] = static_cast<int8_t>(d);
        skip[k] = static_cast<int8_t>(sk);
        pred[k] = static_cast<int8_t>(pm);
        for (int q = 0; q < 4; ++q) mode4[g4(xx + (q & 1) * 4, yy + (q >> 1) * 4)] = static_cast<int8_t>(md);
        mot[k] = mv;
        coded[k] = 1;
      }
  }

  // inter_pred_idc (9.3.3.7, 2Nx2N PU of a CU at depth d): PRED_BI "1", PRED_L0 "00", PRED_L1 "01"
  void write_inter_pred_idc(int dir, int d) {
    e.encode(dir == DIR_BI, ctx[CTX_INTER_PRED + d]);
    if (dir != DIR_BI) e.encode(dir == DIR_L1, ctx[CTX_INTER_PRED + 4]);
  }

  // a CU, then the QpY of its granules (8.6.1: the quantization group's prediction until a
  // cu_qp_delta has been coded, the coded QP from then on)
  void write_cu(int x, int y, int log2, int d) {
    write_cu_body(x, y, log2, d);
    const int q = qp_coded ? qp_ctb : qp_pred_cur, n = 1 << log2;
    for (int yy = y; yy < y + n; yy += 8)
      for (int xx = x; xx < x + n; xx += 8) qpy[g(xx, yy)] = static_cast<int8_t>(q);
  }
  void write_cu_body(int x, int y, int log2, int d) {
    const int n = 1 << log2;
    const CuInfo& ci = cu_at(x, y);
    const bool cb_y = any_nonzero(0, x, y, n);
    const bool cb_cb = any_nonzero(1, x / 2, y / 2, n / 2), cb_cr = any_nonzero(2, x / 2, y / 2, n / 2);
    const bool intra = ci.pred == CU_INTRA || !inter_slice;
    Motion mv{static_cast<uint8_t>(cu_dir(ci)), {static_cast<int8_t>(ci.pad[0]), static_cast<int8_t>(ci.pad[1])},
              {{ci.mv[0], ci.mv[1]}, {ci.mv1[0], ci.mv1[1]}}};
    if (!intra && (mv.dir & ~3 || (!bslice && mv.dir != DIR_L0)))
      throw std::runtime_error("HEVC: inter CU direction not allowed in this slice");
    if (!intra && (((mv.dir & DIR_L0) && (mv.r[0] < 0 || mv.r[0] >= nref(0))) ||
                   ((mv.dir & DIR_L1) && (mv.r[1] < 0 || mv.r[1] >= nref(1)))))
      throw std::runtime_error("HEVC: inter CU refIdx outside the active list");
    for (int X = 0; X < 2; ++X)
      if (!((mv.dir >> X) & 1)) {
        mv.m[X] = Mv{0, 0};
        mv.r[X] = 0;
      }
    if (inter_slice) {
      int skip_ctx = (avail(x - 1, y) && skip[g(x - 1, y)]) + (avail(x, y - 1) && skip[g(x, y - 1)]);
      int midx = -1;
      Motion ml[5];
      if (!intra) {
        const int nm = merge_list(x, y, n, ml);
        for (int k = 0; k < nm; ++k)
          if (ml[k] == mv) {
            midx = k;
            break;
          }
      }
      const bool is_skip = !intra && midx >= 0 && !cb_y && !cb_cb && !cb_cr;
      e.encode(is_skip, ctx[CTX_CU_SKIP + skip_ctx]);
      if (is_skip) {
        write_merge_idx(midx);
        mark(x, y, n, d, 1, CU_INTER, 1, mv);
        ++st.skip_cus;
        return;
      }
      e.encode(intra, ctx[CTX_PRED_MODE]);
      if (!intra) {
        e.encode(1, ctx[CTX_PART_MODE]);  // PART_2Nx2N
        const bool merge = midx >= 0;
        e.encode(merge, ctx[CTX_MERGE_FLAG]);
        if (merge) {
          write_merge_idx(midx);
          ++st.merge_cus;
        } else {
          if (bslice) write_inter_pred_idc(mv.dir, d);
          for (int X = 0; X < 2; ++X) {
            if (!((mv.dir >> X) & 1)) continue;
            if (nref(X) > 1) write_ref_idx(mv.r[X], nref(X) - 1);
            Mv ap[2];
            amvp_list(x, y, n, X, mv.r[X], ap);
            const Mv& v = mv.m[X];
            auto cost = [&](const Mv& p) { return std::abs(v.x - p.x) + std::abs(v.y - p.y); };
            const int idx = cost(ap[1]) < cost(ap[0]) ? 1 : 0;
            write_mvd_pair(v.x - ap[idx].x, v.y - ap[idx].y);  // (mvd_l1_zero_flag 0)
            e.encode(idx, ctx[CTX_MVP_IDX]);
          }
        }
        const bool root = cb_y || cb_cb || cb_cr;
        if (!merge) e.encode(root, ctx[CTX_RQT_ROOT_CBF]);
        mark(x, y, n, d, 0, CU_INTER, 1, mv);
        ++st.inter_cus;
        if (root) {
          if (ci.flags & 16) write_tu_inter_split(x, y, log2, cb_cb, cb_cr);
          else write_tu(x, y, log2, false, 0, cb_y, cb_cb, cb_cr);
        }
        return;
      }
    }
    // intra CU: PART_2Nx2N, or PART_NxN at the minimum CB size (four 4x4 PUs, CuInfo flags
    // bit 3, PU modes in the bytes of the unused motion vector)
    const bool nxn = log2 == kMinCbLog2 && (ci.flags & 8);
    if (log2 == kMinCbLog2) e.encode(nxn ? 0 : 1, ctx[CTX_PART_MODE]);
    const int npu = nxn ? 4 : 1, h = nxn ? n / 2 : n;
    int m[4], mpm[4], rem[4];
    for (int k = 0; k < npu; ++k) {
      m[k] = nxn ? reinterpret_cast<const uint8_t*>(ci.mv)[k] : ci.mode;
      if (m[k] > 34) throw std::runtime_error("intra mode out of range");
      const int xk = x + (k & 1) * h, yk = y + (k >> 1) * h;
      // 8.4.2 most probable modes; an NxN PU's left / above neighbour may be an earlier PU
      auto cand_of = [&](int xn, int yn, bool above) {
        if (xn >= x && yn >= y) return m[(xn - x >= h) + 2 * (yn - y >= h)];
        if (!avail(xn, yn) || pred[g(xn, yn)] != CU_INTRA) return 1;
        if (above && (yn >> L) != (yk >> L)) return 1;
        return static_cast<int>(mode4[g4(xn, yn)]);
      };
      const int ca = cand_of(xk - 1, yk, false), cb = cand_of(xk, yk - 1, true);
      int cand[3];
      if (ca == cb) {
        if (ca < 2) {
          cand[0] = 0;
          cand[1] = 1;
          cand[2] = 26;
        } else {
          cand[0] = ca;
          cand[1] = 2 + ((ca + 29) % 32);
          cand[2] = 2 + ((ca - 2 + 1) % 32);
        }
      } else {
        cand[0] = ca;
        cand[1] = cb;
        cand[2] = (ca != 0 && cb != 0) ? 0 : ((ca != 1 && cb != 1) ? 1 : 26);
      }
      mpm[k] = -1;
      for (int j = 0; j < 3; ++j)
        if (cand[j] == m[k]) mpm[k] = j;
      std::sort(cand, cand + 3);
      rem[k] = m[k];
      for (int j = 2; j >= 0; --j)
        if (rem[k] > cand[j]) --rem[k];
    }
    for (int k = 0; k < npu; ++k) e.encode(mpm[k] >= 0, ctx[CTX_PREV_INTRA]);
    for (int k = 0; k < npu; ++k) {
      if (mpm[k] >= 0) {
        e.bypass(mpm[k] > 0);
        if (mpm[k] > 0) e.bypass(mpm[k] > 1);
      } else {
        e.bypass_bits(rem[k], 5);
      }
    }
    e.encode(0, ctx[CTX_CHROMA_MODE]);  // intra_chroma_pred_mode = 4 (DM: the mode of PU 0)
    mark(x, y, n, d, 0, CU_INTRA, m[0], Motion{});
    if (nxn)
      for (int k = 1; k < 4; ++k) mode4[g4(x + (k & 1) * h, y + (k >> 1) * h)] = static_cast<int8_t>(m[k]);
    ++st.intra_cus;
    if (nxn) write_tu_nxn(x, y, m, cb_cb, cb_cr);
    else write_tu(x, y, log2, true, m[0], cb_y, cb_cb, cb_cr);
  }

  // transform_tree of an intra PART_NxN CU (7.3.8.8 / 7.3.8.10): chroma cbfs at depth 0,
  // split_transform_flag inferred (IntraSplitFlag), four 4x4 luma TUs with cbf_luma at
  // depth 1; cbfChroma of every 4x4 TU is the parent's, and the 4x4 chroma blocks follow
  // the last luma TU (blkIdx 3)
  void write_tu_nxn(int x, int y, const int* m, bool cb_cb, bool cb_cr) {
    e.encode(cb_cb, ctx[CTX_CBF_CHROMA + 0]);
    e.encode(cb_cr, ctx[CTX_CBF_CHROMA + 0]);
    for (int k = 0; k < 4; ++k) {
      const int xk = x + (k & 1) * 4, yk = y + (k >> 1) * 4;
      const bool cy = any_nonzero(0, xk, yk, 4);
      e.encode(cy, ctx[CTX_CBF_LUMA + 0]);
      if (c.cu_qp_delta && !qp_coded && (cy || cb_cb || cb_cr)) write_qp_delta();
      if (cy) write_residual(0, xk, yk, 2, mdcs(m[k]), 1);
    }
    if (cb_cb) write_residual(1, x / 2, y / 2, 2, mdcs(m[0]), 1);
    if (cb_cr) write_residual(2, x / 2, y / 2, 2, mdcs(m[0]), 1);
  }

  // ref_idx_lX (9.3.3.1 TR, cMax = num_ref_idx_active - 1): two context-coded bins, then bypass
  void write_ref_idx(int r, int cmax) {
    for (int i = 0; i < cmax; ++i) {
      const int b = r > i;
      if (i < 2) e.encode(b, ctx[CTX_REF_IDX + i]);
      else e.bypass(b);
      if (!b) break;
    }
  }

  void write_merge_idx(int idx) {
    if (c.max_merge <= 1) return;
    e.encode(idx > 0, ctx[CTX_MERGE_IDX]);
    for (int k = 1; k < c.max_merge - 1 && idx >= k; ++k) e.bypass(idx > k);
  }

  void write_mvd_pair(int dx, int dy) {
    const int ax = std::abs(dx), ay = std::abs(dy);
    e.encode(ax > 0, ctx[CTX_MVD_G0]);
    e.encode(ay > 0, ctx[CTX_MVD_G0]);
    if (ax > 0) e.encode(ax > 1, ctx[CTX_MVD_G1]);
    if (ay > 0) e.encode(ay > 1, ctx[CTX_MVD_G1]);
    if (ax > 0) {
      if (ax > 1) write_eg1(ax - 2);
      e.bypass(dx < 0);
    }
    if (ay > 0) {
      if (ay > 1) write_eg1(ay - 2);
      e.bypass(dy < 0);
    }
  }
  void write_eg1(uint32_t v) { write_egk(v, 1); }

  // transform_tree at depth 0 with TU = CU (7.3.8.8 / 7.3.8.10)
  // inter CU whose residual quadtree splits once (CuInfo flags bit 4): split_transform_flag,
  // chroma cbfs at depth 0, then per quarter TU (z-order) its chroma cbfs under a set parent,
  // cbf_luma (always coded below depth 0) and the transform unit
  void write_tu_inter_split(int x, int y, int log2, bool cb_cb, bool cb_cr) {
    if (c.tu_inter_depth < 1 || log2 < 4) throw std::runtime_error("HEVC: inter TU split needs depth 1 and a 16x16+ CU");
    e.encode(1, ctx[CTX_SPLIT_TRANSFORM + 5 - log2]);
    e.encode(cb_cb, ctx[CTX_CBF_CHROMA + 0]);
    e.encode(cb_cr, ctx[CTX_CBF_CHROMA + 0]);
    const int h = 1 << (log2 - 1);
    for (int k = 0; k < 4; ++k) {
      const int xc = x + (k & 1) * h, yc = y + (k >> 1) * h;
      const bool ccb = cb_cb && any_nonzero(1, xc / 2, yc / 2, h / 2);
      const bool ccr = cb_cr && any_nonzero(2, xc / 2, yc / 2, h / 2);
      if (cb_cb) e.encode(ccb, ctx[CTX_CBF_CHROMA + 1]);
      if (cb_cr) e.encode(ccr, ctx[CTX_CBF_CHROMA + 1]);
      const bool cy = any_nonzero(0, xc, yc, h);
      e.encode(cy, ctx[CTX_CBF_LUMA + 0]);
      if (c.cu_qp_delta && !qp_coded && (cy || ccb || ccr)) write_qp_delta();
      if (cy) write_residual(0, xc, yc, log2 - 1, 0, block_mask(0, xc, yc, h));
      if (ccb) write_residual(1, xc / 2, yc / 2, log2 - 2, 0, block_mask(1, xc / 2, yc / 2, h / 2));
      if (ccr) write_residual(2, xc / 2, yc / 2, log2 - 2, 0, block_mask(2, xc / 2, yc / 2, h / 2));
    }
  }

  void write_tu(int x, int y, int log2, bool intra, int m, bool cb_y, bool cb_cb, bool cb_cr) {
    // split_transform_flag 0 where the inter depth allows a split (intra: depth 0 at 2Nx2N)
    if (!intra && c.tu_inter_depth > 0 && log2 > 2) e.encode(0, ctx[CTX_SPLIT_TRANSFORM + 5 - log2]);
    e.encode(cb_cb, ctx[CTX_CBF_CHROMA + 0]);
    e.encode(cb_cr, ctx[CTX_CBF_CHROMA + 0]);
    if (intra || cb_cb || cb_cr) e.encode(cb_y, ctx[CTX_CBF_LUMA + 1]);
    else if (!cb_y) throw std::runtime_error("inter TU: cbf_luma inferred 1 but the luma block is empty");
    if (c.cu_qp_delta && !qp_coded && (cb_y || cb_cb || cb_cr)) write_qp_delta();
    const int stride = W, cstride = W / 2;
    if (cb_y) {
      const int scan = (intra && log2 == 3) ? mdcs(m) : 0;
      write_residual(0, x, y, log2, scan, block_mask(0, x, y, 1 << log2));
    }
    const int scan_c = (intra && log2 - 1 == 2) ? mdcs(m) : 0;
    const int nc = 1 << (log2 - 1);
    if (cb_cb) write_residual(1, x / 2, y / 2, log2 - 1, scan_c, block_mask(1, x / 2, y / 2, nc));
    if (cb_cr) write_residual(2, x / 2, y / 2, log2 - 1, scan_c, block_mask(2, x / 2, y / 2, nc));
  }

  // cu_qp_delta_abs (9.3.3.10: TR prefix cMax 5, ctxInc 0 then 1; EG0 bypass suffix) and
  // the bypass sign, in the first TU of the CTB with a coded block
  void write_qp_delta() {
    const int d = qp_ctb - qp_pred_cur;
    const int qbd = 6 * (c.bit_depth - 8);
    if (d < -(26 + qbd / 2) || d > 25 + qbd / 2) throw std::runtime_error("HEVC: CuQpDeltaVal out of range");
    const int a = std::abs(d), pre = std::min(a, 5);
    for (int i = 0; i < pre; ++i) e.encode(1, ctx[CTX_CU_QP_DELTA + (i > 0)]);
    if (pre < 5) e.encode(0, ctx[CTX_CU_QP_DELTA + (pre > 0)]);
    else write_egk(static_cast<uint32_t>(a - 5), 0);
    if (a) e.bypass(d < 0);
    qp_coded = true;
  }
  void write_egk(uint32_t v, int k) {  // 9.3.3.3 k-th order Exp-Golomb, bypass
    while (v >= (1u << k)) {
      e.bypass(1);
      v -= 1u << k;
      ++k;
    }
    e.bypass(0);
    while (k--) e.bypass((v >> k) & 1);
  }

  // qPY_PRED of the quantization group at (xq, yq) (8.6.1): the average of the QpY left of and
  // above it when those lie in the same CTB, each replaced by qPY_PREV otherwise
  int qg_pred(int xq, int yq) const {
    auto same_ctb = [&](int x, int y) { return (x >> L) == (xq >> L) && (y >> L) == (yq >> L); };
    const int qa = (avail(xq - 1, yq) && same_ctb(xq - 1, yq)) ? qpy[g(xq - 1, yq)] : qp_prev;
    const int qb = (avail(xq, yq - 1) && same_ctb(xq, yq - 1)) ? qpy[g(xq, yq - 1)] : qp_prev;
    return (qa + qb + 1) >> 1;
  }

  // coding_quadtree (7.3.8.4) of one CTU (CTU coordinates)
  void write_ctu(int cx, int cy) {
    if (!c.ctu64) {
      write_block_tree(cx, cy, 0);
      return;
    }
    const int x0 = cx << 6, y0 = cy << 6;
    const bool inside = x0 + 64 <= W && y0 + 64 <= H;
    const bool one = inside && cu64_ok(cx, cy);
    if (inside) e.encode(!one, ctx[CTX_SPLIT_CU + split_ctx(x0, y0, 0)]);  // else the split is inferred
    if (one) {
      write_cu64_skip(x0, y0);
      return;
    }
    for (int q = 0; q < 4; ++q) {
      const int bx = (x0 >> 5) + (q & 1), by = (y0 >> 5) + (q >> 1);
      if ((bx << 5) < W && (by << 5) < H) write_block_tree(bx, by, 1);
    }
  }

  int split_ctx(int x, int y, int d) const {
    return (avail(x - 1, y) && depth[g(x - 1, y)] > d) + (avail(x, y - 1) && depth[g(x, y - 1)] > d);
  }

  // one 32x32 record block = one quantization group; dofs: its depth in the CTU quadtree
  void write_block_tree(int rx, int ry, int dofs) {
    const CtuInfo& t = ctu[ry * wctb + rx];
    const int x0 = rx * kCtb, y0 = ry * kCtb;
    qp_ctb = t.qp;
    qp_coded = false;
    qp_pred_cur = c.cu_qp_delta ? qg_pred(x0, y0) : fp.qp;
    scan_ctb_nz(x0, y0);
    const bool s32 = t.split & 1;
    e.encode(s32, ctx[CTX_SPLIT_CU + split_ctx(x0, y0, dofs)]);
    if (!s32) {
      write_cu(x0, y0, 5, dofs);
    } else {
      for (int q = 0; q < 4; ++q) {
        const int x1 = x0 + (q & 1) * 16, y1 = y0 + (q >> 1) * 16;
        const bool s16 = (t.split >> (1 + q)) & 1;
        e.encode(s16, ctx[CTX_SPLIT_CU + split_ctx(x1, y1, dofs + 1)]);
        if (!s16) {
          write_cu(x1, y1, 4, dofs + 1);
          continue;
        }
        for (int r = 0; r < 4; ++r) write_cu(x1 + (r & 1) * 8, y1 + (r >> 1) * 8, 3, dofs + 2);
      }
    }
    // qPY_PREV of the next quantization group: the QpY of this group's last CU
    if (c.cu_qp_delta) qp_prev = qp_coded ? qp_ctb : qp_pred_cur;
  }

  // a 64x64 skip CU stands for the CTU's four blocks when each is one 32x32 inter CU, all with
  // one motion, no level anywhere, and that motion is in the 64x64 CU's merge list (the
  // reconstruction is the same: motion compensation is per sample and every inner edge has
  // boundary strength 0)
  int cu64_midx = -1;
  bool cu64_ok(int cx, int cy) {
    const int x0 = cx << 6, y0 = cy << 6;
    if (!inter_slice) return false;
    Motion m0{};
    for (int q = 0; q < 4; ++q) {
      const int bx = (x0 >> 5) + (q & 1), by = (y0 >> 5) + (q >> 1);
      const CtuInfo& t = ctu[by * wctb + bx];
      const CuInfo& ci = cu[static_cast<size_t>(by * wctb + bx) * kCusPerCtb];
      if ((t.split & 1) || ci.pred != CU_INTER) return false;
      Motion m{static_cast<uint8_t>(cu_dir(ci)), {static_cast<int8_t>(ci.pad[0]), static_cast<int8_t>(ci.pad[1])},
               {{ci.mv[0], ci.mv[1]}, {ci.mv1[0], ci.mv1[1]}}};
      for (int X = 0; X < 2; ++X)
        if (!((m.dir >> X) & 1)) {
          m.m[X] = Mv{0, 0};
          m.r[X] = 0;
        }
      if (q == 0) m0 = m;
      else if (!(m == m0)) return false;
      scan_ctb_nz(bx << 5, by << 5);
      if (nz_luma || nz_chroma[0] || nz_chroma[1]) return false;
    }
    Motion ml[5];
    const int nm = merge_list(x0, y0, 64, ml);
    cu64_midx = -1;
    for (int k = 0; k < nm && cu64_midx < 0; ++k)
      if (ml[k] == m0) cu64_midx = k;
    cu64_mot = m0;
    return cu64_midx >= 0;
  }
  Motion cu64_mot;
  void write_cu64_skip(int x0, int y0) {
    const int skip_ctx = (avail(x0 - 1, y0) && skip[g(x0 - 1, y0)]) + (avail(x0, y0 - 1) && skip[g(x0, y0 - 1)]);
    e.encode(1, ctx[CTX_CU_SKIP + skip_ctx]);
    write_merge_idx(cu64_midx);
    mark(x0, y0, 64, 0, 1, CU_INTER, 1, cu64_mot);
    ++st.skip_cus;
    // one quantization group per CU at least as large as the group: QpY = the prediction
    const int q = c.cu_qp_delta ? qg_pred(x0, y0) : fp.qp;
    for (int yy = y0; yy < y0 + 64; yy += 8)
      for (int xx = x0; xx < x0 + 64; xx += 8) qpy[g(xx, yy)] = static_cast<int8_t>(q);
    if (c.cu_qp_delta) qp_prev = q;
  }
};

}  // namespace

std::vector<uint8_t> hevc_write_slice(const HevcConfig& c, const HevcFrameParams& fp, const CtuInfo* ctu,
                                      const CuInfo* cu, const int16_t* coef_y, const int16_t* coef_cb,
                                      const int16_t* coef_cr, HevcSliceStats* stats, const PackedLevels* packed) {
  BitWriter bw;
  // 7.3.6.1 slice_segment_header
  const bool idr = fp.idr != 0;
  bw.put_bit(1);              // first_slice_segment_in_pic_flag
  if (idr) bw.put_bit(0);     // no_output_of_prior_pics_flag
  bw.put_ue(0);               // slice_pic_parameter_set_id
  bw.put_ue(fp.slice_type);   // slice_type
  const bool inter = fp.slice_type != 2, bslice = fp.slice_type == 0;
  if (bslice && fp.ref_poc[1] < 0) throw std::runtime_error("HEVC: a B slice needs ref_poc[1]");
  if (inter && c.tmvp && !fp.col.set) throw std::runtime_error("HEVC: TMVP needs the collocated picture's records");
  if (!idr) {
    bw.put(fp.poc & 255, 8);  // slice_pic_order_cnt_lsb
    const int r0 = fp.ref_poc[0] >= 0 ? fp.ref_poc[0] : fp.poc - 1;
    // the short-term RPS: explicit, or the list references alone (all used)
    std::vector<std::pair<int, int>> neg, pos;  // (POC, used)
    if (fp.n_rps >= 0) {
      if (fp.n_rps > 8) throw std::runtime_error("HEVC: at most 8 RPS entries");
      for (int i = 0; i < fp.n_rps; ++i) {
        const int q = fp.rps_poc[i];
        if (q == fp.poc) throw std::runtime_error("HEVC: the RPS holds the current picture");
        (q < fp.poc ? neg : pos).emplace_back(q, fp.rps_used[i] ? 1 : 0);
      }
    } else {
      if (inter) neg.emplace_back(r0, 1);
      if (bslice) pos.emplace_back(fp.ref_poc[1], 1);
    }
    std::sort(neg.begin(), neg.end(), [](auto& a, auto& b) { return a.first > b.first; });  // closest first
    std::sort(pos.begin(), pos.end());
    // RefPicList0[0] = the closest used picture before (P: or after when none), RefPicList1[0]
    // = the closest used picture after (8.3.4 with one active entry per list)
    int l0 = -1, l1 = -1;
    for (auto& e : neg)
      if (e.second && l0 < 0) l0 = e.first;
    for (auto& e : pos)
      if (e.second && l1 < 0) l1 = e.first;
    if (inter && (l0 != r0 || (bslice && l1 != fp.ref_poc[1])))
      throw std::runtime_error("HEVC: RefPicList0 must precede and RefPicList1 follow the current picture (closest used RPS entries)");
    // several active pictures per list: each list must be the default construction (8.3.4,
    // RefPicListTemp0 = used pictures before, closest first, then after; list 1 the other way)
    for (int l = 0; l < (bslice ? 2 : (inter ? 1 : 0)); ++l) {
      const int nr = fp.num_ref[l];
      if (nr < 1 || nr > kMaxRefs) throw std::runtime_error("HEVC: num_ref outside 1..4");
      if (nr == 1) continue;
      std::vector<int> tmp;
      for (auto& e : l == 0 ? neg : pos)
        if (e.second) tmp.push_back(e.first);
      for (auto& e : l == 0 ? pos : neg)
        if (e.second) tmp.push_back(e.first);
      if (tmp.empty()) throw std::runtime_error("HEVC: no used reference picture");
      for (int i = 0; i < nr; ++i)
        if ((i == 0 ? (l == 0 ? r0 : fp.ref_poc[1]) : fp.list_poc[l][i]) != tmp[i % tmp.size()])
          throw std::runtime_error("HEVC: list_poc is not the default RefPicList construction of the RPS");
    }
    if (inter && !bslice && neg.size() == 1 && pos.empty() && neg[0].first == fp.poc - 1 && neg[0].second) {
      bw.put_bit(1);          // short_term_ref_pic_set_sps_flag (the single SPS set: no index bits)
    } else {
      // st_ref_pic_set(num_short_term_ref_pic_sets = 1) in the slice header (7.3.7)
      bw.put_bit(0);          // short_term_ref_pic_set_sps_flag
      bw.put_bit(0);          // inter_ref_pic_set_prediction_flag
      bw.put_ue(static_cast<uint32_t>(neg.size()));  // num_negative_pics
      bw.put_ue(static_cast<uint32_t>(pos.size()));  // num_positive_pics
      int prev = fp.poc;
      for (auto& e : neg) {
        bw.put_ue(prev - e.first - 1);  // delta_poc_s0_minus1
        bw.put_bit(e.second);           // used_by_curr_pic_s0_flag
        prev = e.first;
      }
      prev = fp.poc;
      for (auto& e : pos) {
        bw.put_ue(e.first - prev - 1);  // delta_poc_s1_minus1
        bw.put_bit(e.second);           // used_by_curr_pic_s1_flag
        prev = e.first;
      }
    }
    if (c.tmvp) bw.put_bit(1);  // slice_temporal_mvp_enabled_flag
  }
  if (c.sao) {
    bw.put_bit(1);            // slice_sao_luma_flag
    bw.put_bit(1);            // slice_sao_chroma_flag
  }
  if (inter) {
    // num_ref_idx_active_override_flag: the PPS defaults are one picture per list
    const int n0 = fp.num_ref[0], n1 = bslice ? fp.num_ref[1] : 1;
    const bool over = n0 != 1 || n1 != 1;
    bw.put_bit(over ? 1 : 0);
    if (over) {
      bw.put_ue(n0 - 1);              // num_ref_idx_l0_active_minus1
      if (bslice) bw.put_ue(n1 - 1);  // num_ref_idx_l1_active_minus1
    }
    if (bslice) bw.put_bit(0);  // mvd_l1_zero_flag
    if (c.tmvp && bslice) bw.put_bit(0);  // collocated_from_l0_flag: the collocated picture is RefPicList1[0]
    // collocated_ref_idx 0: RefPicList1[0] (B) / RefPicList0[0] (P)
    if (c.tmvp && ((bslice && n1 > 1) || (!bslice && n0 > 1))) bw.put_ue(0);
    if (c.weightp && !bslice) {
      // pred_weight_table (7.3.6.3): log2 denominators 6 / 6; weights on RefPicList0[0] only
      // (the other entries' flags are 0); the chroma offset is coded as its difference from the
      // weight-dependent prediction (7.4.7.3)
      bw.put_ue(6);                 // luma_log2_weight_denom
      bw.put_se(0);                 // delta_chroma_log2_weight_denom
      for (int i = 0; i < n0; ++i) bw.put_bit(i == 0 && fp.wp ? 1 : 0);  // luma_weight_l0_flag[i]
      for (int i = 0; i < n0; ++i) bw.put_bit(i == 0 && fp.wp ? 1 : 0);  // chroma_weight_l0_flag[i]
      if (fp.wp) {
        bw.put_se(fp.wp_w[0] - 64);  // delta_luma_weight_l0
        bw.put_se(fp.wp_o[0]);       // luma_offset_l0
        for (int j = 1; j < 3; ++j) {
          bw.put_se(fp.wp_w[j] - 64);  // delta_chroma_weight_l0
          bw.put_se(fp.wp_o[j] - 128 + ((128 * fp.wp_w[j]) >> 6));  // delta_chroma_offset_l0
        }
      }
    }
    bw.put_ue(5 - c.max_merge);  // five_minus_max_num_merge_cand
  }
  bw.put_se(fp.qp - 26);      // slice_qp_delta (init_qp 26)
  // CTUs (64x64 with ctu64, else the 32x32 record blocks themselves)
  const int wctb = c.wctu(), hctb = c.hctu(), n = wctb * hctb;
  PicState ps(static_cast<size_t>(c.coded_width() / 8) * (c.coded_height() / 8));
  HevcSliceStats total;
  std::vector<uint8_t> data;  // slice_segment_data() (RBSP, before emulation prevention)
  if (!c.wpp) {
    // byte_alignment()
    bw.put_bit(1);
    bw.align_zero();
    CabacEncoder enc(bw);
    enc.start();
    Writer w(c, fp, ctu, cu, coef_y, coef_cb, coef_cr, enc, ps);
    w.pk = packed;
    for (int i = 0; i < n; ++i) {
      const int rx = i % wctb, ry = i / wctb;
      if (c.sao) w.write_sao(rx, ry);
      w.write_ctu(rx, ry);
      enc.terminate(i == n - 1);  // end_of_slice_segment_flag
    }
    enc.finish();
    bw.put_bit(1);  // rbsp_slice_segment_trailing_bits: stop bit + alignment
    bw.align_zero();
    total = w.st;
    total.bins = enc.bins();
  } else {
    // Wavefront parallel processing (7.3.8.1, 9.3.1, 9.3.2.4): one substream per CTB row,
    // each row's contexts synchronised from the row above after its second CTB, rows coded
    // by `threads` host threads with a 2-CTB lag.
    std::vector<BitWriter> sub(hctb);
    std::vector<std::array<CtxState, kNumCtx>> saved(hctb);
    std::vector<HevcSliceStats> rst(hctb);
    std::unique_ptr<std::atomic<int>[]> prog(new std::atomic<int>[hctb]);
    for (int r = 0; r < hctb; ++r) prog[r].store(0, std::memory_order_relaxed);
    std::atomic<bool> abort{false};
    std::exception_ptr err;
    std::atomic<int> err_set{0};
    auto wait_for = [&](int r, int need) {
      while (prog[r].load(std::memory_order_acquire) < need) {
        if (abort.load(std::memory_order_relaxed)) throw std::runtime_error("HEVC WPP: aborted");
        std::this_thread::yield();
      }
    };
    const int T = std::max(1, std::min(c.threads, hctb));
    auto worker = [&](int t) {
      try {
        for (int ry = t; ry < hctb; ry += T) {
          CabacEncoder enc(sub[ry]);
          enc.start();
          Writer w(c, fp, ctu, cu, coef_y, coef_cb, coef_cr, enc, ps);
          w.pk = packed;
          if (ry > 0 && wctb >= 2) {  // 9.3.2.4 sync from CTB (1, ry-1)
            wait_for(ry - 1, 2);
            std::copy(saved[ry - 1].begin(), saved[ry - 1].end(), w.ctx);
          }
          for (int rx = 0; rx < wctb; ++rx) {
            if (ry > 0) wait_for(ry - 1, std::min(rx + 2, wctb));
            if (c.sao) w.write_sao(rx, ry);
            w.write_ctu(rx, ry);
            const bool last = ry == hctb - 1 && rx == wctb - 1;
            enc.terminate(last);  // end_of_slice_segment_flag
            if (rx == 1) std::copy(w.ctx, w.ctx + kNumCtx, saved[ry].begin());
            if (rx == wctb - 1 && !last) enc.terminate(1);  // end_of_subset_one_bit
            if (rx == wctb - 1) {
              enc.finish();
              // byte_alignment() after end_of_subset_one_bit; the last row's stop bit is the
              // rbsp_slice_segment_trailing_bits
              sub[ry].put_bit(1);
              sub[ry].align_zero();
              rst[ry] = w.st;
              rst[ry].bins = enc.bins();
            }
            prog[ry].store(rx + 1, std::memory_order_release);
          }
        }
      } catch (...) {
        if (err_set.exchange(1) == 0) err = std::current_exception();
        abort.store(true);
      }
    };
    if (T == 1) {
      worker(0);
    } else {
      std::vector<std::thread> th;
      for (int t = 0; t < T; ++t) th.emplace_back(worker, t);
      for (auto& x : th) x.join();
    }
    if (err) std::rethrow_exception(err);
    // entry points count emulation prevention bytes (7.4.7.1): every substream ends in a
    // non-zero byte, so its escaped size does not depend on its neighbours
    std::vector<uint32_t> esc(hctb);
    for (int r = 0; r < hctb; ++r) {
      const std::vector<uint8_t>& b = sub[r].bytes();
      uint32_t extra = 0;
      int zeros = 0;
      for (uint8_t v : b) {
        if (zeros >= 2 && v <= 3) {
          ++extra;
          zeros = 0;
        }
        zeros = v == 0 ? zeros + 1 : 0;
      }
      esc[r] = static_cast<uint32_t>(b.size()) + extra;
      data.insert(data.end(), b.begin(), b.end());
      total.bins += rst[r].bins;
      total.intra_cus += rst[r].intra_cus;
      total.inter_cus += rst[r].inter_cus;
      total.skip_cus += rst[r].skip_cus;
      total.merge_cus += rst[r].merge_cus;
    }
    bw.put_ue(hctb - 1);  // num_entry_point_offsets
    if (hctb > 1) {
      uint32_t mx = 1;
      for (int r = 0; r + 1 < hctb; ++r) mx = std::max(mx, esc[r]);
      int len = 1;
      while (len < 32 && (static_cast<uint64_t>(mx - 1) >> len) != 0) ++len;
      bw.put_ue(len - 1);  // offset_len_minus1
      for (int r = 0; r + 1 < hctb; ++r) bw.put(esc[r] - 1, len);  // entry_point_offset_minus1
    }
    bw.put_bit(1);  // byte_alignment()
    bw.align_zero();
    bw.append_bytes(data.data(), data.size());
  }
  std::vector<uint8_t> out;
  append_hevc_nal(out, idr ? NAL_IDR_W_RADL : (fp.nal_ref ? NAL_TRAIL_R : NAL_TRAIL_N), bw.bytes());
  if (stats) {
    *stats = total;
    stats->bytes = out.size();
  }
  return out;
}

}  // namespace hevc
}  // namespace mivc
