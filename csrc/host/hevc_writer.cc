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

// 7.3.6.1 slice_segment_header up to slice_qp_delta (the entry points follow the CTU coding)
void slice_header(BitWriter& bw, const HevcConfig& c, const HevcFrameParams& fp) {
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
}

// per-8x8-granule state of one picture's coded CUs (hevc_ctu_coder.h CoderState)
struct PicState {
  std::vector<int8_t> depth, skip, pred, mode4;
  std::vector<Motion> mot;
  std::vector<uint8_t> coded;
  std::vector<int8_t> qpy;
  explicit PicState(size_t n)
      : depth(n, 0), skip(n, 0), pred(n, 0), mode4(4 * n, 1), mot(n, motion_none()), coded(n, 0), qpy(n, 0) {}
  CoderState view() {
    return CoderState{depth.data(), skip.data(), pred.data(), mode4.data(), mot.data(), coded.data(), qpy.data()};
  }
};

// entry points (WPP), byte_alignment(), the substreams, and the NAL around the RBSP
std::vector<uint8_t> finish_slice(BitWriter& bw, const HevcConfig& c, const HevcFrameParams& fp,
                                  const uint8_t* const* sub, const uint32_t* sizes, int nsub) {
  if (c.wpp) {
    if (nsub != c.hctu()) throw std::runtime_error("HEVC: one substream per CTU row with WPP");
    // entry points count emulation prevention bytes (7.4.7.1): every substream ends in a
    // non-zero byte, so its escaped size does not depend on its neighbours
    std::vector<uint32_t> esc(nsub);
    for (int r = 0; r < nsub; ++r) {
      uint32_t extra = 0;
      int zeros = 0;
      for (uint32_t i = 0; i < sizes[r]; ++i) {
        const uint8_t v = sub[r][i];
        if (zeros >= 2 && v <= 3) {
          ++extra;
          zeros = 0;
        }
        zeros = v == 0 ? zeros + 1 : 0;
      }
      esc[r] = sizes[r] + extra;
    }
    bw.put_ue(nsub - 1);  // num_entry_point_offsets
    if (nsub > 1) {
      uint32_t mx = 1;
      for (int r = 0; r + 1 < nsub; ++r) mx = std::max(mx, esc[r]);
      int len = 1;
      while (len < 32 && (static_cast<uint64_t>(mx - 1) >> len) != 0) ++len;
      bw.put_ue(len - 1);  // offset_len_minus1
      for (int r = 0; r + 1 < nsub; ++r) bw.put(esc[r] - 1, len);  // entry_point_offset_minus1
    }
  } else if (nsub != 1) {
    throw std::runtime_error("HEVC: one substream per slice without WPP");
  }
  bw.put_bit(1);  // byte_alignment()
  bw.align_zero();
  for (int r = 0; r < nsub; ++r) bw.append_bytes(sub[r], sizes[r]);
  std::vector<uint8_t> out;
  append_hevc_nal(out, fp.idr ? NAL_IDR_W_RADL : (fp.nal_ref ? NAL_TRAIL_R : NAL_TRAIL_N), bw.bytes());
  return out;
}

}  // namespace

CoderPic hevc_coder_pic(const HevcConfig& c, const HevcFrameParams& fp) {
  CoderPic p{};
  p.W = c.coded_width();
  p.H = c.coded_height();
  p.wctb = c.wctb();
  p.hctb = c.hctb();
  p.wctu = c.wctu();
  p.hctu = c.hctu();
  p.L = c.ctb_log2();
  p.ctu64 = c.ctu64;
  p.sao = c.sao;
  p.max_merge = c.max_merge;
  p.tmvp = c.tmvp;
  p.cu_qp_delta = c.cu_qp_delta;
  p.bit_depth = c.bit_depth;
  p.tu_inter_depth = c.tu_inter_depth;
  p.sdh = c.sdh;
  p.wpp = c.wpp;
  p.slice_type = fp.slice_type;
  p.qp = fp.qp;
  p.poc = fp.poc;
  for (int l = 0; l < 2; ++l) {
    p.ref_poc[l] = fp.ref_poc[l];
    p.num_ref[l] = fp.num_ref[l];
    p.col_ref_poc[l] = fp.col.ref_poc[l];
    for (int i = 0; i < kMaxRefs; ++i) {
      p.list_poc[l][i] = fp.list_poc[l][i];
      p.col_list_poc[l][i] = fp.col.list_poc[l][i];
    }
  }
  p.col_set = fp.col.set;
  p.col_poc = fp.col.poc;
  return p;
}

std::vector<uint8_t> hevc_assemble_slice(const HevcConfig& c, const HevcFrameParams& fp, const uint8_t* const* sub,
                                         const uint32_t* sizes, int nsub) {
  BitWriter bw;
  slice_header(bw, c, fp);
  return finish_slice(bw, c, fp, sub, sizes, nsub);
}

std::vector<uint8_t> hevc_write_slice(const HevcConfig& c, const HevcFrameParams& fp, const CtuInfo* ctu,
                                      const CuInfo* cu, const int16_t* coef_y, const int16_t* coef_cb,
                                      const int16_t* coef_cr, HevcSliceStats* stats, const PackedLevels* packed,
                                      std::vector<std::vector<uint8_t>>* substreams) {
  BitWriter bw;
  slice_header(bw, c, fp);
  // CTUs (64x64 with ctu64, else the 32x32 record blocks themselves): one substream per CTU
  // row with WPP (7.3.8.1, 9.3.1, 9.3.2.4: each row's contexts synchronised from the row
  // above after its second CTU; rows coded by `threads` host threads with a 2-CTU lag), else
  // one for the slice
  const CoderPic P = hevc_coder_pic(c, fp);
  const int wctu = P.wctu, hctu = P.hctu;
  PicState ps(static_cast<size_t>(P.W / 8) * (P.H / 8));
  const CoderState cs = ps.view();
  CoderLevels lv;
  if (packed) {
    lv.nzmap = packed->nzmap;
    lv.ctb_off = packed->ctb_off;
    lv.levels = packed->levels;
    lv.nblocks = packed->nblocks;
  } else {
    lv.plane[0] = coef_y;
    lv.plane[1] = coef_cb;
    lv.plane[2] = coef_cr;
  }
  const CuInfo* col = (fp.col.set && c.tmvp && fp.slice_type != 2) ? fp.col.cu : nullptr;
  const int nsub = c.wpp ? hctu : 1;
  std::vector<BitWriter> sub(nsub);
  std::vector<std::array<CtxState, kNumCtx>> saved(hctu);
  std::vector<HevcSliceStats> rst(nsub);
  std::unique_ptr<std::atomic<int>[]> prog(new std::atomic<int>[hctu]);
  for (int r = 0; r < hctu; ++r) prog[r].store(0, std::memory_order_relaxed);
  std::atomic<bool> abort{false};
  std::exception_ptr err;
  std::atomic<int> err_set{0};
  auto wait_for = [&](int r, int need) {
    while (prog[r].load(std::memory_order_acquire) < need) {
      if (abort.load(std::memory_order_relaxed)) throw std::runtime_error("HEVC WPP: aborted");
      std::this_thread::yield();
    }
  };
  auto code_rows = [&](int r0, int r1, int s) {  // rows [r0, r1) into substream s
    CtuCoder<BitWriter> w;
    CtxState ctx[kNumCtx];
    w.begin(&P, ctu, cu, col, lv, cs, ctx, &sub[s]);
    for (int ry = r0; ry < r1; ++ry) {
      if (c.wpp && ry > 0 && wctu >= 2) {  // 9.3.2.4 sync from CTU (1, ry-1)
        wait_for(ry - 1, 2);
        std::copy(saved[ry - 1].begin(), saved[ry - 1].end(), ctx);
      }
      for (int rx = 0; rx < wctu; ++rx) {
        if (c.wpp && ry > 0) wait_for(ry - 1, std::min(rx + 2, wctu));
        w.code_ctu(rx, ry);
        if (w.err) throw std::runtime_error(coder_error_text(w.err));
        if (rx == 1) std::copy(ctx, ctx + kNumCtx, saved[ry].begin());
        prog[ry].store(rx + 1, std::memory_order_release);
      }
    }
    HevcSliceStats& t = rst[s];
    t.bins = w.e.bins();
    t.intra_cus = w.st.intra_cus;
    t.inter_cus = w.st.inter_cus;
    t.skip_cus = w.st.skip_cus;
    t.merge_cus = w.st.merge_cus;
  };
  const int T = c.wpp ? std::max(1, std::min(c.threads, hctu)) : 1;
  auto worker = [&](int t) {
    try {
      if (!c.wpp) {
        code_rows(0, hctu, 0);
        return;
      }
      for (int ry = t; ry < hctu; ry += T) {
        // each row restarts the engine and the contexts: a coder per row
        code_rows(ry, ry + 1, ry);
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
  std::vector<const uint8_t*> ptrs(nsub);
  std::vector<uint32_t> sizes(nsub);
  HevcSliceStats total;
  for (int r = 0; r < nsub; ++r) {
    ptrs[r] = sub[r].bytes().data();
    sizes[r] = static_cast<uint32_t>(sub[r].bytes().size());
    total.bins += rst[r].bins;
    total.intra_cus += rst[r].intra_cus;
    total.inter_cus += rst[r].inter_cus;
    total.skip_cus += rst[r].skip_cus;
    total.merge_cus += rst[r].merge_cus;
  }
  if (substreams)  // the slice data as coded, before the entry points (tests of hevc_assemble_slice)
    for (int r = 0; r < nsub; ++r) substreams->push_back(sub[r].bytes());
  std::vector<uint8_t> out = finish_slice(bw, c, fp, ptrs.data(), sizes.data(), nsub);
  if (stats) {
    *stats = total;
    stats->bytes = out.size();
  }
  return out;
}

}  // namespace hevc
}  // namespace mivc
