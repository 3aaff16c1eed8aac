#include "h264_syntax.h"

#include <cmath>
#include <cstring>
#include <stdexcept>

#include "../common/h264_cabac_tables.h"  // kZigzag8x8

namespace mivc {
namespace h264 {

void flat_scaling(uint8_t (*sl4)[16], uint8_t (*sl8)[64]) {
  std::memset(sl4, 16, 6 * 16);
  std::memset(sl8, 16, 2 * 64);
}
SPS::SPS() { flat_scaling(sl4, sl8); }
PPS::PPS() { flat_scaling(sl4, sl8); }

namespace {

// scan position -> raster index of a 4x4 / 8x8 list
int scan_raster(int n, int j) { return n == 16 ? kZigzag4x4[j] : kZigzag8x8[j]; }

// 7.3.2.1.1.1 scaling_list(): delta-coded in scan order; returns useDefaultScalingMatrixFlag
bool read_scaling_list(BitReader& br, uint8_t* out_raster, int n) {
  int last = 8, next = 8;
  bool use_default = false;
  for (int j = 0; j < n; ++j) {
    if (next != 0) {
      const int delta = br.get_se_range(-128, 127, "delta_scale");
      next = (last + delta + 256) % 256;
      use_default = j == 0 && next == 0;
    }
    const int v = next == 0 ? last : next;
    out_raster[scan_raster(n, j)] = static_cast<uint8_t>(v);
    last = v;
  }
  return use_default;
}

void write_scaling_list(BitWriter& bw, const uint8_t* raster, int n) {
  int last = 8;
  for (int j = 0; j < n; ++j) {
    const int v = raster[scan_raster(n, j)];
    if (v < 1) throw std::runtime_error("scaling list entries must be 1..255");
    int delta = v - last;
    if (delta > 127) delta -= 256;
    if (delta < -128) delta += 256;
    bw.put_se(delta);
    last = v;
  }
}

void default_list(int i, uint8_t* raster) {
  const int intra = i < 3 || i == 6 ? 0 : 1;
  if (i < 6)
    for (int j = 0; j < 16; ++j) raster[kZigzag4x4[j]] = kDefault4x4[intra][j];
  else
    for (int j = 0; j < 64; ++j) raster[kZigzag8x8[j]] = kDefault8x8[intra][j];
}

// lists 0..7 (n8 = 2 for 4:2:0) with fall-back rule A (fallback == nullptr: the defaults for
// lists 0 / 3 / 6 / 7) or rule B (fallback: the sequence-level lists)
void read_matrix(BitReader& br, int n8, uint8_t (*sl4)[16], uint8_t (*sl8)[64], const uint8_t (*fb4)[16],
                 const uint8_t (*fb8)[64]) {
  for (int i = 0; i < 6 + n8; ++i) {
    uint8_t* dst = i < 6 ? sl4[i] : sl8[i - 6];
    const int n = i < 6 ? 16 : 64;
    if (br.get_bit()) {
      if (read_scaling_list(br, dst, n)) default_list(i, dst);
    } else if (i == 0 || i == 3 || i == 6 || i == 7) {
      if (fb4) std::memcpy(dst, i < 6 ? fb4[i] : fb8[i - 6], n);
      else default_list(i, dst);
    } else {
      std::memcpy(dst, sl4[i - 1], 16);  // Cb from Y, Cr from Cb of the same kind
    }
  }
  if (n8 < 2)
    for (int i = n8; i < 2; ++i) default_list(6 + i, sl8[i]);
}

void write_matrix(BitWriter& bw, int n8, const uint8_t (*sl4)[16], const uint8_t (*sl8)[64], const uint8_t* coded) {
  for (int i = 0; i < 6 + n8; ++i) {
    bw.put_bit(coded[i]);
    if (coded[i]) write_scaling_list(bw, i < 6 ? sl4[i] : sl8[i - 6], i < 6 ? 16 : 64);
  }
}

}  // namespace

static bool high_profile(int p) {
  return p == 100 || p == 110 || p == 122 || p == 244 || p == 44 || p == 83 || p == 86 || p == 118 ||
         p == 128 || p == 138 || p == 139 || p == 134 || p == 135;
}

void write_sps(BitWriter& bw, const SPS& s) {
  bw.put(s.profile_idc, 8);
  bw.put(s.constraint_flags & 0xFC, 8);  // 6 constraint flags + reserved_zero_2bits
  bw.put(s.level_idc, 8);
  bw.put_ue(s.sps_id);
  if (high_profile(s.profile_idc)) {
    bw.put_ue(s.chroma_format_idc);
    bw.put_ue(s.bit_depth_luma - 8);
    bw.put_ue(s.bit_depth_chroma - 8);
    bw.put_bit(0);  // qpprime_y_zero_transform_bypass_flag
    bw.put_bit(s.scaling_present);  // seq_scaling_matrix_present_flag
    if (s.scaling_present) write_matrix(bw, 2, s.sl4, s.sl8, s.sl_coded);
  }
  bw.put_ue(s.log2_max_frame_num - 4);
  bw.put_ue(s.poc_type);
  if (s.poc_type == 0) bw.put_ue(s.log2_max_poc_lsb - 4);
  if (s.poc_type == 1) throw std::runtime_error("poc_type 1 not written");
  bw.put_ue(s.max_num_ref_frames);
  bw.put_bit(s.gaps_allowed);
  bw.put_ue(s.width_mbs - 1);
  bw.put_ue(s.height_mbs - 1);
  bw.put_bit(1);  // frame_mbs_only_flag
  bw.put_bit(s.direct_8x8_inference);
  bool crop = s.crop_left || s.crop_right || s.crop_top || s.crop_bottom;
  bw.put_bit(crop);
  if (crop) {
    bw.put_ue(s.crop_left);
    bw.put_ue(s.crop_right);
    bw.put_ue(s.crop_top);
    bw.put_ue(s.crop_bottom);
  }
  bw.put_bit(s.vui_present);
  if (s.vui_present) {
    bw.put_bit(0);  // aspect_ratio_info_present_flag
    bw.put_bit(0);  // overscan_info_present_flag
    bw.put_bit(0);  // video_signal_type_present_flag
    bw.put_bit(0);  // chroma_loc_info_present_flag
    bw.put_bit(1);  // timing_info_present_flag
    bw.put(s.num_units_in_tick, 32);
    bw.put(s.time_scale, 32);
    bw.put_bit(s.fixed_frame_rate);
    bw.put_bit(0);  // nal_hrd_parameters_present_flag
    bw.put_bit(0);  // vcl_hrd_parameters_present_flag
    bw.put_bit(0);  // pic_struct_present_flag
    bw.put_bit(1);  // bitstream_restriction_flag
    bw.put_bit(1);  // motion_vectors_over_pic_boundaries_flag
    bw.put_ue(0);   // max_bytes_per_pic_denom
    bw.put_ue(0);   // max_bits_per_mb_denom
    bw.put_ue(16);  // log2_max_mv_length_horizontal
    bw.put_ue(16);  // log2_max_mv_length_vertical
    bw.put_ue(s.max_num_reorder);   // max_num_reorder_frames (consecutive B-frames)
    bw.put_ue(s.max_num_ref_frames);  // max_dec_frame_buffering
  }
  bw.trailing();
}

void write_pps(BitWriter& bw, const PPS& p) {
  bw.put_ue(p.pps_id);
  bw.put_ue(p.sps_id);
  bw.put_bit(p.entropy_coding_mode);
  bw.put_bit(p.bottom_field_pic_order_present);
  bw.put_ue(0);  // num_slice_groups_minus1
  bw.put_ue(p.num_ref_idx_l0_default - 1);
  bw.put_ue(p.num_ref_idx_l1_default - 1);
  bw.put_bit(p.weighted_pred);
  bw.put(p.weighted_bipred_idc, 2);
  bw.put_se(p.pic_init_qp - 26);
  bw.put_se(p.pic_init_qs - 26);
  bw.put_se(p.chroma_qp_index_offset);
  bw.put_bit(p.deblocking_filter_control_present);
  bw.put_bit(p.constrained_intra_pred);
  bw.put_bit(p.redundant_pic_cnt_present);
  if (p.transform_8x8_mode || p.scaling_present || p.second_chroma_qp_index_offset != p.chroma_qp_index_offset) {
    bw.put_bit(p.transform_8x8_mode);
    bw.put_bit(p.scaling_present);  // pic_scaling_matrix_present_flag
    if (p.scaling_present) write_matrix(bw, p.transform_8x8_mode ? 2 : 0, p.sl4, p.sl8, p.sl_coded);
    bw.put_se(p.second_chroma_qp_index_offset);
  }
  bw.trailing();
}

void write_slice_header(BitWriter& bw, const SliceHeader& h, const SPS& s, const PPS& p) {
  bw.put_ue(h.first_mb);
  bw.put_ue(h.slice_type + 5);
  bw.put_ue(h.pps_id);
  bw.put(h.frame_num & ((1u << s.log2_max_frame_num) - 1), s.log2_max_frame_num);
  if (h.nal_unit_type == NAL_IDR) bw.put_ue(h.idr_pic_id);
  if (s.poc_type == 0) bw.put(h.poc_lsb & ((1u << s.log2_max_poc_lsb) - 1), s.log2_max_poc_lsb);
  if (h.slice_type == SLICE_B) bw.put_bit(h.direct_spatial);
  if (h.slice_type == SLICE_P || h.slice_type == SLICE_B) {
    bw.put_bit(h.num_ref_idx_override);
    if (h.num_ref_idx_override) {
      bw.put_ue(h.num_ref_idx_l0_active - 1);
      if (h.slice_type == SLICE_B) bw.put_ue(h.num_ref_idx_l1_active - 1);
    }
    // ref_pic_list_modification() (7.3.3.1)
    for (int l = 0; l < (h.slice_type == SLICE_B ? 2 : 1); ++l) {
      bw.put_bit(!h.mods[l].empty());
      if (h.mods[l].empty()) continue;
      for (const RefMod& m : h.mods[l]) {
        bw.put_ue(m.idc);
        bw.put_ue(m.value);
      }
      bw.put_ue(3);
    }
  }
  if (p.weighted_bipred_idc == 1 && h.slice_type == SLICE_B)
    throw std::runtime_error("explicit weighted bi-prediction is not written");
  if (p.weighted_pred && h.slice_type == SLICE_P) {
    // pred_weight_table() (7.3.3.2), list 0; references without explicit weights: flags 0
    const WeightTable& w = h.wt;
    const bool any = h.has_weights;
    bw.put_ue(any ? w.luma_log2 : 0);
    bw.put_ue(any ? w.chroma_log2 : 0);  // ChromaArrayType 1
    for (int i = 0; i < h.num_ref_idx_l0_active; ++i) {
      const bool lf = any && w.lflag[0][i];
      bw.put_bit(lf);
      if (lf) {
        bw.put_se(w.lw[0][i]);
        bw.put_se(w.lo[0][i]);
      }
      const bool cf = any && w.cflag[0][i];
      bw.put_bit(cf);
      if (cf)
        for (int j = 0; j < 2; ++j) {
          bw.put_se(w.cw[0][i][j]);
          bw.put_se(w.co[0][i][j]);
        }
    }
  }
  if (h.nal_ref_idc) {
    if (h.nal_unit_type == NAL_IDR) {
      bw.put_bit(h.no_output_of_prior_pics);
      bw.put_bit(h.long_term_reference);
    } else {
      // adaptive_ref_pic_marking_mode_flag: sliding window, or the listed operations (7.3.3.3)
      bw.put_bit(h.adaptive_ref_pic_marking && !h.mmco.empty());
      if (h.adaptive_ref_pic_marking && !h.mmco.empty()) {
        for (const Mmco& m : h.mmco) {
          bw.put_ue(m.op);
          if (m.op == 1 || m.op == 3) bw.put_ue(m.diff_minus1);
          if (m.op == 2) bw.put_ue(m.long_term_pic_num);
          if (m.op == 3 || m.op == 6) bw.put_ue(m.long_term_frame_idx);
          if (m.op == 4) bw.put_ue(m.max_long_term_frame_idx_plus1);
        }
        bw.put_ue(0);
      }
    }
  }
  if (p.entropy_coding_mode && h.slice_type != SLICE_I) bw.put_ue(h.cabac_init_idc);
  bw.put_se(h.slice_qp_delta);
  if (p.deblocking_filter_control_present) {
    bw.put_ue(h.disable_deblocking_filter_idc);
    if (h.disable_deblocking_filter_idc != 1) {
      bw.put_se(h.alpha_offset_div2);
      bw.put_se(h.beta_offset_div2);
    }
  }
}


static void skip_hrd(BitReader& br) {
  const int cpb_cnt = br.get_ue_max(31, "cpb_cnt_minus1") + 1;
  br.get(4);
  br.get(4);
  for (int i = 0; i < cpb_cnt; ++i) {
    br.get_ue();
    br.get_ue();
    br.get_bit();
  }
  br.get(5);
  br.get(5);
  br.get(5);
  br.get(5);
}

SPS parse_sps(BitReader& br) {
  SPS s;
  s.profile_idc = br.get(8);
  s.constraint_flags = br.get(8);
  s.level_idc = br.get(8);
  s.sps_id = br.get_ue_max(31, "seq_parameter_set_id");
  if (high_profile(s.profile_idc)) {
    s.chroma_format_idc = br.get_ue_max(3, "chroma_format_idc");
    if (s.chroma_format_idc == 3) br.get_bit();
    s.bit_depth_luma = br.get_ue_max(6, "bit_depth_luma_minus8") + 8;
    s.bit_depth_chroma = br.get_ue_max(6, "bit_depth_chroma_minus8") + 8;
    br.get_bit();
    s.scaling_present = br.get_bit();
    if (s.scaling_present) {
      if (s.chroma_format_idc == 3) throw std::runtime_error("4:4:4 scaling matrices not supported");
      read_matrix(br, 2, s.sl4, s.sl8, nullptr, nullptr);  // fall-back rule A
    }
  }
  // 4:2:0 at 8 bits (Baseline .. High) or 9..14 bits (High 10 and the 4:2:0 intra / predictive profiles)
  if (s.chroma_format_idc != 1) throw std::runtime_error("only 4:2:0 supported");
  if (s.bit_depth_luma > 14 || s.bit_depth_chroma > 14) throw std::runtime_error("bit depth above 14");
  // one sample depth for all planes: the picture records (DecodedPicture, the int16 batch planes) carry one
  // depth, so a stream with BitDepthC != BitDepthY is refused here rather than mis-scaled downstream
  if (s.bit_depth_luma != s.bit_depth_chroma) throw std::runtime_error("luma and chroma bit depths differ");
  s.log2_max_frame_num = br.get_ue_max(12, "log2_max_frame_num_minus4") + 4;
  s.poc_type = br.get_ue_max(2, "pic_order_cnt_type");
  if (s.poc_type == 0) {
    s.log2_max_poc_lsb = br.get_ue_max(12, "log2_max_pic_order_cnt_lsb_minus4") + 4;
  } else if (s.poc_type == 1) {
    s.delta_pic_order_always_zero = br.get_bit();
    // deliberate restriction: the spec bounds these offsets to +-(2^31-1); this decoder accepts +-2^24
    // so the 32-bit expected-POC sums (8.2.1.2) cannot overflow, and refuses anything larger
    s.offset_for_non_ref_pic = br.get_se_range(-(1 << 24), 1 << 24, "offset_for_non_ref_pic");
    s.offset_for_top_to_bottom = br.get_se_range(-(1 << 24), 1 << 24, "offset_for_top_to_bottom_field");
    const int n = br.get_ue_max(255, "num_ref_frames_in_pic_order_cnt_cycle");
    for (int i = 0; i < n; ++i) s.offset_for_ref_frame.push_back(br.get_se_range(-(1 << 24), 1 << 24, "offset_for_ref_frame"));
  }
  s.max_num_ref_frames = br.get_ue_max(16, "max_num_ref_frames");
  s.gaps_allowed = br.get_bit();
  // level 6.2 (MaxFS 139264 MBs, A.3.1 f/g): each side is at most sqrt(8 * MaxFS) = 1055 MBs
  s.width_mbs = br.get_ue_max(1054, "pic_width_in_mbs_minus1") + 1;
  s.height_mbs = br.get_ue_max(1054, "pic_height_in_map_units_minus1") + 1;
  s.frame_mbs_only = br.get_bit();
  if (!s.frame_mbs_only) throw std::runtime_error("interlaced streams not supported");
  s.direct_8x8_inference = br.get_bit();
  if (br.get_bit()) {
    s.crop_left = br.get_ue_max(8 * s.width_mbs, "frame_crop_left_offset");
    s.crop_right = br.get_ue_max(8 * s.width_mbs, "frame_crop_right_offset");
    s.crop_top = br.get_ue_max(8 * s.height_mbs, "frame_crop_top_offset");
    s.crop_bottom = br.get_ue_max(8 * s.height_mbs, "frame_crop_bottom_offset");
    if (2 * (s.crop_left + s.crop_right) >= 16 * s.width_mbs || 2 * (s.crop_top + s.crop_bottom) >= 16 * s.height_mbs)
      throw std::runtime_error("frame cropping removes the whole picture");
  }
  s.vui_present = br.get_bit();
  if (s.vui_present) {
    if (br.get_bit()) {  // aspect_ratio_info_present_flag
      if (br.get(8) == 255) {
        br.get(16);
        br.get(16);
      }
    }
    if (br.get_bit()) br.get_bit();  // overscan
    if (br.get_bit()) {              // video_signal_type
      br.get(3);
      br.get_bit();
      if (br.get_bit()) {
        br.get(8);
        br.get(8);
        br.get(8);
      }
    }
    if (br.get_bit()) {
      br.get_ue();
      br.get_ue();
    }
    if (br.get_bit()) {
      s.num_units_in_tick = br.get(32);
      s.time_scale = br.get(32);
      s.fixed_frame_rate = br.get_bit();
    }
    int nal_hrd = br.get_bit();
    if (nal_hrd) skip_hrd(br);
    int vcl_hrd = br.get_bit();
    if (vcl_hrd) skip_hrd(br);
    if (nal_hrd || vcl_hrd) br.get_bit();
    br.get_bit();  // pic_struct_present_flag
    if (br.get_bit()) {
      s.vui_reorder_present = 1;
      br.get_bit();
      for (int i = 0; i < 4; ++i) br.get_ue();
      s.max_num_reorder = br.get_ue_max(16, "max_num_reorder_frames");
      br.get_ue();
    }
  }
  return s;
}

PPS parse_pps(BitReader& br, const SPS* sps_table) {
  PPS p;
  p.pps_id = br.get_ue_max(255, "pic_parameter_set_id");
  p.sps_id = br.get_ue_max(31, "seq_parameter_set_id");
  p.entropy_coding_mode = br.get_bit();
  p.bottom_field_pic_order_present = br.get_bit();
  if (br.get_ue() != 0) throw std::runtime_error("slice groups (FMO) not supported");
  p.num_ref_idx_l0_default = br.get_ue_max(31, "num_ref_idx_l0_default_active_minus1") + 1;
  p.num_ref_idx_l1_default = br.get_ue_max(31, "num_ref_idx_l1_default_active_minus1") + 1;
  p.weighted_pred = br.get_bit();
  p.weighted_bipred_idc = br.get(2);
  p.pic_init_qp = 26 + br.get_se_range(-26 - 6 * 6, 25, "pic_init_qp_minus26");
  p.pic_init_qs = 26 + br.get_se_range(-26, 25, "pic_init_qs_minus26");
  p.chroma_qp_index_offset = br.get_se_range(-12, 12, "chroma_qp_index_offset");
  p.deblocking_filter_control_present = br.get_bit();
  p.constrained_intra_pred = br.get_bit();
  p.redundant_pic_cnt_present = br.get_bit();
  p.second_chroma_qp_index_offset = p.chroma_qp_index_offset;
  // the picture's scaling lists: the sequence's unless the PPS sends its own
  const SPS& sps = sps_table[p.sps_id];
  std::memcpy(p.sl4, sps.sl4, sizeof(p.sl4));
  std::memcpy(p.sl8, sps.sl8, sizeof(p.sl8));
  if (br.more_rbsp_data()) {
    p.transform_8x8_mode = br.get_bit();
    p.scaling_present = br.get_bit();
    if (p.scaling_present) {
      if (sps.chroma_format_idc == 3) throw std::runtime_error("4:4:4 scaling matrices not supported");
      // fall-back rule B onto the sequence lists when the SPS has them, else rule A
      uint8_t sl4[6][16], sl8[2][64];
      if (sps.scaling_present) read_matrix(br, p.transform_8x8_mode ? 2 : 0, sl4, sl8, sps.sl4, sps.sl8);
      else read_matrix(br, p.transform_8x8_mode ? 2 : 0, sl4, sl8, nullptr, nullptr);
      std::memcpy(p.sl4, sl4, sizeof(sl4));
      std::memcpy(p.sl8, sl8, sizeof(sl8));
    }
    p.second_chroma_qp_index_offset = br.get_se_range(-12, 12, "second_chroma_qp_index_offset");
  }
  return p;
}

SliceHeader parse_slice_header(BitReader& br, int nal_unit_type, int nal_ref_idc, const SPS* sps_table,
                               const PPS* pps_table) {
  SliceHeader h;
  h.nal_unit_type = nal_unit_type;
  h.nal_ref_idc = nal_ref_idc;
  h.first_mb = br.get_ue_max((1u << 20) - 1, "first_mb_in_slice");
  const int st = br.get_ue_max(9, "slice_type");
  h.slice_type = st % 5;
  if (h.slice_type > 2) throw std::runtime_error("SP/SI slices not supported");
  h.pps_id = br.get_ue_max(255, "pic_parameter_set_id");
  const PPS& p = pps_table[h.pps_id];
  const SPS& s = sps_table[p.sps_id];
  h.frame_num = br.get(s.log2_max_frame_num);
  if (nal_unit_type == NAL_IDR) h.idr_pic_id = br.get_ue_max(65535, "idr_pic_id");
  if (s.poc_type == 0) {
    h.poc_lsb = br.get(s.log2_max_poc_lsb);
    if (p.bottom_field_pic_order_present) h.poc_bottom_delta = br.get_se_range(-(1 << 24), 1 << 24, "delta_pic_order_cnt_bottom");
  }
  if (s.poc_type == 1 && !s.delta_pic_order_always_zero) {
    h.delta_poc[0] = br.get_se_range(-(1 << 24), 1 << 24, "delta_pic_order_cnt[0]");
    if (p.bottom_field_pic_order_present) h.delta_poc[1] = br.get_se_range(-(1 << 24), 1 << 24, "delta_pic_order_cnt[1]");
  }
  if (p.redundant_pic_cnt_present && br.get_ue() != 0) throw std::runtime_error("redundant pictures not supported");
  if (h.slice_type == SLICE_B) h.direct_spatial = br.get_bit();
  h.num_ref_idx_l0_active = p.num_ref_idx_l0_default;
  h.num_ref_idx_l1_active = p.num_ref_idx_l1_default;
  if (h.slice_type == SLICE_P || h.slice_type == SLICE_B) {
    h.num_ref_idx_override = br.get_bit();
    if (h.num_ref_idx_override) {
      h.num_ref_idx_l0_active = br.get_ue_max(31, "num_ref_idx_l0_active_minus1") + 1;
      if (h.slice_type == SLICE_B) h.num_ref_idx_l1_active = br.get_ue_max(31, "num_ref_idx_l1_active_minus1") + 1;
    }
    for (int l = 0; l < (h.slice_type == SLICE_B ? 2 : 1); ++l) {
      if (!br.get_bit()) continue;  // ref_pic_list_modification_flag_lX
      for (int guard = 0;; ++guard) {
        if (guard > 64) throw std::runtime_error("ref_pic_list_modification too long");
        const int idc = br.get_ue_max(3, "modification_of_pic_nums_idc");
        if (idc == 3) break;
        // abs_diff_pic_num_minus1 < MaxPicNum (<= 2^16) or long_term_pic_num < 32
        h.mods[l].push_back(RefMod{idc, br.get_ue_max(idc == 2 ? 31 : 65535, "ref_pic_list_modification value")});
      }
    }
  }
  if ((p.weighted_pred && h.slice_type == SLICE_P) || (p.weighted_bipred_idc == 1 && h.slice_type == SLICE_B)) {
    h.has_weights = true;
    WeightTable& w = h.wt;
    w.luma_log2 = br.get_ue_max(7, "luma_log2_weight_denom");
    w.chroma_log2 = br.get_ue_max(7, "chroma_log2_weight_denom");
    for (int l = 0; l < (h.slice_type == SLICE_B ? 2 : 1); ++l) {
      int n = l ? h.num_ref_idx_l1_active : h.num_ref_idx_l0_active;
      for (int i = 0; i < n; ++i) {
        w.lflag[l][i] = static_cast<uint8_t>(br.get_bit());
        w.lw[l][i] = 1 << w.luma_log2;
        w.lo[l][i] = 0;
        if (w.lflag[l][i]) {
          w.lw[l][i] = br.get_se_range(-128, 127, "luma_weight");
          w.lo[l][i] = br.get_se_range(-128, 127, "luma_offset");
        }
        w.cflag[l][i] = static_cast<uint8_t>(br.get_bit());
        for (int c = 0; c < 2; ++c) {
          w.cw[l][i][c] = 1 << w.chroma_log2;
          w.co[l][i][c] = 0;
        }
        if (w.cflag[l][i])
          for (int c = 0; c < 2; ++c) {
            w.cw[l][i][c] = br.get_se_range(-128, 127, "chroma_weight");
            w.co[l][i][c] = br.get_se_range(-128, 127, "chroma_offset");
          }
      }
    }
  }
  if (nal_ref_idc) {
    if (nal_unit_type == NAL_IDR) {
      h.no_output_of_prior_pics = br.get_bit();
      h.long_term_reference = br.get_bit();
    } else {
      h.adaptive_ref_pic_marking = br.get_bit();
      if (h.adaptive_ref_pic_marking) {
        for (int guard = 0;; ++guard) {
          if (guard > 128) throw std::runtime_error("dec_ref_pic_marking too long");
          Mmco m;
          m.op = br.get_ue_max(6, "memory_management_control_operation");
          if (m.op == 0) break;
          if (m.op == 1 || m.op == 3) m.diff_minus1 = br.get_ue_max(65535, "difference_of_pic_nums_minus1");
          if (m.op == 2) m.long_term_pic_num = br.get_ue_max(31, "long_term_pic_num");
          if (m.op == 3 || m.op == 6) m.long_term_frame_idx = br.get_ue_max(15, "long_term_frame_idx");
          if (m.op == 4) m.max_long_term_frame_idx_plus1 = br.get_ue_max(16, "max_long_term_frame_idx_plus1");
          h.mmco.push_back(m);
        }
      }
    }
  }
  if (p.entropy_coding_mode && h.slice_type != SLICE_I) h.cabac_init_idc = br.get_ue_max(2, "cabac_init_idc");
  h.slice_qp_delta = br.get_se_range(-87, 77, "slice_qp_delta");
  h.qp = p.pic_init_qp + h.slice_qp_delta;
  if (p.deblocking_filter_control_present) {
    h.disable_deblocking_filter_idc = br.get_ue_max(2, "disable_deblocking_filter_idc");
    if (h.disable_deblocking_filter_idc != 1) {
      h.alpha_offset_div2 = br.get_se_range(-6, 6, "slice_alpha_c0_offset_div2");
      h.beta_offset_div2 = br.get_se_range(-6, 6, "slice_beta_offset_div2");
    }
  }
  return h;
}

int choose_level(int width_mbs, int height_mbs, double fps) {
  struct L {
    int idc;
    double max_mbps;
    int max_fs;
  };
  static const L lv[] = {{10, 1485, 99},        {11, 3000, 396},       {12, 6000, 396},
                         {13, 11880, 396},      {20, 11880, 396},      {21, 19800, 792},
                         {22, 20250, 1620},     {30, 40500, 1620},     {31, 108000, 3600},
                         {32, 216000, 5120},    {40, 245760, 8192},    {42, 522240, 8704},
                         {50, 589824, 22080},   {51, 983040, 36864},   {52, 2073600, 36864},
                         {60, 4177920, 139264}, {61, 8355840, 139264}, {62, 16711680, 139264}};
  int fs = width_mbs * height_mbs;
  double mbps = fs * fps;
  for (const L& l : lv) {
    double maxdim = std::sqrt(8.0 * l.max_fs);
    if (fs <= l.max_fs && mbps <= l.max_mbps && width_mbs <= maxdim && height_mbs <= maxdim) return l.idc;
  }
  return 62;
}

}  // namespace h264
}  // namespace mivc
