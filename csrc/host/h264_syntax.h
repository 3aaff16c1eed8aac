// H.264 high-level syntax: sequence/picture parameter sets and slice headers
// (clauses 7.3.2.1, 7.3.2.2, 7.3.3) -- writer for our encoder and parser for the
// independent decoder.
#pragma once
#include <cstdint>
#include <vector>

#include "../common/h264_mb.h"
#include "bitstream.h"

namespace mivc {
namespace h264 {

enum NalType { NAL_SLICE = 1, NAL_IDR = 5, NAL_SEI = 6, NAL_SPS = 7, NAL_PPS = 8, NAL_AUD = 9 };

struct SPS {
  int profile_idc = 66;
  int constraint_flags = 0xC0;  // constraint_set0..5 (bit7 = set0); 0xC0 = Constrained Baseline
  int level_idc = 40;
  int sps_id = 0;
  int chroma_format_idc = 1;
  int bit_depth_luma = 8, bit_depth_chroma = 8;
  int log2_max_frame_num = 16;
  int poc_type = 2;
  int log2_max_poc_lsb = 8;
  int max_num_ref_frames = 1;
  int gaps_allowed = 0;
  int width_mbs = 0, height_mbs = 0;
  int frame_mbs_only = 1;
  int direct_8x8_inference = 1;
  int crop_left = 0, crop_right = 0, crop_top = 0, crop_bottom = 0;  // in crop units (2 for 4:2:0)
  // VUI timing (optional)
  int vui_present = 0;
  uint32_t num_units_in_tick = 1, time_scale = 60;
  int fixed_frame_rate = 1;
  int max_num_reorder = 0;      // VUI bitstream_restriction max_num_reorder_frames (written)
  int vui_reorder_present = 0;  // parsed: bitstream_restriction present
  // poc type 1 fields
  int delta_pic_order_always_zero = 0;
  int offset_for_non_ref_pic = 0, offset_for_top_to_bottom = 0;
  std::vector<int> offset_for_ref_frame;
  // scaling matrices (7.3.2.1.1.1): seq_scaling_matrix_present_flag and the lists after fall-back
  // rule A, as weights in raster order: [0..5] 4x4 (Intra Y, Cb, Cr, Inter Y, Cb, Cr), [6..7] 8x8
  // (Intra Y, Inter Y).  Writing: sl_coded[i] says whether list i is sent (else it falls back).
  int scaling_present = 0;
  uint8_t sl4[6][16];
  uint8_t sl8[2][64];
  uint8_t sl_coded[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  SPS();
};

struct PPS {
  int pps_id = 0, sps_id = 0;
  int entropy_coding_mode = 0;  // 0 = CAVLC, 1 = CABAC
  int bottom_field_pic_order_present = 0;
  int num_ref_idx_l0_default = 1, num_ref_idx_l1_default = 1;
  int weighted_pred = 0, weighted_bipred_idc = 0;
  int pic_init_qp = 26, pic_init_qs = 26;
  int chroma_qp_index_offset = 0;
  int deblocking_filter_control_present = 1;
  int constrained_intra_pred = 0;
  int redundant_pic_cnt_present = 0;
  int transform_8x8_mode = 0;
  int second_chroma_qp_index_offset = 0;
  // pic_scaling_matrix_present_flag and the effective lists of the picture (fall-back rule B
  // onto the SPS lists, or the SPS lists when absent); layout as SPS::sl4 / sl8
  int scaling_present = 0;
  uint8_t sl4[6][16];
  uint8_t sl8[2][64];
  uint8_t sl_coded[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  PPS();
};

// flat scaling weights (16) in every list
void flat_scaling(uint8_t (*sl4)[16], uint8_t (*sl8)[64]);

// ref_pic_list_modification() operation (7.3.3.1)
struct RefMod {
  int idc;    // modification_of_pic_nums_idc 0..2
  int value;  // abs_diff_pic_num_minus1 or long_term_pic_num
};
// dec_ref_pic_marking() memory_management_control_operation (7.3.3.3)
struct Mmco {
  int op;
  int diff_minus1 = 0, long_term_pic_num = 0, long_term_frame_idx = 0, max_long_term_frame_idx_plus1 = 0;
};
// pred_weight_table() (7.3.3.2)
struct WeightTable {
  int luma_log2 = 0, chroma_log2 = 0;
  // [list][ref_idx]: luma weight, offset, chroma weight[2], offset[2]; flag = explicitly present
  int lw[2][32] = {}, lo[2][32] = {}, cw[2][32][2] = {}, co[2][32][2] = {};
  uint8_t lflag[2][32] = {}, cflag[2][32] = {};
};

struct SliceHeader {
  int nal_unit_type = NAL_IDR;
  int nal_ref_idc = 3;
  int first_mb = 0;
  int slice_type = SLICE_I;  // 0..2 (we write +5: all slices of the picture share the type)
  int pps_id = 0;
  int frame_num = 0;
  int idr_pic_id = 0;
  int poc_lsb = 0;
  int num_ref_idx_l0_active = 1;
  int num_ref_idx_override = 0;
  int slice_qp_delta = 0;
  int disable_deblocking_filter_idc = 0;
  int alpha_offset_div2 = 0, beta_offset_div2 = 0;
  int cabac_init_idc = 0;
  int no_output_of_prior_pics = 0, long_term_reference = 0;
  int adaptive_ref_pic_marking = 0;
  int num_ref_idx_l1_active = 1;
  int direct_spatial = 1;       // direct_spatial_mv_pred_flag (B)
  int poc_bottom_delta = 0;
  int delta_poc[2] = {0, 0};    // poc type 1
  std::vector<RefMod> mods[2];
  std::vector<Mmco> mmco;
  bool has_weights = false;
  WeightTable wt;
  // derived by the parser
  int qp = 26;
};

void write_sps(BitWriter& bw, const SPS& s);
void write_pps(BitWriter& bw, const PPS& p);
void write_slice_header(BitWriter& bw, const SliceHeader& h, const SPS& s, const PPS& p);

SPS parse_sps(BitReader& br);
PPS parse_pps(BitReader& br, const SPS* sps_table);
SliceHeader parse_slice_header(BitReader& br, int nal_unit_type, int nal_ref_idc, const SPS* sps_table,
                               const PPS* pps_table);

// Pick level_idc from picture size and frame rate (Table A-1 MaxFS / MaxMBPS).
int choose_level(int width_mbs, int height_mbs, double fps);

}  // namespace h264
}  // namespace mivc
