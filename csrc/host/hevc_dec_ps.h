// HEVC decoder internals: parameter sets, slice segment header, RPS and scaling lists
// (ITU-T H.265 clauses 7.3.2 - 7.3.7, 7.4.3 - 7.4.8, 8.3).  Private to hevc_dec*.cc.
#pragma once
#include <array>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "bitstream.h"
#include "hevc_dec.h"

namespace mivc {
namespace hevc {
namespace dec {

[[noreturn]] inline void fail(const std::string& what) { throw std::runtime_error("HEVC decode: " + what); }

// NAL unit types (Table 7-1)
enum NalType : int {
  TRAIL_N = 0, TRAIL_R = 1, TSA_N = 2, TSA_R = 3, STSA_N = 4, STSA_R = 5, RADL_N = 6, RADL_R = 7, RASL_N = 8,
  RASL_R = 9, BLA_W_LP = 16, BLA_W_RADL = 17, BLA_N_LP = 18, IDR_W_RADL = 19, IDR_N_LP = 20, CRA_NUT = 21,
  VPS_NUT = 32, SPS_NUT = 33, PPS_NUT = 34, AUD_NUT = 35, EOS_NUT = 36, EOB_NUT = 37, FD_NUT = 38,
};
inline bool is_irap(int t) { return t >= 16 && t <= 23; }
inline bool is_idr(int t) { return t == IDR_W_RADL || t == IDR_N_LP; }
inline bool is_bla(int t) { return t >= BLA_W_LP && t <= BLA_N_LP; }
inline bool is_rasl(int t) { return t == RASL_N || t == RASL_R; }
inline bool is_radl(int t) { return t == RADL_N || t == RADL_R; }
// sub-layer non-reference picture (7.4.2.2)
inline bool is_slnr(int t) { return t <= 14 && (t % 2) == 0; }

struct ShortTermRps {
  int num_neg = 0, num_pos = 0;
  int delta[32] = {};   // [0, num_neg): DeltaPocS0 (negative, decreasing), then DeltaPocS1
  uint8_t used[32] = {};
  int num_delta() const { return num_neg + num_pos; }
};

struct ScalingList {
  // ScalingFactor in the kScalingOff layout (raster, x + y * n)
  std::array<uint8_t, kScalingBytes> f{};
};

struct Sps {
  int id = -1;
  int chroma_format = 1;
  int W = 0, H = 0;
  int conf[4] = {0, 0, 0, 0};  // left, right, top, bottom (chroma units)
  int bit_depth = 8, bit_depth_c = 8;
  int log2_max_poc_lsb = 4;
  int max_dec_pic_buffering = 1, max_num_reorder = 0;
  int log2_min_cb = 3, log2_ctb = 4, log2_min_tb = 2, log2_max_tb = 5;
  int depth_inter = 0, depth_intra = 0;
  bool scaling_enabled = false;
  ScalingList scaling;  // SPS lists (or the defaults)
  bool amp = false, sao = false;
  bool pcm = false;
  int pcm_bd = 8, pcm_bd_c = 8, log2_min_pcm = 3, log2_max_pcm = 3;
  bool pcm_loop_filter_disabled = false;
  std::vector<ShortTermRps> st_rps;
  bool long_term = false;
  std::vector<int> lt_poc_lsb;
  std::vector<uint8_t> lt_used;
  bool tmvp = false, strong_intra = false;
  double fps = 0.0;
  // derived
  int wctb = 0, hctb = 0, min_cb_w = 0, min_cb_h = 0;
};

struct Pps {
  int id = -1, sps_id = 0;
  bool dependent_slices = false, output_flag_present = false;
  int extra_bits = 0;
  bool sign_hiding = false, cabac_init_present = false;
  int num_ref_l0 = 1, num_ref_l1 = 1;
  int init_qp = 26;
  bool constrained_intra = false, transform_skip = false;
  bool cu_qp_delta = false;
  int diff_cu_qp_delta_depth = 0;
  int cb_qp_off = 0, cr_qp_off = 0;
  bool slice_chroma_qp_offsets = false;
  bool weighted_pred = false, weighted_bipred = false;
  bool transquant_bypass = false;
  bool tiles = false, wpp = false;
  int tile_cols = 1, tile_rows = 1;
  bool uniform_spacing = true;
  std::vector<int> col_width, row_height;  // explicit sizes (CTBs), last inferred
  bool lf_across_tiles = true, lf_across_slices = false;
  bool deblock_override_enabled = false, deblock_disabled = false;
  int beta_off = 0, tc_off = 0;  // already x2
  bool scaling_present = false;
  ScalingList scaling;
  bool lists_modification = false;
  int log2_par_mrg_level = 2;
  bool slice_header_ext = false;
};

struct PredWeights {
  int log2_denom_y = 0, log2_denom_c = 0;
  int w[2][16][3] = {};  // [list][idx][component]
  int o[2][16][3] = {};  // offsets, not yet scaled by the bit depth
  bool flag[2][16][3] = {};
};

struct SliceHeader {
  bool first_slice_in_pic = true;
  bool no_output_of_prior_pics = false;
  int pps_id = 0;
  bool dependent = false;
  int segment_addr = 0;   // slice_segment_address (raster CTB)
  int slice_type = 2;     // 0 B, 1 P, 2 I
  bool pic_output = true;
  int poc_lsb = 0;
  ShortTermRps st;        // the RPS in use (SPS entry or explicit)
  int st_bits = 0;        // bits of st_ref_pic_set() in the slice header (unused: informative)
  // long-term entries of this slice (7-52)
  int num_lt = 0;
  int lt_poc[32] = {};          // PocLsbLt, or the full POC when msb_present
  bool lt_msb_present[32] = {};
  bool lt_used[32] = {};
  bool tmvp = false;
  bool sao_luma = false, sao_chroma = false;
  int num_ref[2] = {0, 0};
  bool list_mod[2] = {false, false};
  int list_entry[2][16] = {};
  bool mvd_l1_zero = false, cabac_init = false, col_from_l0 = true;
  int col_ref_idx = 0;
  PredWeights pw;
  bool weighted = false;
  int max_merge = 5;
  int qp_delta = 0, cb_qp_off = 0, cr_qp_off = 0;
  bool deblock_disabled = false;
  int beta_off = 0, tc_off = 0;  // x2
  bool lf_across_slices = false;
  std::vector<uint32_t> entry_points;
  size_t data_byte = 0;   // rbsp byte offset of slice_segment_data() (after the 2-byte NAL header)
};

// ---------------------------------------------------------------- parsing
void parse_sps(BitReader& br, Sps& s);
void parse_pps(BitReader& br, Pps& p, const Sps* sps_by_id[16]);
// default ScalingFactor (Table 7-5 / 7-6) and the scaling_list_data() parser
void default_scaling(ScalingList& sl);
void parse_scaling_list_data(BitReader& br, ScalingList& sl);
void parse_st_rps(BitReader& br, int idx, int num_in_sps, const std::vector<ShortTermRps>& sets, ShortTermRps& out);
// slice header up to byte_alignment(); `prev` holds the independent header a dependent
// slice segment copies its fields from
void parse_slice_header(BitReader& br, int nal_type, const Sps* const* sps_tab, const Pps* const* pps_tab,
                        const SliceHeader* prev, SliceHeader& sh, int* num_pic_total_curr);

}  // namespace dec
}  // namespace hevc
}  // namespace mivc
