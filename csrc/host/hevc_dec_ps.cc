// HEVC decoder: parameter sets, scaling lists, reference picture sets and the slice
// segment header (ITU-T H.265 7.3.2 - 7.3.7 syntax, 7.4 semantics).
#include "hevc_dec_ps.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>

namespace mivc {
namespace hevc {
namespace dec {

namespace {

int ceil_log2(int v) {
  int n = 0;
  while ((1 << n) < v) ++n;
  return n;
}

// profile_tier_level(1, maxNumSubLayersMinus1) (7.3.3): nothing in it affects decoding
void skip_ptl(BitReader& br, int max_sub_layers_minus1) {
  br.get(8);
  br.get(32);
  br.get(32);
  br.get(16);
  br.get(8);  // general_level_idc
  int pp[8] = {}, lp[8] = {};
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

// Table 7-6 default 8x8 lists, in up-right diagonal scan order
const uint8_t kDefIntra8[64] = {16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 17, 16, 17, 16, 17, 18,
                                17, 18, 18, 17, 18, 21, 19, 20, 21, 20, 19, 21, 24, 22, 22, 24,
                                24, 22, 22, 24, 25, 25, 27, 30, 27, 25, 25, 29, 31, 35, 35, 31,
                                29, 36, 41, 44, 41, 36, 47, 54, 54, 47, 65, 70, 65, 88, 88, 115};
const uint8_t kDefInter8[64] = {16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 17, 17, 17, 17, 17, 18,
                                18, 18, 18, 18, 18, 20, 20, 20, 20, 20, 20, 20, 24, 24, 24, 24,
                                24, 24, 24, 24, 25, 25, 25, 25, 25, 25, 25, 28, 28, 28, 28, 28,
                                28, 33, 33, 33, 33, 33, 41, 41, 41, 41, 54, 54, 54, 71, 71, 91};

// ScalingList[sizeId][matrixId][i] (coded order) + DC -> ScalingFactor (7.4.5)
struct ListData {
  uint8_t c[4][6][64];
  uint8_t dc[4][6];
};

void to_factor(const ListData& L, ScalingList& sl) {
  for (int sid = 0; sid < 4; ++sid)
    for (int m = 0; m < 6; ++m) {
      const int n = 4 << sid;
      uint8_t* f = sl.f.data() + kScalingOff[sid] + m * n * n;
      const int coefs = sid == 0 ? 16 : 64, l2 = sid == 0 ? 2 : 3;
      const int rep = n >> l2;  // 1, 1, 2, 4
      // 32x32 chroma lists (matrixId 1, 2, 4, 5) do not exist for 4:2:0: copy the luma ones
      const int mm = (sid == 3 && m % 3) ? (m < 3 ? 0 : 3) : m;
      for (int i = 0; i < coefs; ++i) {
        const int p = scan_pos(0, l2, i);
        const int x = p & 255, y = p >> 8;
        for (int dy = 0; dy < rep; ++dy)
          for (int dx = 0; dx < rep; ++dx) f[(y * rep + dy) * n + x * rep + dx] = L.c[sid][mm][i];
      }
      if (sid >= 2) f[0] = L.dc[sid][mm];
    }
}

void default_lists(ListData& L) {
  for (int m = 0; m < 6; ++m) {
    std::memset(L.c[0][m], 16, 16);
    for (int sid = 1; sid < 4; ++sid) {
      std::memcpy(L.c[sid][m], m < 3 ? kDefIntra8 : kDefInter8, 64);
      L.dc[sid][m] = 16;
    }
    L.dc[0][m] = L.dc[1][m] = 16;
  }
}

}  // namespace

void default_scaling(ScalingList& sl) {
  ListData L;
  default_lists(L);
  to_factor(L, sl);
}

// 7.3.4 scaling_list_data()
void parse_scaling_list_data(BitReader& br, ScalingList& sl) {
  ListData L;
  default_lists(L);
  for (int sid = 0; sid < 4; ++sid) {
    const int coefs = std::min(64, 1 << (4 + (sid << 1)));
    for (int m = 0; m < 6; m += (sid == 3) ? 3 : 1) {
      if (!br.get(1)) {  // scaling_list_pred_mode_flag = 0: copy (or default)
        const int d = br.get_ue_max(static_cast<uint32_t>(m / (sid == 3 ? 3 : 1)), "scaling_list_pred_matrix_id_delta") *
                      (sid == 3 ? 3 : 1);
        if (d == 0) {
          if (sid == 0) std::memset(L.c[0][m], 16, 16);
          else std::memcpy(L.c[sid][m], m < 3 ? kDefIntra8 : kDefInter8, 64);
          L.dc[sid][m] = 16;
        } else {
          std::memcpy(L.c[sid][m], L.c[sid][m - d], 64);
          L.dc[sid][m] = L.dc[sid][m - d];
        }
      } else {
        int next = 8;
        if (sid > 1) {
          const int dc = br.get_se_range(-7, 247, "scaling_list_dc_coef_minus8") + 8;
          next = dc;
          L.dc[sid][m] = static_cast<uint8_t>(dc);
        }
        for (int i = 0; i < coefs; ++i) {
          const int dlt = br.get_se_range(-128, 127, "scaling_list_delta_coef");
          next = (next + dlt + 256) % 256;
          if (next == 0) fail("scaling list entry 0");
          L.c[sid][m][i] = static_cast<uint8_t>(next);
        }
        if (sid <= 1) L.dc[sid][m] = L.c[sid][m][0];
      }
    }
  }
  to_factor(L, sl);
}

// 7.3.7 st_ref_pic_set(stRpsIdx) + 7.4.8 derivation
void parse_st_rps(BitReader& br, int idx, int num_in_sps, const std::vector<ShortTermRps>& sets, ShortTermRps& out) {
  out = ShortTermRps();
  bool inter = false;
  if (idx != 0) inter = br.get(1);
  if (inter) {
    int delta_idx = 1;
    if (idx == num_in_sps) delta_idx = br.get_ue_max(static_cast<uint32_t>(idx - 1), "delta_idx_minus1") + 1;
    const ShortTermRps& ref = sets[idx - delta_idx];
    const int sign = br.get(1);
    const int abs_delta = br.get_ue_max(32767, "abs_delta_rps_minus1") + 1;
    const int delta_rps = (1 - 2 * sign) * abs_delta;
    const int nd = ref.num_delta();
    uint8_t used[33], use_delta[33];
    for (int j = 0; j <= nd; ++j) {
      used[j] = static_cast<uint8_t>(br.get(1));
      use_delta[j] = used[j] ? 1 : static_cast<uint8_t>(br.get(1));
    }
    auto S0 = [&](int j) { return ref.delta[j]; };
    auto S1 = [&](int j) { return ref.delta[ref.num_neg + j]; };
    int d0[32], d1[32];
    uint8_t u0[32], u1[32];
    int i = 0;
    for (int j = ref.num_pos - 1; j >= 0; --j) {  // (7-61)
      const int dp = S1(j) + delta_rps;
      if (dp < 0 && use_delta[ref.num_neg + j]) {
        if (i >= 16) fail("RPS too large");
        d0[i] = dp;
        u0[i++] = used[ref.num_neg + j];
      }
    }
    if (delta_rps < 0 && use_delta[nd]) {
      if (i >= 16) fail("RPS too large");
      d0[i] = delta_rps;
      u0[i++] = used[nd];
    }
    for (int j = 0; j < ref.num_neg; ++j) {
      const int dp = S0(j) + delta_rps;
      if (dp < 0 && use_delta[j]) {
        if (i >= 16) fail("RPS too large");
        d0[i] = dp;
        u0[i++] = used[j];
      }
    }
    const int nneg = i;
    i = 0;
    for (int j = ref.num_neg - 1; j >= 0; --j) {  // (7-62)
      const int dp = S0(j) + delta_rps;
      if (dp > 0 && use_delta[j]) {
        if (i >= 16) fail("RPS too large");
        d1[i] = dp;
        u1[i++] = used[j];
      }
    }
    if (delta_rps > 0 && use_delta[nd]) {
      if (i >= 16) fail("RPS too large");
      d1[i] = delta_rps;
      u1[i++] = used[nd];
    }
    for (int j = 0; j < ref.num_pos; ++j) {
      const int dp = S1(j) + delta_rps;
      if (dp > 0 && use_delta[ref.num_neg + j]) {
        if (i >= 16) fail("RPS too large");
        d1[i] = dp;
        u1[i++] = used[ref.num_neg + j];
      }
    }
    out.num_neg = nneg;
    out.num_pos = i;
    for (int k = 0; k < nneg; ++k) {
      out.delta[k] = d0[k];
      out.used[k] = u0[k];
    }
    for (int k = 0; k < i; ++k) {
      out.delta[nneg + k] = d1[k];
      out.used[nneg + k] = u1[k];
    }
  } else {
    const uint32_t nneg = br.get_ue(), npos = br.get_ue();
    if (nneg > 16 || npos > 16 || nneg + npos > 16) fail("num_negative/positive_pics out of range");
    out.num_neg = static_cast<int>(nneg);
    out.num_pos = static_cast<int>(npos);
    int poc = 0;
    for (int k = 0; k < out.num_neg; ++k) {
      poc -= br.get_ue_max(32767, "delta_poc_s0_minus1") + 1;
      out.delta[k] = poc;
      out.used[k] = static_cast<uint8_t>(br.get(1));
    }
    poc = 0;
    for (int k = 0; k < out.num_pos; ++k) {
      poc += br.get_ue_max(32767, "delta_poc_s1_minus1") + 1;
      out.delta[out.num_neg + k] = poc;
      out.used[out.num_neg + k] = static_cast<uint8_t>(br.get(1));
    }
  }
}

// E.2.1 vui_parameters(): only the timing information is kept
static void parse_vui(BitReader& br, Sps& s, int max_sub_layers_minus1) {
  if (br.get(1)) {  // aspect_ratio_info_present_flag
    if (br.get(8) == 255) {
      br.get(16);
      br.get(16);
    }
  }
  if (br.get(1)) br.get(1);  // overscan
  if (br.get(1)) {           // video_signal_type_present_flag
    br.get(3);
    br.get(1);
    if (br.get(1)) br.get(24);
  }
  if (br.get(1)) {  // chroma_loc_info_present_flag
    br.get_ue();
    br.get_ue();
  }
  br.get(1);  // neutral_chroma_indication_flag
  br.get(1);  // field_seq_flag
  br.get(1);  // frame_field_info_present_flag
  if (br.get(1)) {  // default_display_window_flag
    for (int i = 0; i < 4; ++i) br.get_ue();
  }
  if (br.get(1)) {  // vui_timing_info_present_flag
    const uint32_t num_units = br.get(32), time_scale = br.get(32);
    if (num_units) s.fps = static_cast<double>(time_scale) / num_units;
  }
  (void)max_sub_layers_minus1;  // HRD and bitstream restrictions follow; not needed
}

// 7.3.2.2 seq_parameter_set_rbsp()
void parse_sps(BitReader& br, Sps& s) {
  s = Sps();
  br.get(4);  // sps_video_parameter_set_id
  const int msl = br.get(3);
  if (msl > 6) fail("sps_max_sub_layers_minus1 out of range");
  br.get(1);
  skip_ptl(br, msl);
  const uint32_t id = br.get_ue();
  if (id > 15) fail("sps id out of range");
  s.id = static_cast<int>(id);
  s.chroma_format = br.get_ue_max(3, "chroma_format_idc");
  if (s.chroma_format != 1) fail("only 4:2:0 (Main / Main 10) is supported");
  s.W = br.get_ue_max(1u << 16, "pic_width_in_luma_samples");
  s.H = br.get_ue_max(1u << 16, "pic_height_in_luma_samples");
  if (br.get(1))
    for (int i = 0; i < 4; ++i) s.conf[i] = br.get_ue_max(1u << 16, "conf_win_offset");
  s.bit_depth = 8 + br.get_ue_max(8, "bit_depth_luma_minus8");
  s.bit_depth_c = 8 + br.get_ue_max(8, "bit_depth_chroma_minus8");
  if (s.bit_depth > 10 || s.bit_depth_c > 10) fail("bit depth above 10 (Main 10) is not supported");
  s.log2_max_poc_lsb = br.get_ue_max(12, "log2_max_pic_order_cnt_lsb_minus4") + 4;
  const int sub = br.get(1);
  for (int i = sub ? 0 : msl; i <= msl; ++i) {
    s.max_dec_pic_buffering = br.get_ue_max(15, "sps_max_dec_pic_buffering_minus1") + 1;
    s.max_num_reorder = br.get_ue_max(15, "sps_max_num_reorder_pics");
    br.get_ue();
  }
  s.log2_min_cb = br.get_ue_max(3, "log2_min_luma_coding_block_size_minus3") + 3;
  s.log2_ctb = s.log2_min_cb + br.get_ue_max(3, "log2_diff_max_min_luma_coding_block_size");
  s.log2_min_tb = br.get_ue_max(3, "log2_min_luma_transform_block_size_minus2") + 2;
  s.log2_max_tb = s.log2_min_tb + br.get_ue_max(3, "log2_diff_max_min_luma_transform_block_size");
  if (s.log2_ctb < 4 || s.log2_ctb > 6) fail("CTB size must be 16, 32 or 64");
  if (s.log2_min_cb > s.log2_ctb || s.log2_max_tb > 5 || s.log2_min_tb >= s.log2_min_cb || s.log2_max_tb > s.log2_ctb)
    fail("coding / transform block sizes out of range");
  s.depth_inter = br.get_ue_max(4, "max_transform_hierarchy_depth_inter");
  s.depth_intra = br.get_ue_max(4, "max_transform_hierarchy_depth_intra");
  if (s.depth_inter > s.log2_ctb - s.log2_min_tb || s.depth_intra > s.log2_ctb - s.log2_min_tb)
    fail("max_transform_hierarchy_depth out of range");
  s.scaling_enabled = br.get(1);
  default_scaling(s.scaling);
  if (s.scaling_enabled && br.get(1)) parse_scaling_list_data(br, s.scaling);
  s.amp = br.get(1);
  s.sao = br.get(1);
  s.pcm = br.get(1);
  if (s.pcm) {
    s.pcm_bd = static_cast<int>(br.get(4)) + 1;
    s.pcm_bd_c = static_cast<int>(br.get(4)) + 1;
    s.log2_min_pcm = br.get_ue_max(2, "log2_min_pcm_luma_coding_block_size_minus3") + 3;
    s.log2_max_pcm = s.log2_min_pcm + br.get_ue_max(2, "log2_diff_max_min_pcm_luma_coding_block_size");
    s.pcm_loop_filter_disabled = br.get(1);
    if (s.pcm_bd > s.bit_depth || s.pcm_bd_c > s.bit_depth_c || s.log2_max_pcm > std::min(s.log2_ctb, 5))
      fail("PCM parameters out of range");
  }
  const uint32_t nst = br.get_ue();
  if (nst > 64) fail("num_short_term_ref_pic_sets out of range");
  s.st_rps.resize(nst);
  for (uint32_t i = 0; i < nst; ++i) parse_st_rps(br, static_cast<int>(i), static_cast<int>(nst), s.st_rps, s.st_rps[i]);
  s.long_term = br.get(1);
  if (s.long_term) {
    const uint32_t nlt = br.get_ue();
    if (nlt > 32) fail("num_long_term_ref_pics_sps out of range");
    for (uint32_t i = 0; i < nlt; ++i) {
      s.lt_poc_lsb.push_back(static_cast<int>(br.get(s.log2_max_poc_lsb)));
      s.lt_used.push_back(static_cast<uint8_t>(br.get(1)));
    }
  }
  s.tmvp = br.get(1);
  s.strong_intra = br.get(1);
  if (br.get(1)) {  // vui_parameters_present_flag
    try {
      parse_vui(br, s, msl);
    } catch (const std::exception&) {
      // a truncated or unusual VUI does not affect decoding
    }
  }
  const int ctb = 1 << s.log2_ctb, mcb = 1 << s.log2_min_cb;
  if (s.W <= 0 || s.H <= 0 || s.W % mcb || s.H % mcb) fail("picture size must be a multiple of MinCbSizeY");
  if (s.W > 16888 || s.H > 16888) fail("picture too large");
  s.wctb = (s.W + ctb - 1) / ctb;
  s.hctb = (s.H + ctb - 1) / ctb;
  s.min_cb_w = s.W / mcb;
  s.min_cb_h = s.H / mcb;
}

// 7.3.2.3 pic_parameter_set_rbsp()
void parse_pps(BitReader& br, Pps& p, const Sps* sps_by_id[16]) {
  p = Pps();
  const uint32_t id = br.get_ue(), sid = br.get_ue();
  if (id > 63 || sid > 15) fail("pps / sps id out of range");
  p.id = static_cast<int>(id);
  p.sps_id = static_cast<int>(sid);
  p.dependent_slices = br.get(1);
  p.output_flag_present = br.get(1);
  p.extra_bits = br.get(3);
  p.sign_hiding = br.get(1);
  p.cabac_init_present = br.get(1);
  {
    const uint32_t n0 = br.get_ue(), n1 = br.get_ue();  // bounded before the +1 (no wrap)
    if (n0 > 14 || n1 > 14) fail("num_ref_idx_default_active out of range");
    p.num_ref_l0 = static_cast<int>(n0) + 1;
    p.num_ref_l1 = static_cast<int>(n1) + 1;
  }
  p.init_qp = 26 + br.get_se_range(-38, 25, "init_qp_minus26");
  p.constrained_intra = br.get(1);
  p.transform_skip = br.get(1);
  p.cu_qp_delta = br.get(1);
  if (p.cu_qp_delta) p.diff_cu_qp_delta_depth = br.get_ue_max(3, "diff_cu_qp_delta_depth");
  p.cb_qp_off = br.get_se_range(-12, 12, "pps_cb_qp_offset");
  p.cr_qp_off = br.get_se_range(-12, 12, "pps_cr_qp_offset");
  p.slice_chroma_qp_offsets = br.get(1);
  p.weighted_pred = br.get(1);
  p.weighted_bipred = br.get(1);
  p.transquant_bypass = br.get(1);
  p.tiles = br.get(1);
  p.wpp = br.get(1);
  if (p.tiles) {
    p.tile_cols = br.get_ue_max(19, "num_tile_columns_minus1") + 1;
    p.tile_rows = br.get_ue_max(21, "num_tile_rows_minus1") + 1;
    p.uniform_spacing = br.get(1);
    if (!p.uniform_spacing) {
      // a CTB count is < 2^11 for any picture the SPS accepts; build_tiles checks the sum
      for (int i = 0; i < p.tile_cols - 1; ++i) p.col_width.push_back(br.get_ue_max(1u << 11, "column_width_minus1") + 1);
      for (int i = 0; i < p.tile_rows - 1; ++i) p.row_height.push_back(br.get_ue_max(1u << 11, "row_height_minus1") + 1);
    }
    p.lf_across_tiles = br.get(1);
  }
  p.lf_across_slices = br.get(1);
  if (br.get(1)) {  // deblocking_filter_control_present_flag
    p.deblock_override_enabled = br.get(1);
    p.deblock_disabled = br.get(1);
    if (!p.deblock_disabled) {
      p.beta_off = br.get_se_range(-6, 6, "pps_beta_offset_div2") * 2;
      p.tc_off = br.get_se_range(-6, 6, "pps_tc_offset_div2") * 2;
    }
  }
  p.scaling_present = br.get(1);
  if (p.scaling_present) parse_scaling_list_data(br, p.scaling);
  p.lists_modification = br.get(1);
  p.log2_par_mrg_level = br.get_ue_max(4, "log2_parallel_merge_level_minus2") + 2;
  p.slice_header_ext = br.get(1);
  // pps_extension_present_flag: range / multilayer / SCC extensions are outside Main
  if (br.get(1)) {
    const int range = br.get(1), multilayer = br.get(1), ext3d = br.get(1), scc = br.get(1);
    if (range || multilayer || ext3d || scc) fail("PPS extensions (RExt / SCC / multilayer) are not supported");
  }
  const Sps* s = sps_by_id[p.sps_id];
  if (s) {
    if (p.log2_par_mrg_level > s->log2_ctb) fail("log2_parallel_merge_level out of range");
    if (p.cu_qp_delta && p.diff_cu_qp_delta_depth > s->log2_ctb - s->log2_min_cb) fail("diff_cu_qp_delta_depth out of range");
  }
}

// 7.3.6 slice_segment_header()
void parse_slice_header(BitReader& br, int nal_type, const Sps* const* sps_tab, const Pps* const* pps_tab,
                        const SliceHeader* prev, SliceHeader& sh, int* num_pic_total_curr) {
  SliceHeader h;
  h.first_slice_in_pic = br.get(1);
  if (nal_type >= BLA_W_LP && nal_type <= 23) h.no_output_of_prior_pics = br.get(1);
  const uint32_t pid = br.get_ue();
  if (pid > 63 || !pps_tab[pid]) fail("slice refers to a missing PPS");
  h.pps_id = static_cast<int>(pid);
  const Pps& pps = *pps_tab[pid];
  if (!sps_tab[pps.sps_id]) fail("PPS refers to a missing SPS");
  const Sps& sps = *sps_tab[pps.sps_id];
  const int nctb = sps.wctb * sps.hctb;
  if (!h.first_slice_in_pic) {
    if (pps.dependent_slices) h.dependent = br.get(1);
    h.segment_addr = static_cast<int>(br.get(ceil_log2(nctb)));
    if (h.segment_addr >= nctb) fail("slice_segment_address out of range");
  }
  if (h.dependent) {
    if (!prev) fail("dependent slice segment without a preceding slice");
    const int addr = h.segment_addr;
    const bool first = h.first_slice_in_pic;
    h = *prev;
    h.first_slice_in_pic = first;
    h.dependent = true;
    h.segment_addr = addr;
    h.entry_points.clear();
  } else {
    for (int i = 0; i < pps.extra_bits; ++i) br.get(1);
    const uint32_t st = br.get_ue();
    if (st > 2) fail("slice_type out of range");
    h.slice_type = static_cast<int>(st);
    if (is_irap(nal_type) && h.slice_type != 2) fail("IRAP picture with a P / B slice");
    if (pps.output_flag_present) h.pic_output = br.get(1);
    int npc = 0;
    if (!is_idr(nal_type)) {
      h.poc_lsb = static_cast<int>(br.get(sps.log2_max_poc_lsb));
      if (br.get(1)) {  // short_term_ref_pic_set_sps_flag
        if (sps.st_rps.empty()) fail("short_term_ref_pic_set_sps_flag without SPS sets");
        int idx = 0;
        if (sps.st_rps.size() > 1) idx = static_cast<int>(br.get(ceil_log2(static_cast<int>(sps.st_rps.size()))));
        if (idx >= static_cast<int>(sps.st_rps.size())) fail("short_term_ref_pic_set_idx out of range");
        h.st = sps.st_rps[idx];
      } else {
        const size_t b0 = br.pos();
        parse_st_rps(br, static_cast<int>(sps.st_rps.size()), static_cast<int>(sps.st_rps.size()), sps.st_rps, h.st);
        h.st_bits = static_cast<int>(br.pos() - b0);
      }
      if (sps.long_term) {
        int nsps = 0;
        if (!sps.lt_poc_lsb.empty()) nsps = br.get_ue_max(32, "num_long_term_sps");
        const int npics = br.get_ue_max(32, "num_long_term_pics");
        if (nsps > static_cast<int>(sps.lt_poc_lsb.size()) || nsps + npics > 32) fail("long-term picture count out of range");
        h.num_lt = nsps + npics;
        int msb_cycle_prev = 0;
        for (int i = 0; i < h.num_lt; ++i) {
          int lsb, used;
          if (i < nsps) {
            int k = 0;
            if (sps.lt_poc_lsb.size() > 1) k = static_cast<int>(br.get(ceil_log2(static_cast<int>(sps.lt_poc_lsb.size()))));
            if (k >= static_cast<int>(sps.lt_poc_lsb.size())) fail("lt_idx_sps out of range");
            lsb = sps.lt_poc_lsb[k];
            used = sps.lt_used[k];
          } else {
            lsb = static_cast<int>(br.get(sps.log2_max_poc_lsb));
            used = br.get(1);
          }
          h.lt_used[i] = used != 0;
          h.lt_msb_present[i] = br.get(1);
          int cyc = 0;
          // bounded so that the accumulated cycle (<= 32 entries) times MaxPicOrderCntLsb stays below 2^30
          if (h.lt_msb_present[i]) cyc = br.get_ue_max((1u << (30 - sps.log2_max_poc_lsb)) / 32, "delta_poc_msb_cycle_lt");
          // DeltaPocMsbCycleLt (7-52): accumulates within the SPS entries and within the slice entries
          const int acc = (i == 0 || i == nsps) ? cyc : cyc + msb_cycle_prev;
          msb_cycle_prev = acc;
          h.lt_poc[i] = lsb;
          if (h.lt_msb_present[i]) h.lt_poc[i] = lsb - acc * (1 << sps.log2_max_poc_lsb);  // + PicOrderCntVal - lsb(cur) later
        }
      }
      if (sps.tmvp) h.tmvp = br.get(1);
    }
    for (int i = 0; i < h.st.num_delta(); ++i) npc += h.st.used[i];
    for (int i = 0; i < h.num_lt; ++i) npc += h.lt_used[i];
    *num_pic_total_curr = npc;
    if (sps.sao) {
      h.sao_luma = br.get(1);
      h.sao_chroma = br.get(1);
    }
    if (h.slice_type != 2) {
      h.num_ref[0] = pps.num_ref_l0;
      h.num_ref[1] = h.slice_type == 0 ? pps.num_ref_l1 : 0;
      if (br.get(1)) {  // num_ref_idx_active_override_flag
        // num_ref_idx_lX_active_minus1 is 0..14 (7.4.7.1): bound the raw ue(v) before the +1 so
        // a huge value cannot wrap into a zero or negative count
        const uint32_t n0 = br.get_ue();
        if (n0 > 14) fail("num_ref_idx_l0_active_minus1 out of range");
        h.num_ref[0] = static_cast<int>(n0) + 1;
        if (h.slice_type == 0) {
          const uint32_t n1 = br.get_ue();
          if (n1 > 14) fail("num_ref_idx_l1_active_minus1 out of range");
          h.num_ref[1] = static_cast<int>(n1) + 1;
        }
      }
      if (h.num_ref[0] < 1 || h.num_ref[0] > 15 || h.num_ref[1] < 0 || h.num_ref[1] > 15)
        fail("num_ref_idx_active out of range");
      if (npc == 0) fail("P / B slice without reference pictures");
      if (pps.lists_modification && npc > 1) {
        const int bits = ceil_log2(npc);
        for (int l = 0; l < (h.slice_type == 0 ? 2 : 1); ++l) {
          h.list_mod[l] = br.get(1);
          if (h.list_mod[l])
            for (int i = 0; i < h.num_ref[l]; ++i) {
              h.list_entry[l][i] = static_cast<int>(br.get(bits));
              if (h.list_entry[l][i] >= npc) fail("list_entry out of range");
            }
        }
      }
      if (h.slice_type == 0) h.mvd_l1_zero = br.get(1);
      if (pps.cabac_init_present) h.cabac_init = br.get(1);
      if (h.tmvp) {
        h.col_from_l0 = true;
        if (h.slice_type == 0) h.col_from_l0 = br.get(1);
        const int nr = h.num_ref[h.col_from_l0 ? 0 : 1];
        if (nr > 1) h.col_ref_idx = br.get_ue_max(static_cast<uint32_t>(nr - 1), "collocated_ref_idx");
      }
      h.weighted = (pps.weighted_pred && h.slice_type == 1) || (pps.weighted_bipred && h.slice_type == 0);
      if (h.weighted) {  // 7.3.6.3 pred_weight_table()
        PredWeights& w = h.pw;
        w.log2_denom_y = br.get_ue_max(7, "luma_log2_weight_denom");
        w.log2_denom_c = w.log2_denom_y + br.get_se_range(-7, 7, "delta_chroma_log2_weight_denom");
        if (w.log2_denom_c < 0 || w.log2_denom_c > 7) fail("ChromaLog2WeightDenom out of range");
        for (int l = 0; l < (h.slice_type == 0 ? 2 : 1); ++l) {
          bool lf[16], cf[16];
          for (int i = 0; i < h.num_ref[l]; ++i) lf[i] = br.get(1);
          for (int i = 0; i < h.num_ref[l]; ++i) cf[i] = br.get(1);
          for (int i = 0; i < h.num_ref[l]; ++i) {
            w.w[l][i][0] = 1 << w.log2_denom_y;
            w.o[l][i][0] = 0;
            w.flag[l][i][0] = lf[i];
            if (lf[i]) {
              const int dw = br.get_se_range(-128, 127, "delta_luma_weight");
              const int off = br.get_se_range(-128, 127, "luma_offset");
              w.w[l][i][0] += dw;
              w.o[l][i][0] = off;
            }
            for (int j = 1; j < 3; ++j) {
              w.w[l][i][j] = 1 << w.log2_denom_c;
              w.o[l][i][j] = 0;
              w.flag[l][i][j] = cf[i];
            }
            if (cf[i]) {
              for (int j = 1; j < 3; ++j) {
                const int dw = br.get_se_range(-128, 127, "delta_chroma_weight");
                const int doff = br.get_se_range(-512, 511, "delta_chroma_offset");
                const int cw = (1 << w.log2_denom_c) + dw;
                w.w[l][i][j] = cw;
                // (7-56) ChromaOffset, wpOffsetHalfRangeC = 128
                const int o = (128 - ((128 * cw) >> w.log2_denom_c)) + doff;
                w.o[l][i][j] = o < -128 ? -128 : (o > 127 ? 127 : o);
              }
            }
          }
        }
      }
      const uint32_t fm = br.get_ue();
      if (fm > 4) fail("five_minus_max_num_merge_cand out of range");
      h.max_merge = 5 - static_cast<int>(fm);
    }
    h.qp_delta = br.get_se_range(-128, 128, "slice_qp_delta");
    if (pps.slice_chroma_qp_offsets) {
      h.cb_qp_off = br.get_se_range(-12, 12, "slice_cb_qp_offset");
      h.cr_qp_off = br.get_se_range(-12, 12, "slice_cr_qp_offset");
    }
    h.deblock_disabled = pps.deblock_disabled;
    h.beta_off = pps.beta_off;
    h.tc_off = pps.tc_off;
    bool override_flag = false;
    if (pps.deblock_override_enabled) override_flag = br.get(1);
    if (override_flag) {
      h.deblock_disabled = br.get(1);
      if (!h.deblock_disabled) {
        h.beta_off = br.get_se_range(-6, 6, "slice_beta_offset_div2") * 2;
        h.tc_off = br.get_se_range(-6, 6, "slice_tc_offset_div2") * 2;
      }
    }
    h.lf_across_slices = pps.lf_across_slices;
    if (pps.lf_across_slices && (h.sao_luma || h.sao_chroma || !h.deblock_disabled)) h.lf_across_slices = br.get(1);
  }
  if (pps.tiles || pps.wpp) {
    const uint32_t ne = br.get_ue();
    if (ne > static_cast<uint32_t>(nctb)) fail("num_entry_point_offsets out of range");
    if (ne > 0) {
      const int len = br.get_ue_max(31, "offset_len_minus1") + 1;
      for (uint32_t k = 0; k < ne; ++k) h.entry_points.push_back(br.get(len) + 1);
    }
  }
  if (pps.slice_header_ext) {
    const uint32_t n = br.get_ue();
    if (n > 256) fail("slice_segment_header_extension_length out of range");
    for (uint32_t i = 0; i < n; ++i) br.get(8);
  }
  if (br.get(1) != 1) fail("slice header byte_alignment()");
  while (!br.byte_aligned())
    if (br.get(1)) fail("slice header alignment bit");
  h.data_byte = br.pos() / 8;
  sh = h;
}

}  // namespace dec
}  // namespace hevc
}  // namespace mivc

namespace mivc {
namespace hevc {

namespace {
struct HNal {
  size_t start, end;  // byte range in the input incl. start code
  int type;
  bool first_slice;   // VCL: first_slice_segment_in_pic_flag
};
std::vector<HNal> scan_nals(const uint8_t* p, size_t n) {
  std::vector<HNal> out;
  const std::vector<NalUnit> nals = parse_annexb(p, n, false);
  for (const NalUnit& u : nals) {
    const size_t hdr = u.offset + (p[u.offset + 2] == 1 ? 3 : 4);
    if (hdr + 2 >= u.offset + u.size) continue;
    HNal h;
    h.start = u.offset;
    h.end = u.offset + u.size;
    h.type = (p[hdr] >> 1) & 63;
    h.first_slice = h.type <= 31 && (p[hdr + 2] & 0x80);
    out.push_back(h);
  }
  return out;
}
}  // namespace

HevcStreamInfo hevc_stream_info(const uint8_t* p, size_t n) {
  HevcStreamInfo si;
  const std::vector<NalUnit> nals = parse_annexb(p, n);
  bool have_sps = false;
  for (const NalUnit& u : nals) {
    const size_t hdr = u.offset + (p[u.offset + 2] == 1 ? 3 : 4);
    const int type = (p[hdr] >> 1) & 63;
    if (u.rbsp.size() < 2) continue;
    if (type == dec::SPS_NUT && !have_sps) {
      BitReader br(u.rbsp.data() + 1, u.rbsp.size() - 1);
      dec::Sps s;
      dec::parse_sps(br, s);
      si.width = s.W - 2 * (s.conf[0] + s.conf[1]);
      si.height = s.H - 2 * (s.conf[2] + s.conf[3]);
      si.bit_depth = s.bit_depth;
      si.fps = s.fps;
      have_sps = true;
    } else if (type <= 21 && !(type >= 10 && type <= 15) && (u.rbsp[1] & 0x80)) {
      ++si.pictures;
      if (dec::is_irap(type)) ++si.irap;
    }
  }
  return si;
}

// IRAP access units that can start an independently decodable piece: IDR, BLA, or a CRA
// with no RASL picture following it (its leading pictures would reference the previous
// piece and be dropped, as ffmpeg's segment muxer + decoder would lose them)
std::vector<std::vector<uint8_t>> hevc_split_pieces(const uint8_t* p, size_t n, int min_frames) {
  const std::vector<HNal> nals = scan_nals(p, n);
  // access unit starts: the first of (parameter sets / AUD / prefix SEI ...) before a first slice
  struct Au {
    size_t first_nal, vcl_nal;
    int type;
  };
  std::vector<Au> aus;
  size_t pending = 0;
  bool have_pending = false;
  for (size_t i = 0; i < nals.size(); ++i) {
    const int t = nals[i].type;
    const bool vcl = t <= 31;
    if (!vcl && (t == dec::VPS_NUT || t == dec::SPS_NUT || t == dec::PPS_NUT || t == dec::AUD_NUT || t == 39 ||
                 (t >= 41 && t <= 44))) {
      if (!have_pending) {
        pending = i;
        have_pending = true;
      }
      continue;
    }
    if (vcl && nals[i].first_slice) {
      aus.push_back(Au{have_pending ? pending : i, i, t});
      have_pending = false;
    } else if (vcl) {
      have_pending = false;
    }
  }
  if (aus.empty()) throw std::runtime_error("HEVC split: no pictures");
  if (!dec::is_irap(aus[0].type)) throw std::runtime_error("HEVC split: the stream does not start with an IRAP picture");
  auto clean_start = [&](size_t a) {
    if (!dec::is_irap(aus[a].type)) return false;
    if (aus[a].type != dec::CRA_NUT) return true;
    for (size_t b = a + 1; b < aus.size(); ++b) {
      if (dec::is_rasl(aus[b].type)) return false;
      if (!dec::is_radl(aus[b].type)) break;  // the first trailing picture ends the leading ones
    }
    return true;
  };
  std::vector<size_t> cuts = {0};
  for (size_t a = 1; a < aus.size(); ++a)
    if (static_cast<int>(a - cuts.back()) >= min_frames && clean_start(a)) cuts.push_back(a);
  // parameter sets in force at each cut (latest VPS / SPS / PPS per id seen before it)
  std::vector<std::vector<uint8_t>> out;
  std::map<int, std::pair<size_t, size_t>> vps, sps, pps;
  size_t scan = 0;
  auto id_of = [&](const HNal& h) {
    // parameter-set ids: VPS 4 bits after the header; SPS / PPS ue(v): read from the escaped bytes
    const size_t hdr = h.start + (p[h.start + 2] == 1 ? 3 : 4);
    std::vector<uint8_t> rb;
    int zeros = 0;
    for (size_t j = hdr + 2; j < h.end && rb.size() < 16; ++j) {
      if (zeros >= 2 && p[j] == 3) {
        zeros = 0;
        continue;
      }
      rb.push_back(p[j]);
      zeros = p[j] == 0 ? zeros + 1 : 0;
    }
    if (rb.empty()) return 0;
    BitReader br(rb.data(), rb.size());
    if (h.type == dec::VPS_NUT) return static_cast<int>(br.get(4));
    if (h.type == dec::SPS_NUT) {
      br.get(4);
      const int msl = br.get(3);
      br.get(1);
      // profile_tier_level: skip like parse_sps
      br.get(32);
      br.get(32);
      br.get(32);
      int pp[8] = {}, lp[8] = {};
      for (int i = 0; i < msl; ++i) {
        pp[i] = br.get(1);
        lp[i] = br.get(1);
      }
      if (msl > 0)
        for (int i = msl; i < 8; ++i) br.get(2);
      for (int i = 0; i < msl; ++i) {
        if (pp[i]) {
          br.get(32);
          br.get(32);
          br.get(24);
        }
        if (lp[i]) br.get(8);
      }
      return br.get_ue_max(15, "sps_seq_parameter_set_id");
    }
    return br.get_ue_max(63, "pps_pic_parameter_set_id");
  };
  for (size_t c = 0; c < cuts.size(); ++c) {
    const size_t a0 = cuts[c], a1 = c + 1 < cuts.size() ? cuts[c + 1] : aus.size();
    const size_t n0 = aus[a0].first_nal, n1 = a1 < aus.size() ? aus[a1].first_nal : nals.size();
    for (; scan < n0; ++scan) {
      const HNal& h = nals[scan];
      try {
        if (h.type == dec::VPS_NUT) vps[id_of(h)] = {h.start, h.end};
        if (h.type == dec::SPS_NUT) sps[id_of(h)] = {h.start, h.end};
        if (h.type == dec::PPS_NUT) pps[id_of(h)] = {h.start, h.end};
      } catch (const std::exception&) {
      }
    }
    std::vector<uint8_t> piece;
    // re-emit the parameter sets seen before the cut (the piece's own come after and win)
    for (auto* m : {&vps, &sps, &pps})
      for (auto& kv : *m) {
        if (p[kv.second.first + 2] == 1) piece.push_back(0);
        piece.insert(piece.end(), p + kv.second.first, p + kv.second.second);
      }
    const size_t b0 = nals[n0].start, b1 = n1 < nals.size() ? nals[n1].start : n;
    piece.insert(piece.end(), p + b0, p + b1);
    out.push_back(std::move(piece));
  }
  return out;
}

}  // namespace hevc
}  // namespace mivc
