// HEVC (H.265) Main / Main 10 bitstream layer: parameter sets, slice headers and the
// CABAC coding of CTUs from decision records (hevc_writer.cc), plus an independent
// decoder (hevc_decoder.cc) that is the conformance oracle of the test-suite.
//
// Coding tools used by this encoder: 32x32 CTBs, CU quadtree
// 32/16/8, PART_2Nx2N, TU = CU (max_transform_hierarchy_depth 0), 35 intra modes
// with DM chroma, P slices with one reference picture (merge/skip + AMVP), one QP per
// CTB through cu_qp_delta (adaptive quantisation; or one QP per slice), deblocking and
// SAO, WPP substreams (every picture is one slice; pictures entropy-code in parallel on
// host threads).
//
// Reference parity: `-vcodec libx265 -crf 26` (server.go:67-68, client.go:115).
#pragma once
#include <cstdint>
#include <memory>
#include <vector>

#include "../common/hevc_ctu_coder.h"
#include "../common/hevc_tables.h"

namespace mivc {
namespace hevc {

struct HevcConfig {
  int width = 0, height = 0;   // display size
  int bit_depth = 8;           // 8 (Main) or 10 (Main 10)
  double fps = 30.0;
  int sao = 1;
  int deblock = 1;
  int max_merge = 5;
  int wpp = 0;                 // entropy_coding_sync_enabled_flag: one CABAC substream per CTB row
  int cu_qp_delta = 0;         // cu_qp_delta_enabled_flag: per-CTB QpY from CtuInfo::qp (AQ)
  int sdh = 0;                 // sign_data_hiding_enabled_flag (the levels must carry the parity)
  int tu_inter_depth = 0;      // max_transform_hierarchy_depth_inter: 1 = inter CUs may split their TU once
  int threads = 1;             // host threads coding the WPP substreams of one picture
  int level_idc = 0;           // > 0: general_level_idc (30 x level, -level); must fit the size / rate
  int bframes = 0;             // > 0: B pictures between the anchors (DPB of 2 references, 1 reordered picture)
  int pyramid = 0;             // reference B pictures (DPB of 3 references, 2 reordered pictures)
  int tmvp = 0;                // sps_temporal_mvp_enabled_flag: temporal merge / AMVP candidates (needs FrameParams::col)
  // 64x64 CTUs (x265 --ctu 64): the decision records stay per 32x32 block (CtuInfo / CuInfo as
  // for 32x32 CTBs); the writer codes each CTU's four blocks in z-order (a block's quadtree one
  // level down), one quantization group per 32x32 block (diff_cu_qp_delta_depth 1), SAO
  // parameters from the CTU's first block, and a 64x64 skip CU where the four blocks are one
  // uniform residual-free motion that is in the 64x64 merge list
  int ctu64 = 0;
  // weighted_pred_flag (x265 --weightp): P slices carry pred_weight_table() with log2
  // denominators 6 (luma and chroma) and the picture's FrameParams::wp weights
  int weightp = 0;
  // x265 --ref: the most active list-0 pictures of a P slice (HevcFrameParams::num_ref); sizes
  // the DPB (sps_max_dec_pic_buffering)
  int refs = 1;
  int ctb_log2() const { return ctu64 ? 6 : kCtbLog2; }
  int wctu() const { return (coded_width() + (1 << ctb_log2()) - 1) >> ctb_log2(); }
  int hctu() const { return (coded_height() + (1 << ctb_log2()) - 1) >> ctb_log2(); }
  int coded_width() const { return (width + kCtb - 1) / kCtb * kCtb; }
  int coded_height() const { return (height + kCtb - 1) / kCtb * kCtb; }
  int wctb() const { return coded_width() / kCtb; }
  int hctb() const { return coded_height() / kCtb; }
};

// The collocated picture of temporal motion vector prediction (8.5.3.2.8): its decision
// records (same layout as the current picture's) and the POCs its motion points to.
constexpr int kMaxRefs = 4;   // active pictures per reference list this encoder codes

struct HevcColPic {
  int set = 0;                 // must be 1 in P / B slices when HevcConfig::tmvp is on
  const CuInfo* cu = nullptr;  // nullptr: an intra picture (no temporal candidates)
  int poc = 0;
  int ref_poc[2] = {0, 0};     // POC of the col picture's RefPicList0[0] / RefPicList1[0]
  // POCs of the col picture's RefPicListX[i] (its CuInfo records carry refIdx in pad[0] / pad[1]);
  // entries past the list's end repeat ref_poc[X]
  int list_poc[2][kMaxRefs] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
};

struct HevcFrameParams {
  int idr = 1;
  int poc = 0;          // picture order count
  int qp = 30;          // SliceQpY
  int slice_type = 2;   // 2 = I, 1 = P, 0 = B
  int nal_ref = 1;      // 0: a sub-layer non-reference picture (TRAIL_N)
  // one reference picture per list: RefPicList0[0] / RefPicList1[0] POCs (-1: P slices use
  // poc - 1); the slice's short-term RPS holds exactly these pictures
  int ref_poc[2] = {-1, -1};
  // several active pictures per list (x265 --ref): num_ref[X] entries of RefPicListX, whose POCs
  // are list_poc[X][0 ..] (list_poc[X][0] = ref_poc[X]); the lists must be the default
  // construction (8.3.4) from the RPS's used pictures.  CuInfo pad[0] / pad[1] = refIdx L0 / L1
  int num_ref[2] = {1, 1};
  int list_poc[2][kMaxRefs] = {{-1, -1, -1, -1}, {-1, -1, -1, -1}};
  // explicit short-term RPS (n_rps >= 0): every picture the DPB keeps, with used_by_curr;
  // RefPicList0[0] / RefPicList1[0] must be the closest used picture before / after
  int n_rps = -1;
  int rps_poc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint8_t rps_used[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  HevcColPic col;       // with HevcConfig::tmvp: the collocated picture (L1[0] in B, L0[0] in P)
  // with HevcConfig::weightp, P slices: explicit weights of RefPicList0[0] (wp = 0: flags off)
  // -- luma weight / offset, then Cb, Cr (weights over 2^6, offsets in 8-bit units)
  int wp = 0;
  int wp_w[3] = {64, 64, 64};
  int wp_o[3] = {0, 0, 0};
};

struct HevcSliceStats {
  uint64_t bins = 0;
  uint64_t bytes = 0;
  int intra_cus = 0, inter_cus = 0, skip_cus = 0, merge_cus = 0;
};

// VPS + SPS + PPS as Annex-B NAL units
std::vector<uint8_t> hevc_parameter_sets(const HevcConfig& cfg);

// Quantised levels in the GPU encoder's packed form (hevc_nz_pack, hevc_filters.hip): only
// the non-zero 4x4 blocks cross PCIe.  Per CTB (raster): nzmap[2 ci] luma sub-block bits
// (by * 8 + bx), nzmap[2 ci + 1] Cb bits 0-15 and Cr bits 16-31 (by * 4 + bx); ctb_off[ci]
// = index of the CTB's first block in `levels`; blocks in luma, Cb, Cr, bit order, 16
// levels each (raster inside the block).
struct PackedLevels {
  const uint64_t* nzmap = nullptr;
  const uint32_t* ctb_off = nullptr;
  const int16_t* levels = nullptr;
  size_t nblocks = 0;  // blocks available in `levels` (bounds check)
};

// One slice NAL (Annex-B) for a whole picture.  ctu: [wctb*hctb]; cu: [wctb*hctb*16]
// (z-order granules); coef planes sized like the coded picture (luma) / half (chroma), or
// null with `packed` given.
std::vector<uint8_t> hevc_write_slice(const HevcConfig& cfg, const HevcFrameParams& fp, const CtuInfo* ctu,
                                      const CuInfo* cu, const int16_t* coef_y, const int16_t* coef_cb,
                                      const int16_t* coef_cr, HevcSliceStats* stats,
                                      const PackedLevels* packed = nullptr,
                                      std::vector<std::vector<uint8_t>>* substreams = nullptr);

// The slice-data coder's view of a picture (hevc_ctu_coder.h): sizes, tools, slice type, QP,
// reference / collocated POCs (the collocated records pointer is passed separately)
CoderPic hevc_coder_pic(const HevcConfig& cfg, const HevcFrameParams& fp);

// One slice NAL from substreams coded elsewhere (the GPU entropy kernel): the slice header of
// `fp`, the entry points of the nsub substreams (one per CTU row with WPP, else one), the
// substreams, emulation prevention -- byte-identical to hevc_write_slice on the same records.
std::vector<uint8_t> hevc_assemble_slice(const HevcConfig& cfg, const HevcFrameParams& fp, const uint8_t* const* sub,
                                         const uint32_t* sizes, int nsub);

struct HevcPicture {
  int width = 0, height = 0;            // cropped (display) size
  int coded_width = 0, coded_height = 0;
  int bit_depth = 8;
  int poc = 0, idr = 0, slice_type = 2, qp = 0;
  std::vector<uint16_t> y, u, v;        // coded-size planes
  // parse records (the encoder's decision format, see hevc_tables.h)
  std::vector<CtuInfo> ctu;
  std::vector<CuInfo> cu;
  std::vector<int16_t> coef_y, coef_cb, coef_cr;
};

class HevcDecoder {
 public:
  HevcDecoder();
  ~HevcDecoder();
  void decode(const uint8_t* data, size_t n);
  std::vector<HevcPicture>& out() { return out_; }
  void set_skip_loop_filters(bool v) { skip_filters_ = v; }  // tests: unfiltered reconstruction
  struct Impl;

 private:
  std::unique_ptr<Impl> impl_;
  std::vector<HevcPicture> out_;
  bool skip_filters_ = false;
};

}  // namespace hevc
}  // namespace mivc
