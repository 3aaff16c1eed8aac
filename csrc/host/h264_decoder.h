// Independent H.264 decoder (CAVLC + CABAC; I, P and B slices; Baseline/Main/High/High 10;
// 8- to 14-bit 4:2:0; progressive).
//
// Written directly from ITU-T H.264 clauses 7-9 and kept deliberately separate
// from the encoder-side writer (cavlc_writer.cc) and the HIP kernels: it shares
// only the constant tables.  It is the conformance oracle of the test-suite
// (SURVEY.md §4.2 tier T2: "encoder recon == our decoder output, bit-exact") and
// the decode stage of the transcode path (BASELINE config 3).
//
// Reference parity: the reference delegates decoding to ffmpeg
// (client.go:115-118 `ffmpeg -i <idx>.mp4 ...`).
#pragma once
#include <cstdint>
#include <memory>
#include <vector>

#include "h264_syntax.h"

namespace mivc {
namespace h264 {

// Weighted-prediction table of one picture (parse-only mode), int16 entries:
// [0] mode (0 default, 1 explicit, 2 implicit), [1] luma_log2_weight_denom,
// [2] chroma_log2_weight_denom, [kWpLw + l*32 + i] luma weight, [kWpLo + ...] luma offset,
// [kWpCw + (l*32 + i)*2 + c] chroma weight, [kWpCo + ...] chroma offset,
// [kWpImp + (i*8 + j)*2 + k] implicit weights w0/w1 of (refIdxL0 i, refIdxL1 j), i, j < 8.
// [kWpScale + list * 16 + raster] the PPS's 4x4 scaling lists (Intra Y/Cb/Cr, Inter Y/Cb/Cr),
// [kWpScale + 96 + list * 64 + raster] its 8x8 lists (Intra Y, Inter Y),
// [kWpFlags] bit 0: constrained_intra_pred_flag.
enum : int { kWpLw = 4, kWpLo = 68, kWpCw = 132, kWpCo = 260, kWpImp = 388, kWpScale = 516, kWpFlags = 740,
             kWpEntries = 742 };

struct DecodedPicture {
  int width = 0, height = 0;          // cropped display size
  int coded_width = 0, coded_height = 0;
  int crop_x = 0, crop_y = 0;
  int frame_num = 0;
  int poc = 0;                        // PicOrderCnt (pictures come out in increasing POC)
  int idr = 0;
  int slice_type = 0;
  int bit_depth = 8;                  // BitDepthY (chroma has the SPS's BitDepthC)
  std::vector<uint8_t> y, u, v;       // coded size planes (8-bit streams)
  std::vector<uint16_t> y16, u16, v16; // coded size planes of High 10 (9..14-bit) streams
  // per-MB side info (coded raster order)
  std::vector<int8_t> mb_kind;        // MbKind as decoded (P_Skip = MBK_PSKIP)
  std::vector<int8_t> mb_qp;          // QP_Y
  std::vector<int16_t> mv;            // [mb][16][2] quarter-pel L0 MV per 4x4 block
  std::vector<int8_t> ref;            // [mb][16]
  std::vector<uint8_t> nz;            // [mb][16] non-zero luma coefficients per 4x4 block
  // parse-only mode (GPU reconstruction): per-MB decision records in the encoder's layout
  // (csrc/common/h264_mb.h: MbHeader + kCoefPerMb levels), plus the slice parameters
  std::vector<uint8_t> hdr;           // [mb][64] MbHeader
  std::vector<int16_t> coef;          // packed 16-level blocks (scan order, not dequantised)
  std::vector<uint32_t> blk_mask;     // [mb] which blocks are present: bits 0-15 luma (blkIdx),
                                      // 16 I16x16 DC, 17 chroma DC (Cb 0-3, Cr 4-7), 18-25 chroma AC
  std::vector<uint32_t> blk_off;      // [mb] index of the MB's first block in coef (units of 16)
  int pic_id = 0, ref_id = -1;        // decode-order id of this picture / of its L0 ref 0
  int nal_ref = 1;
  int slice_qp = 0, alpha_off = 0, beta_off = 0, chroma_qp_offset = 0, deblock = 1;
  bool gpu_ok = true;                 // false: a feature the GPU path does not cover (I_PCM,
                                      // Intra8x8, several slices, constrained intra, mmco5 ...)
  // parse-only motion / filter side info for GPU reconstruction of P and B pictures
  // (per-8x8 quadrant motion is in hdr; MBs with smaller partitions carry MBF_SUB4 and a
  // kSubEntry side-pool entry, csrc/common/h264_mb.h)
  std::vector<int16_t> sub;           // side pool, kSubEntry int16 per MBF_SUB4 macroblock
  std::vector<uint8_t> bs;            // [mb][16] boundary strength, 4 bits per segment
                                      // i = dir * 16 + edge * 4 + k (byte i / 2, low nibble even i)
  std::vector<int32_t> list_ids;      // [2][32] decode-order picture id of RefPicList0/1[i], -1
  std::vector<int16_t> wp;            // kWpEntries: weighted-prediction table (see kWp* below)
  // copy the cropped planes out as one contiguous I420 frame
  std::vector<uint8_t> cropped_i420() const;
  std::vector<uint16_t> cropped_i420_16() const;  // the 16-bit planes (bit_depth > 8)
};

class Decoder {
 public:
  Decoder();
  ~Decoder();
  // Decode a complete Annex-B stream; pictures are appended to out() in output
  // (display) order -- in parse-only mode in decoding order.
  void decode(const uint8_t* data, size_t n);
  void flush();
  std::vector<DecodedPicture>& out() { return out_; }
  // Disable the in-loop filter (testing only: lets a test compare unfiltered recon)
  void set_skip_deblock(bool v) { skip_deblock_ = v; }
  // Entropy-decode only: fill DecodedPicture::hdr/coef/nz and skip pixel reconstruction
  void set_parse_only(bool v);
  // the effective scaling lists of a parsed PPS (raster weights: 6 x 16, then 2 x 64)
  void pps_scaling(int pps_id, uint8_t* sl4, uint8_t* sl8) const;

  struct Impl;

 private:
  std::unique_ptr<Impl> impl_;
  std::vector<DecodedPicture> out_;
  bool skip_deblock_ = false;
};

}  // namespace h264
}  // namespace mivc
