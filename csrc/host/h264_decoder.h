// Independent H.264 decoder (CAVLC; I and P slices; 8-bit 4:2:0; progressive).
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

struct DecodedPicture {
  int width = 0, height = 0;          // cropped display size
  int coded_width = 0, coded_height = 0;
  int crop_x = 0, crop_y = 0;
  int frame_num = 0;
  int idr = 0;
  int slice_type = 0;
  std::vector<uint8_t> y, u, v;       // coded size planes
  // per-MB side info (coded raster order)
  std::vector<int8_t> mb_kind;        // MbKind as decoded (P_Skip = MBK_PSKIP)
  std::vector<int8_t> mb_qp;          // QP_Y
  std::vector<int16_t> mv;            // [mb][16][2] quarter-pel L0 MV per 4x4 block
  std::vector<int8_t> ref;            // [mb][16]
  std::vector<uint8_t> nz;            // [mb][16] non-zero luma coefficients per 4x4 block
  // copy the cropped planes out as one contiguous I420 frame
  std::vector<uint8_t> cropped_i420() const;
};

class Decoder {
 public:
  Decoder();
  ~Decoder();
  // Decode a complete Annex-B stream; pictures are appended to out() in
  // decoding order (== output order: no B-frames are supported).
  void decode(const uint8_t* data, size_t n);
  void flush();
  std::vector<DecodedPicture>& out() { return out_; }
  // Disable the in-loop filter (testing only: lets a test compare unfiltered recon)
  void set_skip_deblock(bool v) { skip_deblock_ = v; }

  struct Impl;

 private:
  std::unique_ptr<Impl> impl_;
  std::vector<DecodedPicture> out_;
  bool skip_deblock_ = false;
};

}  // namespace h264
}  // namespace mivc
