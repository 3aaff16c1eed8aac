// CPU reference H.264 encoder (the "cpu_ref" backend).
//
// Role: (1) the always-available backend for BASELINE config 1 (the reference's
// CPU `ffmpeg -vcodec libx264` subprocess, client.go:115, when no ffmpeg binary
// exists -- this image has none) and for CPU-only tests of the job API and the
// distributed pipeline; (2) a readable, scalar statement of the encoding
// algorithm that the gfx950 kernels implement in parallel form.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../common/h264_mb.h"
#include "h264_syntax.h"

namespace mivc {
namespace h264 {

struct EncoderConfig {
  int width = 0, height = 0;
  double fps = 30.0;
  int qp = 26;          // used when crf < 0
  double crf = -1.0;    // >= 0 selects the CRF rate control (per-frame QP from complexity)
  int keyint = 250;     // IDR period inside a segment
  int me_range = 16;
  int subpel = 2;       // 0 integer, 1 half, 2 quarter
  int use_i4x4 = 1;
  int deblock = 1;
  int chroma_qp_offset = 0;
  int aud = 0;
  int vui = 1;
  // tool set: entropy 0 CAVLC / 1 CABAC; t8x8 = High profile 8x8 transform (+ I8x8);
  // bframes = consecutive B pictures (POC type 0 and reordering); refs = active L0 refs
  int cabac = 0;
  int t8x8 = 0;
  // sample bit depth of the written stream: 9..14 = High 10 SPS (the CPU encoder itself is 8-bit;
  // the record writer takes deeper I_PCM samples and QPs down to -QpBdOffsetY)
  int bit_depth = 8;
  int bit_depth_chroma = 0;  // 0: = bit_depth (else written as BitDepthC; decoder-rejection tests)
  int bframes = 0;
  int pyramid = 0;          // x264 --b-pyramid normal: some B pictures are references (reorder depth 2)
  int refs = 1;
  int weighted_bipred = 0;  // 2 = implicit weights (x264 --weightb)
  int constrained_intra = 0;  // constrained_intra_pred_flag (writer / decoder tests)
  int weightp = 0;          // weighted_pred_flag: P slices carry pred_weight_table() (x264 --weightp)
  int level_idc = 0;        // > 0: written as level_idc (-level); must fit the size / rate
  // scaling matrices (High profile, t8x8): 0 flat; 1 the default matrices (x264 --cqm jvt: SPS
  // flag, no list sent); 2 the lists below in the SPS; 3 the lists below in the PPS over the
  // default matrices in the SPS (fall-back rule B).  Lists not
  // in cqm_coded (bit i = list i) fall back per 7.4.2.1.1 / 7.4.2.2.  Weights in raster order.
  int cqm = 0;
  int cqm_coded = 0xFF;
  uint8_t cqm4[6][16] = {};
  uint8_t cqm8[2][64] = {};
};

struct FrameStats {
  int type = 0;  // SliceType
  int qp = 0;
  int bytes = 0;
  double psnr_y = 0;
};

class CpuEncoder {
 public:
  explicit CpuEncoder(const EncoderConfig& cfg);
  // Encode frames of one closed-GOP segment (I420, tightly packed, width*height*3/2 bytes each).
  // Returns the Annex-B stream (SPS/PPS + slices).  idr_pic_id distinguishes
  // consecutive segments once concatenated.
  std::vector<uint8_t> encode(const uint8_t* frames, int nframes, int idr_pic_id);
  const std::vector<FrameStats>& stats() const { return stats_; }
  // Reconstructed (decoded, deblocked, cropped) frames of the last encode()
  const std::vector<uint8_t>& recon() const { return recon_; }
  // Encoder-side (pre-deblocking) reconstruction in coded size (Y then U, V per frame):
  // must equal the decoder's output with the loop filter disabled.
  const std::vector<uint8_t>& recon_unfiltered() const { return recon_unf_; }

 private:
  EncoderConfig cfg_;
  std::vector<FrameStats> stats_;
  std::vector<uint8_t> recon_;
  std::vector<uint8_t> recon_unf_;
};

// Shared helpers exposed for tests
SPS make_sps(const EncoderConfig& cfg);
PPS make_pps(const EncoderConfig& cfg);

}  // namespace h264
}  // namespace mivc
