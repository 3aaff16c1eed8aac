// Host side of the batched GPU decoders: many segments parsed on C++ threads and kept in
// C++, and the packer that lays one picture step of every slot out in one (pinned) host
// buffer, so a step reaches the device with a single copy and Python never touches the
// per-macroblock records.
//
// Reference parity: the reference decodes a piece inside ffmpeg (client.go:115-118); this is
// the hand-off between the bit-serial entropy decode (host) and the GPU reconstruction
// (csrc/kernels/decode.hip) of the batched transcode (models/transcode.py).
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "h264_decoder.h"
#include "hevc_dec.h"
#include <memory>

namespace mivc {

struct H264Parsed {
  std::vector<h264::DecodedPicture> pics;  // decoding order
  std::string error;                       // non-empty: the segment did not parse
};

// entropy decode (parse-only) of one segment / of many on `threads` C++ threads
H264Parsed h264_parse_segment(const std::string& data);
std::vector<H264Parsed> h264_parse_many(const std::vector<std::string>& segs, int threads);

// byte offsets of one picture step's sections in the packed buffer (256-byte aligned)
struct H264StepLayout {
  size_t hdr = 0;   // [B][nmb] MbHeader (MBF_SUB4 indices made global to the step)
  size_t mask = 0;  // [B][nmb] uint32 present-block masks
  size_t off = 0;   // [B][nmb] uint32 first block, global to the step's coef section
  size_t bs = 0;    // [B][nmb][16] packed boundary strengths
  size_t wp = 0;    // [B][kWpEntries] int16 weighted-prediction tables
  size_t coef = 0;  // packed levels of every active slot
  size_t sub = 0;   // side-pool entries of every active slot
  size_t total = 0;
};

class H264Batch {
 public:
  std::vector<H264Parsed> segs;
  // slot j reconstructs picture t of segment slots[j] (-1 or t past its end: idle slot)
  H264StepLayout layout(int t, const std::vector<int>& slots, int nmb) const;
  void pack(int t, const std::vector<int>& slots, int nmb, uint8_t* dst, int threads) const;

 private:
  const h264::DecodedPicture* pic(int t, int seg) const;
};

// ---------------------------------------------------------------- HEVC
struct HevcParsed {
  std::unique_ptr<hevc::HevcStreamDecoder> dec;  // pictures() in decoding order
  std::vector<int> order;                        // output order (indices into pictures())
  std::string error;
};
std::vector<HevcParsed> hevc_parse_many(const std::vector<std::string>& segs, int threads, bool recon);

// sections of one HEVC picture step (csrc/kernels/hevc_decode.h HevcDecParams); 256-byte aligned
struct HevcStepLayout {
  size_t meta = 0, tu_base = 0, coef_base = 0, op_base = 0, ref_base = 0, slice_base = 0, ctb_ops = 0;
  size_t mvf = 0, mvf_sub = 0, bs = 0, ctbs = 0, sao = 0, tus = 0, coefs = 0, ops = 0, refs = 0, slices = 0, scaling = 0;
  size_t total = 0;
  int max_tus = 0;           // most transform blocks of one slot (residual grid)
  bool scaling_on = false;   // a slot uses scaling lists (else the section is empty)
  bool deblock_any = false, sao_any = false;
};

class HevcBatch {
 public:
  HevcBatch() = default;
  HevcBatch(const HevcBatch&) = delete;  // holds the decoders (unique_ptr)
  HevcBatch& operator=(const HevcBatch&) = delete;
  std::vector<HevcParsed> segs;
  // slot j reconstructs picture t (decoding order) of segment slots[j] (-1 / past its end: idle)
  HevcStepLayout layout(int t, const std::vector<int>& slots) const;
  void pack(int t, const std::vector<int>& slots, uint8_t* dst, int threads) const;

 private:
  const hevc::DecPicture* pic(int t, int seg) const;
};

}  // namespace mivc
