// HEVC CABAC arithmetic coding engines (clause 9.3), encoder and decoder.
//
// The encoder follows the low/range formulation with deferred carry handling
// (outstanding 0xFF bytes); the decoder is the normative 9-bit offset engine.  Both
// use the context tables of csrc/common/hevc_tables.h.
#pragma once
#include <array>
#include <cstdint>
#include <stdexcept>
#include <vector>

#include "../common/hevc_ctu_coder.h"
#include "../common/hevc_tables.h"
#include "bitstream.h"
#include "hevc_ctx_tables.h"

namespace mivc {
namespace hevc {

// host arithmetic encoder writing into a BitWriter (the engine of hevc_ctu_coder.h)
class CabacEncoder : public CabacEngine<BitWriter> {
 public:
  explicit CabacEncoder(BitWriter& bw) { out = &bw; }
};

class CabacDecoder {
 public:
  CabacDecoder(const uint8_t* p, size_t n, size_t byte_pos) : p_(p), n_(n), pos_(byte_pos * 8) {}

  void start() {
    range_ = 510;
    offset_ = read_bits(9);
  }

  int decode(CtxState& c) {
    const uint32_t lps = kRangeLps[c.state][(range_ >> 6) & 3];
    range_ -= lps;
    int bin;
    if (offset_ >= range_) {
      bin = 1 - c.mps;
      offset_ -= range_;
      range_ = lps;
      if (c.state == 0) c.mps = static_cast<uint8_t>(1 - c.mps);
      c.state = kTransIdxLps[c.state];
    } else {
      bin = c.mps;
      if (c.state < 62) ++c.state;
    }
    while (range_ < 256) {
      range_ <<= 1;
      offset_ = (offset_ << 1) | read_bit();
    }
    return bin;
  }

  int bypass() {
    offset_ = (offset_ << 1) | read_bit();
    if (offset_ >= range_) {
      offset_ -= range_;
      return 1;
    }
    return 0;
  }

  uint32_t bypass_bits(int n) {
    uint32_t v = 0;
    for (int i = 0; i < n; ++i) v = (v << 1) | static_cast<uint32_t>(bypass());
    return v;
  }

  // after a terminating bin equal to 1 the engine has consumed the flush's final 1 bit;
  // skip the alignment zeros to the next substream
  void align() {
    while (pos_ & 7) {
      if (read_bit() != 0) throw std::runtime_error("CABAC: non-zero alignment bit");
    }
  }
  size_t byte_pos() const { return pos_ >> 3; }

  int terminate() {
    range_ -= 2;
    if (offset_ >= range_) return 1;
    while (range_ < 256) {
      range_ <<= 1;
      offset_ = (offset_ << 1) | read_bit();
    }
    return 0;
  }

 private:
  uint32_t read_bit() {
    if (pos_ >= n_ * 8) {
      ++pos_;
      if (pos_ > n_ * 8 + 64) throw std::runtime_error("CABAC: read past the end of the slice data");
      return 0;
    }
    const uint32_t b = (p_[pos_ >> 3] >> (7 - (pos_ & 7))) & 1u;
    ++pos_;
    return b;
  }
  uint32_t read_bits(int n) {
    uint32_t v = 0;
    for (int i = 0; i < n; ++i) v = (v << 1) | read_bit();
    return v;
  }

  const uint8_t* p_;
  size_t n_;
  size_t pos_;
  uint32_t range_ = 510, offset_ = 0;
};

}  // namespace hevc
}  // namespace mivc
