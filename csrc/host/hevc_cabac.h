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

#include "../common/hevc_tables.h"
#include "bitstream.h"
#include "hevc_ctx_tables.h"

namespace mivc {
namespace hevc {

struct CtxState {
  uint8_t state = 0;
  uint8_t mps = 0;
};

// 9.3.2.2: contexts initialised for a slice of the given initType and SliceQpY
// writer context index -> index in the spec initValue table (hevc_ctx_tables.h, dec::DCtx)
inline constexpr std::array<uint8_t, kNumCtx> writer_ctx_map() {
  std::array<uint8_t, kNumCtx> m{};
  auto run = [&m](int w, int d, int n) {
    for (int i = 0; i < n; ++i) m[w + i] = static_cast<uint8_t>(d + i);
  };
  run(CTX_SAO_MERGE, dec::C_SAO_MERGE, 1);
  run(CTX_SAO_TYPE, dec::C_SAO_TYPE, 1);
  run(CTX_SPLIT_CU, dec::C_SPLIT_CU, 3);
  run(CTX_CU_SKIP, dec::C_SKIP, 3);
  run(CTX_PRED_MODE, dec::C_PRED_MODE, 1);
  run(CTX_PART_MODE, dec::C_PART_MODE, 4);
  run(CTX_PREV_INTRA, dec::C_PREV_INTRA, 1);
  run(CTX_CHROMA_MODE, dec::C_CHROMA_MODE, 1);
  run(CTX_MERGE_FLAG, dec::C_MERGE_FLAG, 1);
  run(CTX_MERGE_IDX, dec::C_MERGE_IDX, 1);
  run(CTX_MVD_G0, dec::C_MVD_G0, 1);
  run(CTX_MVD_G1, dec::C_MVD_G1, 1);
  run(CTX_MVP_IDX, dec::C_MVP, 1);
  run(CTX_RQT_ROOT_CBF, dec::C_ROOT_CBF, 1);
  run(CTX_SPLIT_TRANSFORM, dec::C_SPLIT_TF, 3);
  run(CTX_CBF_LUMA, dec::C_CBF_LUMA, 2);
  run(CTX_CBF_CHROMA, dec::C_CBF_CHROMA, 4);
  run(CTX_LAST_X, dec::C_LAST_X, 18);
  run(CTX_LAST_Y, dec::C_LAST_Y, 18);
  run(CTX_CSBF, dec::C_CSBF, 4);
  run(CTX_SIG, dec::C_SIG, 42);
  run(CTX_GT1, dec::C_GT1, 24);
  run(CTX_GT2, dec::C_GT2, 6);
  run(CTX_REF_IDX, dec::C_REF_IDX, 2);
  run(CTX_CU_QP_DELTA, dec::C_QP_DELTA, 2);
  run(CTX_INTER_PRED, dec::C_INTER_PRED, 5);
  return m;
}
inline constexpr std::array<uint8_t, kNumCtx> kWriterCtxToSpec = writer_ctx_map();

// 9.3.2.2 initialisation; init_type 0 = I, 1 = P, 2 = B (cabac_init_flag 0)
inline void init_contexts(CtxState* ctx, int init_type, int slice_qp) {
  const int qp = slice_qp < 0 ? 0 : (slice_qp > 51 ? 51 : slice_qp);
  for (int i = 0; i < kNumCtx; ++i) {
    const int v = dec::kInit[init_type][kWriterCtxToSpec[i]];
    const int m = (v >> 4) * 5 - 45, n = ((v & 15) << 3) - 16;
    int pre = ((m * qp) >> 4) + n;
    pre = pre < 1 ? 1 : (pre > 126 ? 126 : pre);
    if (pre <= 63) {
      ctx[i].state = static_cast<uint8_t>(63 - pre);
      ctx[i].mps = 0;
    } else {
      ctx[i].state = static_cast<uint8_t>(pre - 64);
      ctx[i].mps = 1;
    }
  }
}

// next state after an MPS ([0]) or LPS ([1]) bin (9.3.4.3.2.2)
struct NextStateTable {
  uint8_t t[2][64];
  constexpr NextStateTable() : t() {
    for (int i = 0; i < 64; ++i) {
      t[0][i] = static_cast<uint8_t>(i < 62 ? i + 1 : i);
      t[1][i] = kTransIdxLps[i];
    }
  }
};
static constexpr NextStateTable kNextStateT{};
static constexpr const uint8_t (&kNextState)[2][64] = kNextStateT.t;

class CabacEncoder {
 public:
  explicit CabacEncoder(BitWriter& bw) : bw_(bw) {}

  void start() {
    low_ = 0;
    range_ = 510;
    bits_left_ = 23;
    num_buffered_ = 0;
    buffered_ = 0xFF;
    bins_ = 0;
  }

  // branch-free regular bin (9.3.4.3.2): the LPS / MPS choice selects range and low with
  // conditional moves, the renormalisation shift is a count of leading zeros, and the
  // state transition is one table entry (an unpredictable bin costs no mispredict)
  void encode(int bin, CtxState& c) {
    // members are read into locals before the context (uint8_t, may alias anything) is
    // written, so they stay in registers
    const uint32_t s = c.state, mps = c.mps;
    uint32_t range = range_, low = low_;
    const uint32_t lps = kRangeLps[s][(range >> 6) & 3];
    const uint32_t rmps = range - lps;
    const bool is_lps = static_cast<uint32_t>(bin) != mps;
    const uint32_t r = is_lps ? lps : rmps;
    low += is_lps ? rmps : 0u;
    const int nb = __builtin_clz(r) - 23;  // r in [2, 510]: shifts until r >= 256
    const int left = bits_left_ - nb;
    range_ = r << nb;
    low_ = low << nb;
    bits_left_ = left;
    ++bins_;
    c.mps = static_cast<uint8_t>(mps ^ static_cast<uint32_t>(is_lps && s == 0));
    c.state = kNextState[is_lps][s];
    if (left < 12) write_out();
  }

  void bypass(int bin) {
    ++bins_;
    low_ <<= 1;
    if (bin) low_ += range_;
    if (--bits_left_ < 12) write_out();
  }

  // n bypass bins, most significant first (n <= 16 per call keeps low_ in range)
  void bypass_bits(uint32_t v, int n) {
    while (n > 8) {
      n -= 8;
      bypass_chunk((v >> n) & 255u, 8);
    }
    if (n > 0) bypass_chunk(v & ((1u << n) - 1u), n);
  }

  void terminate(int bin) {
    ++bins_;
    range_ -= 2;
    if (bin) {
      low_ += range_;
      low_ <<= 7;
      range_ = 2 << 7;
      bits_left_ -= 7;
    } else if (range_ >= 256) {
      return;
    } else {
      low_ <<= 1;
      range_ <<= 1;
      --bits_left_;
    }
    if (bits_left_ < 12) write_out();
  }

  // flush after the terminating bin of the slice (end_of_slice_segment_flag == 1)
  void finish() {
    if ((low_ >> (32 - bits_left_)) != 0) {
      bw_.put(buffered_ + 1, 8);
      while (num_buffered_ > 1) {
        bw_.put(0x00, 8);
        --num_buffered_;
      }
      low_ -= 1u << (32 - bits_left_);
    } else {
      if (num_buffered_ > 0) bw_.put(buffered_, 8);
      while (num_buffered_ > 1) {
        bw_.put(0xFF, 8);
        --num_buffered_;
      }
    }
    bw_.put(low_ >> 8, 24 - bits_left_);
  }

  uint64_t bins() const { return bins_; }

 private:
  static int renorm_bits(uint32_t lps) {
    int n = 0;
    while ((lps << n) < 256) ++n;
    return n;
  }
  void bypass_chunk(uint32_t v, int n) {
    bins_ += n;
    low_ <<= n;
    low_ += range_ * v;
    bits_left_ -= n;
    if (bits_left_ < 12) write_out();
  }
  void write_out() {
    const uint32_t lead = low_ >> (24 - bits_left_);
    bits_left_ += 8;
    low_ &= 0xFFFFFFFFu >> bits_left_;
    if (lead == 0xFF) {
      ++num_buffered_;
    } else if (num_buffered_ > 0) {
      const uint32_t carry = lead >> 8;
      bw_.put(buffered_ + carry, 8);
      buffered_ = lead & 0xFF;
      const uint32_t fill = (0xFF + carry) & 0xFF;
      while (num_buffered_ > 1) {
        bw_.put(fill, 8);
        --num_buffered_;
      }
    } else {
      num_buffered_ = 1;
      buffered_ = lead;
    }
  }

  BitWriter& bw_;
  uint32_t low_ = 0, range_ = 510;
  int bits_left_ = 23;
  int num_buffered_ = 0;
  uint32_t buffered_ = 0xFF;
  uint64_t bins_ = 0;
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
