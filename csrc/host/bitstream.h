// Bit-level writer/reader, Exp-Golomb codes and NAL/Annex-B framing (H.264 clause
// 7.2, 7.3.1, 9.1, Annex B).
//
// Reference parity: the reference never touches a bitstream itself; its only
// "bitstream" operations are ffmpeg's stream-copy segmenting and concatenation
// (server.go:199-201, server.go:357).  These primitives are what our native
// split/merge (annexb.cc) and the entropy coders are built on.
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace mivc {

class BitWriter {
 public:
  BitWriter() { buf_.reserve(1 << 16); }
  void put(uint32_t value, int nbits) {  // nbits in [0,32]
    if (nbits <= 0) return;
    if (nbits < 32) value &= (1u << nbits) - 1u;
    acc_ = (acc_ << nbits) | value;  // acc_ is 64-bit; at most 7 + 32 bits in flight
    nacc_ += nbits;
    while (nacc_ >= 8) {
      nacc_ -= 8;
      buf_.push_back(static_cast<uint8_t>(acc_ >> nacc_));
    }
    acc_ &= (nacc_ ? ((1ull << nacc_) - 1ull) : 0ull);
  }
  void put_bit(int b) { put(b ? 1u : 0u, 1); }
  void put_ue(uint32_t v) {
    uint64_t x = static_cast<uint64_t>(v) + 1;
    int len = 0;
    while ((x >> len) > 1) ++len;  // floor(log2(x))
    if (len > 0) put(0, len);
    if (len + 1 > 32) {
      put(static_cast<uint32_t>(x >> 32), len + 1 - 32);
      put(static_cast<uint32_t>(x), 32);
    } else {
      put(static_cast<uint32_t>(x), len + 1);
    }
  }
  void put_se(int32_t v) { put_ue(v <= 0 ? static_cast<uint32_t>(-2ll * v) : static_cast<uint32_t>(2ll * v - 1)); }
  void put_te(uint32_t v, uint32_t range) {
    if (range == 1) put_bit(!v); else put_ue(v);
  }
  // rbsp_trailing_bits(): stop bit + zero alignment
  void trailing() {
    put_bit(1);
    align_zero();
  }
  void align_zero() {
    if (nacc_) put(0, 8 - nacc_);
  }
  bool byte_aligned() const { return nacc_ == 0; }
  size_t bit_pos() const { return buf_.size() * 8 + nacc_; }
  const std::vector<uint8_t>& bytes() const { return buf_; }
  std::vector<uint8_t>& bytes() { return buf_; }
  void append_bytes(const uint8_t* p, size_t n) {
    if (nacc_) throw std::runtime_error("append_bytes on unaligned writer");
    buf_.insert(buf_.end(), p, p + n);
  }

 private:
  std::vector<uint8_t> buf_;
  uint64_t acc_ = 0;
  int nacc_ = 0;
};

class BitReader {
 public:
  BitReader(const uint8_t* p, size_t n) : p_(p), n_(n) {}
  uint32_t get(int nbits) {
    uint32_t v = 0;
    for (int i = 0; i < nbits; ++i) v = (v << 1) | get_bit();
    return v;
  }
  uint32_t get_bit() {
    if (pos_ >= n_ * 8) throw std::runtime_error("bitstream overrun");
    uint32_t b = (p_[pos_ >> 3] >> (7 - (pos_ & 7))) & 1u;
    ++pos_;
    return b;
  }
  uint32_t peek(int nbits) const {
    uint32_t v = 0;
    size_t q = pos_;
    for (int i = 0; i < nbits; ++i, ++q) {
      uint32_t b = q < n_ * 8 ? (p_[q >> 3] >> (7 - (q & 7))) & 1u : 0u;
      v = (v << 1) | b;
    }
    return v;
  }
  void skip(int nbits) { pos_ += nbits; }
  void seek(size_t bitpos) { pos_ = bitpos; }
  uint32_t get_ue() {
    int lz = 0;
    while (get_bit() == 0) {
      if (++lz > 32) throw std::runtime_error("invalid exp-golomb code");
    }
    if (lz == 0) return 0;
    const uint64_t v = (1ull << lz) - 1 + get(lz);
    if (v > 0xffffffffull) throw std::runtime_error("exp-golomb code above 2^32 - 1");  // no silent wrap
    return static_cast<uint32_t>(v);
  }
  int32_t get_se() {
    const uint32_t k = get_ue();
    if (!(k & 1)) return -static_cast<int32_t>(k / 2);
    const uint64_t m = (static_cast<uint64_t>(k) + 1) / 2;  // (k + 1) / 2 without the 32-bit wrap
    if (m > 0x7fffffffu) throw std::runtime_error("se(v) out of range");
    return static_cast<int32_t>(m);
  }
  // Range-checked Exp-Golomb reads.  Every syntax element that is narrowed to `int`, used as
  // an index or a count, or has a constant added goes through these: the raw code is compared
  // with the element's legal range BEFORE any narrowing or arithmetic, so a crafted 32-leading-
  // zero code (up to 2^32-1) can neither wrap into a small / negative int nor overflow later.
  int get_ue_max(uint32_t maxv, const char* what) {
    if (maxv > 0x7fffffffu) maxv = 0x7fffffffu;
    const uint32_t v = get_ue();
    if (v > maxv) throw std::runtime_error(std::string(what) + " out of range");
    return static_cast<int>(v);
  }
  int get_se_range(int lo, int hi, const char* what) {
    const uint32_t k = get_ue();
    // se(v) magnitude is ceil(k / 2); compare in 64 bits before forming the signed value
    const int64_t v = (k & 1) ? static_cast<int64_t>(k / 2) + 1 : -static_cast<int64_t>(k / 2);
    if (v < lo || v > hi) throw std::runtime_error(std::string(what) + " out of range");
    return static_cast<int>(v);
  }
  uint32_t get_te(uint32_t range) { return range == 1 ? !get_bit() : get_ue(); }
  bool byte_aligned() const { return (pos_ & 7) == 0; }
  size_t pos() const { return pos_; }
  size_t size_bits() const { return n_ * 8; }
  // more_rbsp_data(): true if there is more data before the rbsp_stop_one_bit.
  bool more_rbsp_data() const {
    if (pos_ >= n_ * 8) return false;
    // find last 1 bit in the buffer (the stop bit)
    size_t last = n_;
    while (last > 0 && p_[last - 1] == 0) --last;
    if (last == 0) return false;
    uint8_t b = p_[last - 1];
    int tz = 0;
    while (((b >> tz) & 1) == 0) ++tz;
    size_t stop_pos = (last - 1) * 8 + (7 - tz);
    return pos_ < stop_pos;
  }
  const uint8_t* data() const { return p_; }

 private:
  const uint8_t* p_;
  size_t n_;
  size_t pos_ = 0;
};

// NAL unit: header byte + RBSP with emulation prevention (clause 7.4.1), prefixed
// by a 4-byte Annex-B start code.
inline void append_nal(std::vector<uint8_t>& out, int nal_ref_idc, int nal_unit_type,
                       const std::vector<uint8_t>& rbsp) {
  static const uint8_t sc[4] = {0, 0, 0, 1};
  out.insert(out.end(), sc, sc + 4);
  out.push_back(static_cast<uint8_t>(((nal_ref_idc & 3) << 5) | (nal_unit_type & 31)));
  int zeros = 0;
  for (uint8_t b : rbsp) {
    if (zeros >= 2 && b <= 3) {
      out.push_back(3);
      zeros = 0;
    }
    out.push_back(b);
    zeros = (b == 0) ? zeros + 1 : 0;
  }
}

struct NalUnit {
  int nal_ref_idc = 0;
  int nal_unit_type = 0;
  size_t offset = 0;       // offset of the start code in the Annex-B stream
  size_t size = 0;         // bytes incl. start code
  std::vector<uint8_t> rbsp;  // payload with emulation-prevention bytes removed
  std::vector<uint32_t> epb;  // rbsp index of the byte each removed emulation-prevention byte preceded
};

// Split an Annex-B byte stream into NAL units (B.2) and unescape the payloads.
inline std::vector<NalUnit> parse_annexb(const uint8_t* p, size_t n, bool unescape = true) {
  std::vector<NalUnit> out;
  std::vector<size_t> starts;      // position of first payload byte
  std::vector<size_t> sc_starts;   // position of start code
  size_t i = 0;
  while (i + 3 <= n) {
    if (p[i] == 0 && p[i + 1] == 0 && p[i + 2] == 1) {
      size_t s = i;
      if (s > 0 && p[s - 1] == 0) s -= 1;  // 4-byte start code
      sc_starts.push_back(s);
      starts.push_back(i + 3);
      i += 3;
    } else {
      ++i;
    }
  }
  for (size_t k = 0; k < starts.size(); ++k) {
    size_t b = starts[k];
    size_t e = (k + 1 < starts.size()) ? sc_starts[k + 1] : n;
    while (e > b && p[e - 1] == 0) --e;  // trailing_zero_8bits
    if (e <= b) continue;
    NalUnit u;
    u.offset = sc_starts[k];
    u.size = ((k + 1 < starts.size()) ? sc_starts[k + 1] : n) - sc_starts[k];
    u.nal_ref_idc = (p[b] >> 5) & 3;
    u.nal_unit_type = p[b] & 31;
    if (unescape) {
      u.rbsp.reserve(e - b);
      int zeros = 0;
      for (size_t j = b + 1; j < e; ++j) {
        uint8_t c = p[j];
        if (zeros >= 2 && c == 3) {
          zeros = 0;
          u.epb.push_back(static_cast<uint32_t>(u.rbsp.size()));
          continue;
        }
        u.rbsp.push_back(c);
        zeros = (c == 0) ? zeros + 1 : 0;
      }
    }
    out.push_back(std::move(u));
  }
  return out;
}

}  // namespace mivc
