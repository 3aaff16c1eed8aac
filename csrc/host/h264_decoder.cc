// Independent H.264 decoder -- see h264_decoder.h.  Clause numbers refer to
// ITU-T H.264 (04/2017).  Constrained Baseline, Main and High profiles (progressive,
// 8-bit 4:2:0): CAVLC and CABAC, I/P/B slices, 4x4 and 8x8 transforms, Intra4x4/8x8/
// 16x16, all partition sizes, multiple references with list modification, spatial and
// temporal direct prediction, explicit and implicit weighted prediction, POC types
// 0/1/2, sliding-window and MMCO reference marking, output in display order.
//
// It shares only constant tables with the encoder side (the CABAC writer in
// csrc/common/h264_cabac.h, the GPU kernels): every parsing rule, context selection,
// prediction and transform here is written separately from the spec, so an
// encoder/decoder round trip checks one against the other.
#include "h264_decoder.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "../common/h264_cabac_tables.h"
#include "../common/h264_mb.h"
#include "../common/h264_tables.h"

namespace mivc {
namespace h264 {

std::vector<uint8_t> DecodedPicture::cropped_i420() const {
  std::vector<uint8_t> o(static_cast<size_t>(width) * height * 3 / 2);
  uint8_t* dst = o.data();
  for (int yy = 0; yy < height; ++yy)
    std::memcpy(dst + static_cast<size_t>(yy) * width, y.data() + static_cast<size_t>(yy + crop_y) * coded_width + crop_x,
                width);
  dst += static_cast<size_t>(width) * height;
  int cw = coded_width / 2, w2 = width / 2, h2 = height / 2;
  for (int yy = 0; yy < h2; ++yy)
    std::memcpy(dst + static_cast<size_t>(yy) * w2, u.data() + static_cast<size_t>(yy + crop_y / 2) * cw + crop_x / 2, w2);
  dst += static_cast<size_t>(w2) * h2;
  for (int yy = 0; yy < h2; ++yy)
    std::memcpy(dst + static_cast<size_t>(yy) * w2, v.data() + static_cast<size_t>(yy + crop_y / 2) * cw + crop_x / 2, w2);
  return o;
}

std::vector<uint16_t> DecodedPicture::cropped_i420_16() const {
  std::vector<uint16_t> o(static_cast<size_t>(width) * height * 3 / 2);
  uint16_t* dst = o.data();
  const int cw = coded_width / 2, w2 = width / 2, h2 = height / 2;
  for (int yy = 0; yy < height; ++yy)
    std::memcpy(dst + static_cast<size_t>(yy) * width, y16.data() + static_cast<size_t>(yy + crop_y) * coded_width + crop_x,
                width * sizeof(uint16_t));
  dst += static_cast<size_t>(width) * height;
  for (const std::vector<uint16_t>* pl : {&u16, &v16}) {
    for (int yy = 0; yy < h2; ++yy)
      std::memcpy(dst + static_cast<size_t>(yy) * w2, pl->data() + static_cast<size_t>(yy + crop_y / 2) * cw + crop_x / 2,
                  w2 * sizeof(uint16_t));
    dst += static_cast<size_t>(w2) * h2;
  }
  return o;
}

namespace {

struct Pic {
  int wmb = 0, hmb = 0, W = 0, H = 0;
  int frame_num = 0, frame_num_wrap = 0, poc = 0, idr = 0, slice_type = 0, id = 0, nal_ref = 0;
  bool short_ref = false, long_ref = false;
  int long_idx = -1;
  bool mmco5 = false;
  std::vector<uint16_t> Y, U, V;  // samples of BitDepthY / BitDepthC bits
  std::vector<int> slice;        // per MB slice index, -1 = not decoded
  std::vector<int8_t> kind, qp, qp_dbk, t8x8, skip, chroma_mode;
  std::vector<uint8_t> cbp, direct;  // direct: bit q = quadrant predicted in direct mode
  std::vector<uint8_t> tc;       // [mb][24] TotalCoeff (luma blkIdx 0-15, Cb 4, Cr 4)
  std::vector<uint8_t> nz;       // [mb][16] raster: luma 4x4 (or its 8x8) has non-zero levels
  std::vector<uint8_t> i4;       // [mb][16] raster intra NxN pred mode
  std::vector<uint16_t> cbf_luma;          // [mb] CABAC coded_block_flag, raster bits
  std::vector<uint8_t> cbf_dc, cbf_cac0, cbf_cac1;
  std::vector<int8_t> ref[2];    // [mb][16] raster ref idx, -1 = list unused
  std::vector<int> refpic[2];    // [mb][16] referenced picture id, -1
  std::vector<int16_t> mv[2];    // [mb][16][2]
  std::vector<uint8_t> mvd[2];   // [mb][16][2] min(|mvd|, 255) (CABAC contexts)
  std::vector<uint8_t> rec_hdr;  // parse-only records
  std::vector<int16_t> rec_coef;
  std::vector<uint32_t> rec_mask, rec_off;
  std::vector<int16_t> rec_sub;  // parse-only: kSubEntry int16 per MB with sub-8x8 motion
  bool gpu_ok = true;
  int nslices = 0;
  int slice_qp = 0;
  std::vector<int32_t> list_ids;  // parse-only: reference lists of the (single) slice
  std::vector<int16_t> wp;
  int inited_w = -1, inited_h = -1;  // per-MB arrays sized (and in their default state) for
  void init(int w, int h, bool planes) {
    wmb = w;
    hmb = h;
    W = w * 16;
    H = h * 16;
    size_t n = static_cast<size_t>(w) * h;
    if (!planes && w == inited_w && h == inited_h) {
      // a pooled picture of the same size (parse-only): every MB the new picture decodes is
      // reset by begin_mb, the others by reset_undecoded() when it completes -- the same
      // state as the fills below without streaming ~400 bytes per MB through the cache
      slice.assign(n, -1);
      return;
    }
    inited_w = planes ? -1 : w;
    inited_h = planes ? -1 : h;
    if (planes) {
      Y.assign(static_cast<size_t>(W) * H, 0);
      U.assign(static_cast<size_t>(W / 2) * (H / 2), 0);
      V.assign(U.size(), 0);
    }
    slice.assign(n, -1);
    kind.assign(n, 0);
    qp.assign(n, 0);
    qp_dbk.assign(n, 0);
    t8x8.assign(n, 0);
    skip.assign(n, 0);
    chroma_mode.assign(n, 0);
    cbp.assign(n, 0);
    direct.assign(n, 0);
    tc.assign(n * 24, 0);
    nz.assign(n * 16, 0);
    i4.assign(n * 16, 2);
    cbf_luma.assign(n, 0);
    cbf_dc.assign(n, 0);
    cbf_cac0.assign(n, 0);
    cbf_cac1.assign(n, 0);
    for (int l = 0; l < 2; ++l) {
      ref[l].assign(n * 16, -1);
      refpic[l].assign(n * 16, -1);
      mv[l].assign(n * 32, 0);
      mvd[l].assign(n * 32, 0);
    }
  }
  void init_records() {
    size_t n = static_cast<size_t>(wmb) * hmb;
    rec_hdr.assign(n * sizeof(MbHeader), 0);
    rec_mask.assign(n, 0);
    rec_off.assign(n, 0);
    rec_coef.clear();
    rec_coef.reserve(n * 64);
    rec_sub.clear();
  }
  int px(int x, int y) const { return Y[static_cast<size_t>(y) * W + x]; }
  // back to the default state, keeping the vectors' storage (picture pool)
  void reset_scalars() {
    frame_num = frame_num_wrap = poc = idr = slice_type = id = nal_ref = 0;
    short_ref = long_ref = false;
    long_idx = -1;
    mmco5 = false;
    gpu_ok = true;
    nslices = 0;
    slice_qp = 0;
    list_ids.clear();
    wp.clear();
  }
};
using PicPtr = std::shared_ptr<Pic>;

struct SliceParams {
  int disable_idc = 0, alpha_off = 0, beta_off = 0;
  int cb_off = 0, cr_off = 0;
};

inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
inline int clip_px(int v, int maxv) { return v < 0 ? 0 : (v > maxv ? maxv : v); }
inline int med3(int a, int b, int c) { return std::max(std::min(a, b), std::min(std::max(a, b), c)); }

// --- independent implementations of the normative arithmetic ------------------
// 8.5.12.2 (rows, then columns, then +32 >> 6)
void idct4(int* b) {
  int t[16];
  for (int r = 0; r < 4; ++r) {
    const int* s = b + 4 * r;
    int a0 = s[0] + s[2];
    int a1 = s[0] - s[2];
    int a2 = (s[1] >> 1) - s[3];
    int a3 = s[1] + (s[3] >> 1);
    t[4 * r + 0] = a0 + a3;
    t[4 * r + 1] = a1 + a2;
    t[4 * r + 2] = a1 - a2;
    t[4 * r + 3] = a0 - a3;
  }
  for (int c = 0; c < 4; ++c) {
    int a0 = t[c] + t[8 + c];
    int a1 = t[c] - t[8 + c];
    int a2 = (t[4 + c] >> 1) - t[12 + c];
    int a3 = t[4 + c] + (t[12 + c] >> 1);
    b[c] = (a0 + a3 + 32) >> 6;
    b[4 + c] = (a1 + a2 + 32) >> 6;
    b[8 + c] = (a1 - a2 + 32) >> 6;
    b[12 + c] = (a0 - a3 + 32) >> 6;
  }
}
// 8.5.13.2: one 8-point pass of the inverse 8x8 transform (in/out stride s)
void idct8_1d(int* d, int s) {
  int d0 = d[0], d1 = d[s], d2 = d[2 * s], d3 = d[3 * s], d4 = d[4 * s], d5 = d[5 * s], d6 = d[6 * s], d7 = d[7 * s];
  int a0 = d0 + d4, a4 = d0 - d4, a2 = (d2 >> 1) - d6, a6 = d2 + (d6 >> 1);
  int b0 = a0 + a6, b2 = a4 + a2, b4 = a4 - a2, b6 = a0 - a6;
  int a1 = -d3 + d5 - d7 - (d7 >> 1);
  int a3 = d1 + d7 - d3 - (d3 >> 1);
  int a5 = -d1 + d7 + d5 + (d5 >> 1);
  int a7 = d3 + d5 + d1 + (d1 >> 1);
  int b1 = a1 + (a7 >> 2), b7 = a7 - (a1 >> 2), b3 = a3 + (a5 >> 2), b5 = (a3 >> 2) - a5;
  d[0] = b0 + b7;
  d[s] = b2 + b5;
  d[2 * s] = b4 + b3;
  d[3 * s] = b6 + b1;
  d[4 * s] = b6 - b1;
  d[5 * s] = b4 - b3;
  d[6 * s] = b2 - b5;
  d[7 * s] = b0 - b7;
}
void idct8(int* b) {
  for (int r = 0; r < 8; ++r) idct8_1d(b + 8 * r, 1);
  for (int c = 0; c < 8; ++c) idct8_1d(b + c, 8);
  for (int i = 0; i < 64; ++i) b[i] = (b[i] + 32) >> 6;
}
// LevelScale4x4 = weightScale4x4 * normAdjust4x4 (8.5.9); w = the scaling-list weight of
// position (x, y) (16 = flat)
int level_scale(int qp_mod6, int x, int y, int w = 16) {
  static const int v[6][3] = {{10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};
  int cls = ((x & 1) == 0 && (y & 1) == 0) ? 0 : (((x & 1) == 1 && (y & 1) == 1) ? 1 : 2);
  return w * v[qp_mod6][cls];
}
// LevelScale8x8 = weightScale8x8 * normAdjust8x8 (8.5.9, eq. 8-318)
int level_scale8(int qp_mod6, int x, int y, int w = 16) {
  static const int v[6][6] = {{20, 18, 32, 19, 25, 24}, {22, 19, 35, 21, 28, 26}, {26, 23, 42, 24, 33, 31},
                              {28, 25, 45, 26, 35, 33}, {32, 28, 51, 30, 40, 38}, {36, 32, 58, 34, 46, 43}};
  int k;
  if (x % 4 == 0 && y % 4 == 0) k = 0;
  else if (x % 2 == 1 && y % 2 == 1) k = 1;
  else if (x % 4 == 2 && y % 4 == 2) k = 2;
  else if ((x % 4 == 0 && y % 2 == 1) || (x % 2 == 1 && y % 4 == 0)) k = 3;
  else if ((x % 4 == 0 && y % 4 == 2) || (x % 4 == 2 && y % 4 == 0)) k = 4;
  else k = 5;
  return w * v[qp_mod6][k];
}
// 8.5.12.1 scaling of one AC/4x4 coefficient (w4: the block's scaling list, raster)
int scale4(int c, int qp, int x, int y, const uint8_t* w4) {
  int ls = level_scale(qp % 6, x, y, w4[y * 4 + x]);
  if (qp >= 24) return (c * ls) << (qp / 6 - 4);
  return (c * ls + (1 << (3 - qp / 6))) >> (4 - qp / 6);
}
// 8.5.13.1 scaling of one 8x8 coefficient
int scale8(int c, int qp, int x, int y, const uint8_t* w8) {
  int ls = level_scale8(qp % 6, x, y, w8[y * 8 + x]);
  if (qp >= 36) return (c * ls) << (qp / 6 - 6);
  return (c * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
}

// CAVLC VLC lookup by peeking
int read_vlc(BitReader& br, const uint8_t* lens, const uint8_t* bits, int n) {
  uint32_t pk = br.peek(16);
  for (int i = 0; i < n; ++i) {
    int l = lens[i];
    if (!l) continue;
    if ((pk >> (16 - l)) == bits[i]) {
      br.skip(l);
      return i;
    }
  }
  throw std::runtime_error("invalid VLC code");
}

// ---------------------------------------------------------------- CABAC decoding engine (9.3.1.2, 9.3.3.2)
struct CabacDec {
  // The 9.3.3.2 engine (codIRange / codIOffset, spec arithmetic) over a direct view of the
  // slice data: renormalisation takes all its bits in one read (count of leading zeros of the
  // range) from a big-endian 64-bit window instead of bit by bit through BitReader (the host
  // parse of the transcode path was bound by that).  `pos` is the exact bit position of the
  // next unread bit; BitReader is re-synchronised when the engine hands the stream back
  // (end of slice, I_PCM samples).
  BitReader* br = nullptr;
  const uint8_t* data = nullptr;
  size_t nbytes = 0, pos = 0;
  uint32_t range = 510, offset = 0;
  uint8_t st[kCabacContexts];
  // n (1..25) bits at pos; zeros past the end (malformed streams only)
  uint32_t read_bits(int n) {
    const size_t byte = pos >> 3;
    uint64_t w;
    if (byte + 8 <= nbytes) {
      std::memcpy(&w, data + byte, 8);
      w = __builtin_bswap64(w);
    } else {
      w = 0;
      for (int k = 0; k < 8; ++k) w |= static_cast<uint64_t>(byte + k < nbytes ? data[byte + k] : 0) << (56 - 8 * k);
    }
    const uint32_t v = static_cast<uint32_t>((w << (pos & 7)) >> (64 - n));
    pos += static_cast<size_t>(n);
    return v;
  }
  void init_engine() {
    data = br->data();
    nbytes = br->size_bits() / 8;
    pos = br->pos();
    range = 510;
    offset = read_bits(9);
    if (offset == 510 || offset == 511) throw std::runtime_error("CABAC: bad initial codIOffset");
  }
  void renorm() {  // range in [2, 255]: shift it back to [256, 510] in one step
    const int n = __builtin_clz(range) - 23;
    range <<= n;
    offset = (offset << n) | read_bits(n);
  }
  // next state (pStateIdx << 1 | valMPS) after an MPS / an LPS, 9.3.3.2.1.1 (Table 9-45)
  struct NextState {
    uint8_t mps[128], lps[128];
    NextState() {
      for (int s = 0; s < 128; ++s) {
        const int pst = s >> 1, m = s & 1;
        mps[s] = static_cast<uint8_t>(((pst < 62 ? pst + 1 : 62) << 1) | m);
        lps[s] = static_cast<uint8_t>((kCabacTransLPS[pst] << 1) | (pst == 0 ? 1 - m : m));
      }
    }
  };
  static const NextState& next_state() {
    static const NextState t;
    return t;
  }
  // DecodeDecision without a data-dependent branch (the bin is unpredictable): the MPS / LPS
  // outcome selects offset, range and state by conditional moves
  int decision(int ctx) {
    const int s = st[ctx];
    const uint32_t rlps = kCabacRangeLPS[s >> 1][(range >> 6) & 3];
    const uint32_t rmps = range - rlps;
    const bool lps = offset >= rmps;
    offset = lps ? offset - rmps : offset;
    range = lps ? rlps : rmps;
    const NextState& ns = next_state();
    st[ctx] = lps ? ns.lps[s] : ns.mps[s];
    if (range < 256) renorm();
    return (s & 1) ^ static_cast<int>(lps);
  }
  int bypass() {
    offset = (offset << 1) | read_bits(1);
    if (offset >= range) {
      offset -= range;
      return 1;
    }
    return 0;
  }
  int terminate() {
    range -= 2;
    if (offset >= range) {
      br->seek(pos);  // the stream continues with BitReader (PCM samples / trailing bits)
      return 1;
    }
    if (range < 256) renorm();
    return 0;
  }
  int eg(int k) {  // exp-Golomb suffix, bypass bins
    int v = 0;
    for (int guard = 0; bypass(); ++guard) {
      if (guard > 30) throw std::runtime_error("CABAC: bad exp-Golomb prefix");
      v += 1 << k;
      ++k;
    }
    while (k--) v += bypass() << k;
    return v;
  }
};

// per-MB parse result (entropy-coding independent)
struct MbSyn {
  int btype = 0;           // B mb_type value (Table 7-14), 0 = B_Direct_16x16
  int sub[4] = {0, 0, 0, 0};
  int i16_mode = 0, chroma_mode = 0, cbp = 0, t8x8 = 0;
  int i4[16];              // blkIdx order (I8x8: the mode in all four entries of each 8x8)
  int refidx[2][4];
  int mvd[2][4][4][2];     // [list][mbPart][subPart][comp]
  int lum[16][16];
  int lum8[4][64];
  int lumdc[16];
  int cdc[2][4];
  int cac[2][4][16];
};

// sub_mb_type (Tables 7-17 / 7-18): parts, width, height in 4x4 units, pred flags (bit0 L0, bit1 L1)
struct SubInfo {
  int nparts, w4, h4, pred;
};
const SubInfo kBSub[13] = {{4, 1, 1, 0}, {1, 2, 2, 1}, {1, 2, 2, 2}, {1, 2, 2, 3}, {2, 2, 1, 1}, {2, 1, 2, 1}, {2, 2, 1, 2},
                           {2, 1, 2, 2}, {2, 2, 1, 3}, {2, 1, 2, 3}, {4, 1, 1, 1}, {4, 1, 1, 2}, {4, 1, 1, 3}};
const SubInfo kPSub[4] = {{1, 2, 2, 1}, {2, 2, 1, 1}, {2, 1, 2, 1}, {4, 1, 1, 1}};
// B mb_type 0..21 (Table 7-14): partition shape (0 16x16, 1 16x8, 2 8x16), pred of part 0 / 1
struct BType {
  int shape, p0, p1;
};
const BType kBType[22] = {{0, 0, 0}, {0, 1, 0}, {0, 2, 0}, {0, 3, 0}, {1, 1, 1}, {2, 1, 1}, {1, 2, 2}, {2, 2, 2},
                          {1, 1, 2}, {2, 1, 2}, {1, 2, 1}, {2, 2, 1}, {1, 1, 3}, {2, 1, 3}, {1, 2, 3}, {2, 2, 3},
                          {1, 3, 1}, {2, 3, 1}, {1, 3, 2}, {2, 3, 2}, {1, 3, 3}, {2, 3, 3}};

}  // namespace

struct Decoder::Impl {
  SPS sps[32];
  PPS pps[256];
  bool have_sps[32] = {}, have_pps[256] = {};
  PicPtr cur;
  int cur_frame_num = -1, cur_pps = -1, cur_idr_id = -1, cur_poc_lsb = -1;
  std::vector<SliceParams> slices;
  std::vector<PicPtr> dpb;      // reference pictures (short- and long-term)
  std::vector<PicPtr> pending;  // decoded, not yet output (display order)
  std::vector<DecodedPicture>* out_ = nullptr;
  int next_pic_id = 1;
  int crop[4] = {0, 0, 0, 0};
  int max_frame_num = 16;
  bool skip_deblock = false;
  bool parse_only = false;
  // sample bit depths of the active SPS (High 10 and up: 9..14 bits; 7.4.2.1.1) and the QP
  // range extension QpBdOffset = 6 * (BitDepth - 8) (7-4, 7-6)
  int bdY = 8, bdC = 8, maxY = 255, maxC = 255, qpbdY = 0, qpbdC = 0;
  int clipY(int v) const { return clip_px(v, maxY); }
  int clipC(int v) const { return clip_px(v, maxC); }
  // QPc (8.5.8, Table 8-15) for a luma QP and offset: qPI = Clip3(-QpBdOffsetC, 51, QPY + offset)
  int qpc_of(int qpy, int off) const {
    const int qpi = clampi(qpy + off, -qpbdC, 51);
    return qpi < 0 ? qpi : chroma_qp(qpi, 0);
  }
  // POC state (8.2.1)
  int prev_poc_msb = 0, prev_poc_lsb = 0, prev_frame_num_offset = 0, prev_frame_num = 0, frame_num_offset = 0;
  int poc_msb = 0;

  // per-slice state
  SliceHeader sh;
  const PPS* pp = nullptr;
  const SPS* sp = nullptr;
  int slice_idx = 0;
  std::vector<PicPtr> list[2];
  CabacDec cab;
  bool cabac = false;
  int prev_qp_delta_nz = 0;
  int implicit_w[32][32][2];  // implicit bi-prediction weights [refIdxL0][refIdxL1]
  int pic_ref_id = -1;

  // per-MB scratch
  int blk_done[16];  // current MB: 4x4 block (raster) available (decoded / MV assigned)
  int blk_tmp[16];

  // ------------------------------------------------------------ neighbours (6.4.11/6.4.12)
  bool mb_ok(int addr) const { return addr >= 0 && cur->slice[addr] == slice_idx; }
  int mbA(int addr) const { return (addr % cur->wmb) > 0 && mb_ok(addr - 1) ? addr - 1 : -1; }
  int mbB(int addr) const { return addr >= cur->wmb && mb_ok(addr - cur->wmb) ? addr - cur->wmb : -1; }
  // luma location (xN,yN) relative to the current MB -> (mbaddr, raster 4x4 index); -1 if unavailable.
  int nb_loc(int addr, int xN, int yN, int* blk) const {
    int mx = addr % cur->wmb, my = addr / cur->wmb;
    int n;
    if (yN < 0) {
      if (my == 0) return -1;
      if (xN < 0) n = mx > 0 ? addr - cur->wmb - 1 : -1;
      else if (xN < 16) n = addr - cur->wmb;
      else n = mx < cur->wmb - 1 ? addr - cur->wmb + 1 : -1;
    } else if (yN < 16) {
      if (xN < 0) n = mx > 0 ? addr - 1 : -1;
      else if (xN < 16) n = addr;
      else return -1;
    } else {
      return -1;
    }
    if (n < 0) return -1;
    int xW = (xN + 16) & 15, yW = (yN + 16) & 15;
    *blk = (xW >> 2) + 4 * (yW >> 2);
    if (n == addr) return blk_done[*blk] ? n : -1;
    return mb_ok(n) ? n : -1;
  }
  // neighbour lookup that ignores the decoding progress inside the current MB
  int nb_any(int addr, int xN, int yN, int* blk) {
    for (int i = 0; i < 16; ++i) blk_tmp[i] = blk_done[i];
    for (int i = 0; i < 16; ++i) blk_done[i] = 1;
    int n = nb_loc(addr, xN, yN, blk);
    for (int i = 0; i < 16; ++i) blk_done[i] = blk_tmp[i];
    return n;
  }
  bool is_intra(int n) const { return mbk_is_intra(cur->kind[n]); }

  // ------------------------------------------------------------ output (C.4.5.3-style bumping)
  void output_ready(bool all) {
    int depth = 0;
    if (sp) depth = sp->vui_reorder_present ? sp->max_num_reorder : (sp->poc_type == 2 ? 0 : 16);
    std::stable_sort(pending.begin(), pending.end(), [](const PicPtr& a, const PicPtr& b) { return a->poc < b->poc; });
    while (!pending.empty() && (all || static_cast<int>(pending.size()) > depth)) {
      emit(*pending.front());
      pending.erase(pending.begin());
    }
  }
  void fill_common(DecodedPicture& d, const Pic& p, bool side_info = true) const {
    d.coded_width = p.W;
    d.coded_height = p.H;
    d.crop_x = crop[0] * 2;
    d.crop_y = crop[2] * 2;
    d.width = p.W - 2 * (crop[0] + crop[1]);
    d.height = p.H - 2 * (crop[2] + crop[3]);
    d.frame_num = p.frame_num;
    d.poc = p.poc;
    d.idr = p.idr;
    d.slice_type = p.slice_type;
    if (!side_info) return;
    d.mb_kind = p.kind;
    d.mb_qp = p.qp;
    d.mv = p.mv[0];
    d.ref = p.ref[0];
    d.nz = p.nz;
  }
  void emit(const Pic& p) {
    DecodedPicture d;
    fill_common(d, p);
    d.bit_depth = bdY;
    if (bdY == 8 && bdC == 8) {
      d.y.assign(p.Y.begin(), p.Y.end());
      d.u.assign(p.U.begin(), p.U.end());
      d.v.assign(p.V.begin(), p.V.end());
    } else {
      d.y16 = p.Y;
      d.u16 = p.U;
      d.v16 = p.V;
    }
    out_->push_back(std::move(d));
  }

  // MBs no slice of the picture covered get the default per-MB state (Pic::init's fills)
  void reset_undecoded() {
    const int n = cur->wmb * cur->hmb;
    for (int a = 0; a < n; ++a) {
      if (cur->slice[a] >= 0) continue;
      const int keep = cur->slice[a];
      begin_mb(a);
      cur->slice[a] = keep;
      cur->kind[a] = 0;
      cur->qp[a] = 0;
      cur->qp_dbk[a] = 0;
    }
  }

  void finish_picture(std::vector<DecodedPicture>& out) {
    out_ = &out;
    if (!cur) return;
    reset_undecoded();
    if (!skip_deblock && !parse_only) deblock_picture();
    if (parse_only) {
      DecodedPicture d;
      fill_common(d, *cur, false);
      d.hdr = std::move(cur->rec_hdr);
      d.coef = std::move(cur->rec_coef);
      d.blk_mask = std::move(cur->rec_mask);
      d.blk_off = std::move(cur->rec_off);
      d.slice_qp = cur->slice_qp;
      d.pic_id = cur->id;
      d.ref_id = pic_ref_id;
      d.nal_ref = cur->nal_ref != 0;
      // several slices reconstruct on the GPU when they share what the kernels take per
      // picture: reference lists / weights (checked as each slice starts), the filter offsets
      // of the filtered slices (boundary strengths already carry disable_deblocking_filter_idc
      // 1 / 2 per edge) and the chroma QP offset; MbHeader::pad0 carries the slice for the
      // intra kernel's neighbour availability
      const SliceParams* f = nullptr;
      bool ok = cur->gpu_ok && cur->nslices <= 255 && !cur->mmco5;
      for (const SliceParams& sp2 : slices) {
        ok = ok && sp2.cb_off == sp2.cr_off && sp2.cb_off == slices[0].cb_off;
        if (sp2.disable_idc == 1) continue;
        if (!f) f = &sp2;
        ok = ok && sp2.alpha_off == f->alpha_off && sp2.beta_off == f->beta_off;
      }
      d.alpha_off = f ? f->alpha_off : 0;
      d.beta_off = f ? f->beta_off : 0;
      d.chroma_qp_offset = slices.empty() ? 0 : slices[0].cb_off;
      d.deblock = f != nullptr;
      d.gpu_ok = ok;
      d.poc = cur->poc;
      d.sub = std::move(cur->rec_sub);
      d.list_ids = cur->list_ids.empty() ? std::vector<int32_t>(64, -1) : cur->list_ids;
      d.wp = cur->wp.empty() ? std::vector<int16_t>(kWpEntries, 0) : cur->wp;
      d.bs = boundary_strengths();
      out.push_back(std::move(d));
    }
    if (cur->nal_ref) mark_reference();
    else prev_frame_num_offset = frame_num_offset;
    if (!parse_only) {
      pending.push_back(cur);
      output_ready(false);
    }
    cur.reset();
  }

  void update_frame_num_wrap(int frame_num) {
    for (PicPtr& r : dpb)
      if (r->short_ref) r->frame_num_wrap = r->frame_num > frame_num ? r->frame_num - max_frame_num : r->frame_num;
  }

  // 8.2.5 decoded reference picture marking
  void mark_reference() {
    Pic& p = *cur;
    update_frame_num_wrap(p.frame_num);
    if (p.idr) {
      for (PicPtr& r : dpb) r->short_ref = r->long_ref = false;
      dpb.clear();
      if (sh.long_term_reference) {
        p.long_ref = true;
        p.long_idx = 0;
      } else {
        p.short_ref = true;
      }
    } else if (sh.adaptive_ref_pic_marking) {
      for (const Mmco& m : sh.mmco) {
        if (m.op == 1) {
          int pn = p.frame_num - (m.diff_minus1 + 1);
          for (PicPtr& r : dpb)
            if (r->short_ref && r->frame_num_wrap == pn) r->short_ref = false;
        } else if (m.op == 2) {
          for (PicPtr& r : dpb)
            if (r->long_ref && r->long_idx == m.long_term_pic_num) r->long_ref = false;
        } else if (m.op == 3) {
          int pn = p.frame_num - (m.diff_minus1 + 1);
          for (PicPtr& r : dpb)
            if (r->long_ref && r->long_idx == m.long_term_frame_idx) r->long_ref = false;
          for (PicPtr& r : dpb)
            if (r->short_ref && r->frame_num_wrap == pn) {
              r->short_ref = false;
              r->long_ref = true;
              r->long_idx = m.long_term_frame_idx;
            }
        } else if (m.op == 4) {
          for (PicPtr& r : dpb)
            if (r->long_ref && r->long_idx >= m.max_long_term_frame_idx_plus1) r->long_ref = false;
        } else if (m.op == 5) {
          for (PicPtr& r : dpb) r->short_ref = r->long_ref = false;
          p.mmco5 = true;
        } else if (m.op == 6) {
          for (PicPtr& r : dpb)
            if (r->long_ref && r->long_idx == m.long_term_frame_idx) r->long_ref = false;
          p.long_ref = true;
          p.long_idx = m.long_term_frame_idx;
        }
      }
      if (!p.long_ref) p.short_ref = true;
    } else {
      // sliding window (8.2.5.3)
      int n = 0;
      for (PicPtr& r : dpb) n += r->short_ref || r->long_ref;
      int maxr = std::max(1, sp->max_num_ref_frames);
      while (n >= maxr) {
        PicPtr victim;
        for (PicPtr& r : dpb)
          if (r->short_ref && (!victim || r->frame_num_wrap < victim->frame_num_wrap)) victim = r;
        if (!victim) break;
        victim->short_ref = false;
        --n;
      }
      p.short_ref = true;
    }
    dpb.erase(std::remove_if(dpb.begin(), dpb.end(), [](const PicPtr& r) { return !r->short_ref && !r->long_ref; }),
              dpb.end());
    if (p.mmco5) {
      // the picture behaves as an IDR for later POC / frame_num derivations: everything
      // decoded before it is output first
      for (PicPtr& q : pending) q->poc -= 1 << 30;
      p.poc = 0;
      p.frame_num = 0;
      prev_poc_msb = 0;
      prev_poc_lsb = 0;
      prev_frame_num_offset = 0;
      prev_frame_num = 0;
    } else {
      prev_frame_num_offset = frame_num_offset;
      if (sp->poc_type == 0) {
        prev_poc_msb = poc_msb;
        prev_poc_lsb = sh.poc_lsb;
      }
    }
    dpb.push_back(cur);
  }

  // 8.2.1 picture order count
  int derive_poc(const SliceHeader& h) {
    bool idr = h.nal_unit_type == NAL_IDR;
    if (idr) {
      prev_poc_msb = prev_poc_lsb = 0;
      prev_frame_num_offset = 0;
    }
    if (sp->poc_type == 0) {
      int max_lsb = 1 << sp->log2_max_poc_lsb;
      int lsb = h.poc_lsb;
      if (lsb < prev_poc_lsb && prev_poc_lsb - lsb >= max_lsb / 2) poc_msb = prev_poc_msb + max_lsb;
      else if (lsb > prev_poc_lsb && lsb - prev_poc_lsb > max_lsb / 2) poc_msb = prev_poc_msb - max_lsb;
      else poc_msb = prev_poc_msb;
      return poc_msb + lsb;
    }
    if (idr) frame_num_offset = 0;
    else if (prev_frame_num > h.frame_num) frame_num_offset = prev_frame_num_offset + max_frame_num;
    else frame_num_offset = prev_frame_num_offset;
    if (sp->poc_type == 2) {
      if (idr) return 0;
      return h.nal_ref_idc == 0 ? 2 * (frame_num_offset + h.frame_num) - 1 : 2 * (frame_num_offset + h.frame_num);
    }
    // type 1
    int n = static_cast<int>(sp->offset_for_ref_frame.size());
    int abs_fn = n ? frame_num_offset + h.frame_num : 0;
    if (h.nal_ref_idc == 0 && abs_fn > 0) --abs_fn;
    int exp = 0;
    if (abs_fn > 0) {
      int delta_cycle = 0;
      for (int v : sp->offset_for_ref_frame) delta_cycle += v;
      int cycle = (abs_fn - 1) / n, in_cycle = (abs_fn - 1) % n;
      exp = cycle * delta_cycle;
      for (int i = 0; i <= in_cycle; ++i) exp += sp->offset_for_ref_frame[i];
    }
    if (h.nal_ref_idc == 0) exp += sp->offset_for_non_ref_pic;
    return exp + h.delta_poc[0];
  }

  // pictures nobody holds any more are reused: their per-MB arrays keep their storage
  // (no allocation + page faults for ~13 MB of side info per 4K picture)
  std::vector<PicPtr> pic_pool;
  PicPtr new_pic() {
    for (PicPtr& p : pic_pool)
      if (p.use_count() == 1) {
        p->reset_scalars();
        return p;
      }
    auto p = std::make_shared<Pic>();
    if (pic_pool.size() < 40) pic_pool.push_back(p);
    return p;
  }

  void start_picture(const SliceHeader& h) {
    bdY = sp->bit_depth_luma;
    bdC = sp->bit_depth_chroma;
    maxY = (1 << bdY) - 1;
    maxC = (1 << bdC) - 1;
    qpbdY = 6 * (bdY - 8);
    qpbdC = 6 * (bdC - 8);
    cur = new_pic();
    cur->init(sp->width_mbs, sp->height_mbs, !parse_only);
    if (bdY != 8 || bdC != 8) cur->gpu_ok = false;  // the GPU reconstruction kernels are 8-bit
    if (parse_only) cur->init_records();
    cur->slice_qp = h.qp;
    pic_ref_id = -1;
    max_frame_num = 1 << sp->log2_max_frame_num;
    if (h.nal_unit_type == NAL_IDR) {
      if (!parse_only) output_ready(true);
      for (PicPtr& r : dpb) r->short_ref = r->long_ref = false;
      dpb.clear();
    }
    cur->frame_num = h.frame_num;
    cur->idr = h.nal_unit_type == NAL_IDR;
    cur->slice_type = h.slice_type;
    cur->nal_ref = h.nal_ref_idc;
    cur->id = next_pic_id++;
    cur->poc = derive_poc(h);
    prev_frame_num = h.frame_num;
    cur_frame_num = h.frame_num;
    cur_pps = h.pps_id;
    cur_idr_id = cur->idr ? h.idr_pic_id : -1;
    cur_poc_lsb = h.poc_lsb;
    slices.clear();
    crop[0] = sp->crop_left;
    crop[1] = sp->crop_right;
    crop[2] = sp->crop_top;
    crop[3] = sp->crop_bottom;
  }

  // 8.2.4 reference picture lists
  void build_ref_lists() {
    list[0].clear();
    list[1].clear();
    if (sh.slice_type == SLICE_I) return;
    update_frame_num_wrap(sh.frame_num);
    std::vector<PicPtr> st, lt;
    for (PicPtr& r : dpb) {
      if (r->short_ref) st.push_back(r);
      else if (r->long_ref) lt.push_back(r);
    }
    std::sort(lt.begin(), lt.end(), [](const PicPtr& a, const PicPtr& b) { return a->long_idx < b->long_idx; });
    if (sh.slice_type == SLICE_P) {
      std::sort(st.begin(), st.end(), [](const PicPtr& a, const PicPtr& b) { return a->frame_num_wrap > b->frame_num_wrap; });
      list[0] = st;
      list[0].insert(list[0].end(), lt.begin(), lt.end());
    } else {
      std::vector<PicPtr> before, after;
      for (PicPtr& r : st) (r->poc < cur->poc ? before : after).push_back(r);
      std::sort(before.begin(), before.end(), [](const PicPtr& a, const PicPtr& b) { return a->poc > b->poc; });
      std::sort(after.begin(), after.end(), [](const PicPtr& a, const PicPtr& b) { return a->poc < b->poc; });
      list[0] = before;
      list[0].insert(list[0].end(), after.begin(), after.end());
      list[0].insert(list[0].end(), lt.begin(), lt.end());
      list[1] = after;
      list[1].insert(list[1].end(), before.begin(), before.end());
      list[1].insert(list[1].end(), lt.begin(), lt.end());
      if (list[1].size() > 1 && list[1] == list[0]) std::swap(list[1][0], list[1][1]);
    }
    int nl = sh.slice_type == SLICE_B ? 2 : 1;
    for (int l = 0; l < nl; ++l) {
      int n = l ? sh.num_ref_idx_l1_active : sh.num_ref_idx_l0_active;
      if (list[l].empty()) throw std::runtime_error("inter slice without reference pictures");
      // 8.2.4.3 modification
      int pred = sh.frame_num;
      int idx = 0;
      for (const RefMod& m : sh.mods[l]) {
        PicPtr pic;
        if (m.idc < 2) {
          int d = m.value + 1;
          int pn_nowrap = m.idc == 0 ? pred - d : pred + d;
          if (pn_nowrap < 0) pn_nowrap += max_frame_num;
          if (pn_nowrap >= max_frame_num) pn_nowrap -= max_frame_num;
          pred = pn_nowrap;
          int pn = pn_nowrap > sh.frame_num ? pn_nowrap - max_frame_num : pn_nowrap;
          for (PicPtr& r : dpb)
            if (r->short_ref && r->frame_num_wrap == pn) pic = r;
        } else {
          for (PicPtr& r : dpb)
            if (r->long_ref && r->long_idx == m.value) pic = r;
        }
        if (!pic) throw std::runtime_error("ref_pic_list_modification names a missing picture");
        list[l].insert(list[l].begin() + idx, pic);
        for (size_t k = idx + 1; k < list[l].size(); ++k)
          if (list[l][k] == pic) {
            list[l].erase(list[l].begin() + k);
            break;
          }
        ++idx;
      }
      while (static_cast<int>(list[l].size()) < n) list[l].push_back(list[l].back());
      list[l].resize(n);
    }
    // temporal direct (8.4.1.2.3): DistScaleFactor per RefPicList0 entry, once per slice
    tdir_n = 0;
    if (sh.slice_type == SLICE_B && !sh.direct_spatial && !list[1].empty()) {
      const Pic& p1 = *list[1][0];
      tdir_n = std::min<int>(static_cast<int>(list[0].size()), kMaxTdir);
      for (int i = 0; i < tdir_n; ++i) {
        const Pic& p0 = *list[0][i];
        const int tb = clampi(cur->poc - p0.poc, -128, 127), td = clampi(p1.poc - p0.poc, -128, 127);
        tdir_id[i] = p0.id;
        tdir_copy[i] = td == 0 || p0.long_ref;
        if (!tdir_copy[i]) {
          const int tx = (16384 + std::abs(td / 2)) / td;
          tdir_dsf[i] = clampi((tb * tx + 32) >> 6, -1024, 1023);
        }
      }
    }
    // implicit bi-prediction weights (8.4.2.3.1)
    if (sh.slice_type == SLICE_B && pp->weighted_bipred_idc == 2) {
      for (int i = 0; i < sh.num_ref_idx_l0_active; ++i)
        for (int j = 0; j < sh.num_ref_idx_l1_active; ++j) {
          int w0 = 32, w1 = 32;
          const Pic& p0 = *list[0][i];
          const Pic& p1 = *list[1][j];
          int tb = clampi(cur->poc - p0.poc, -128, 127), td = clampi(p1.poc - p0.poc, -128, 127);
          if (td != 0 && !p0.long_ref && !p1.long_ref) {
            int tx = (16384 + std::abs(td / 2)) / td;
            int dsf = clampi((tb * tx + 32) >> 6, -1024, 1023);
            if (!((dsf >> 2) < -64 || (dsf >> 2) > 128)) {
              w0 = 64 - (dsf >> 2);
              w1 = dsf >> 2;
            }
          }
          implicit_w[i][j][0] = w0;
          implicit_w[i][j][1] = w1;
        }
    }
  }

  // ------------------------------------------------------------ slice data
  void decode_slice(const NalUnit& nal, std::vector<DecodedPicture>& out) {
    BitReader br(nal.rbsp.data(), nal.rbsp.size());
    SliceHeader h = parse_slice_header(br, nal.nal_unit_type, nal.nal_ref_idc, sps, pps);
    if (!have_pps[h.pps_id]) throw std::runtime_error("slice references missing PPS");
    const PPS* p = &pps[h.pps_id];
    if (!have_sps[p->sps_id]) throw std::runtime_error("PPS references missing SPS");
    // first VCL NAL unit of a new primary picture (7.4.1.2.4)
    bool new_pic = !cur || h.first_mb == 0 || h.frame_num != cur_frame_num || h.pps_id != cur_pps ||
                   (h.nal_unit_type == NAL_IDR) != (cur && cur->idr) ||
                   (h.nal_unit_type == NAL_IDR && h.idr_pic_id != cur_idr_id) || h.poc_lsb != cur_poc_lsb ||
                   (h.nal_ref_idc != 0) != (cur && cur->nal_ref != 0);
    if (new_pic) finish_picture(out);
    sh = h;
    pp = p;
    sp = &sps[p->sps_id];
    if (new_pic) start_picture(h);
    SliceParams spar;
    spar.disable_idc = h.disable_deblocking_filter_idc;
    spar.alpha_off = h.alpha_offset_div2 * 2;
    spar.beta_off = h.beta_offset_div2 * 2;
    spar.cb_off = p->chroma_qp_index_offset;
    spar.cr_off = p->second_chroma_qp_index_offset;
    slices.push_back(spar);
    slice_idx = static_cast<int>(slices.size()) - 1;
    cur->nslices = static_cast<int>(slices.size());
    if (h.slice_type == SLICE_B) cur->slice_type = SLICE_B;
    else if (h.slice_type == SLICE_P && cur->slice_type == SLICE_I) cur->slice_type = SLICE_P;
    build_ref_lists();
    if (!list[0].empty()) pic_ref_id = list[0][0]->id;
    if (parse_only) record_lists_and_weights();
    cabac = p->entropy_coding_mode != 0;
    int nmb = cur->wmb * cur->hmb;
    int addr = h.first_mb;
    int qp = h.qp;
    if (h.first_mb >= nmb) throw std::runtime_error("first_mb_in_slice past the picture");
    if (qp < -qpbdY || qp > 51) throw std::runtime_error("slice QP out of range");
    if (cabac) {
      while (!br.byte_aligned())  // cabac_alignment_one_bit
        if (!br.get_bit()) throw std::runtime_error("cabac_alignment_one_bit is 0");
      if (h.cabac_init_idc > 2) throw std::runtime_error("bad cabac_init_idc");
      cabac_init_contexts(cab.st, h.slice_type == SLICE_I ? 0 : 1 + h.cabac_init_idc, h.qp);
      cab.br = &br;
      cab.init_engine();
      prev_qp_delta_nz = 0;
      for (;;) {
        if (addr >= nmb) throw std::runtime_error("slice runs past the picture");
        bool skipped = false;
        if (sh.slice_type != SLICE_I) {
          skipped = cabac_skip_flag(addr);
          if (skipped) {
            decode_skip(addr, qp);
            prev_qp_delta_nz = 0;
          }
        }
        if (!skipped) decode_mb(br, addr, qp);
        ++addr;
        if (cab.terminate()) break;  // end_of_slice_flag
      }
      return;
    }
    bool more = true;
    while (more) {
      if (addr >= nmb) throw std::runtime_error("slice runs past the picture");
      if (sh.slice_type != SLICE_I) {
        const int run = br.get_ue_max(static_cast<uint32_t>(nmb), "mb_skip_run");
        for (int i = 0; i < run; ++i) {
          if (addr >= nmb) throw std::runtime_error("skip run past the picture");
          decode_skip(addr, qp);
          ++addr;
        }
        if (run > 0) {
          more = br.more_rbsp_data();
          if (!more) break;
        }
      }
      if (addr >= nmb) throw std::runtime_error("slice runs past the picture");
      decode_mb(br, addr, qp);
      ++addr;
      more = br.more_rbsp_data();
    }
  }

  void begin_mb(int addr) {
    cur->slice[addr] = slice_idx;
    std::memset(blk_done, 0, sizeof(blk_done));
    for (int l = 0; l < 2; ++l) {
      std::memset(&cur->ref[l][addr * 16], 0xFF, 16);
      std::memset(&cur->refpic[l][addr * 16], 0xFF, 16 * sizeof(int));
      std::memset(&cur->mv[l][addr * 32], 0, 32 * sizeof(int16_t));
      std::memset(&cur->mvd[l][addr * 32], 0, 32);
    }
    std::memset(&cur->nz[addr * 16], 0, 16);
    std::memset(&cur->i4[addr * 16], 2, 16);
    std::memset(&cur->tc[addr * 24], 0, 24);
    cur->cbf_luma[addr] = 0;
    cur->cbf_dc[addr] = 0;
    cur->cbf_cac0[addr] = cur->cbf_cac1[addr] = 0;
    cur->t8x8[addr] = 0;
    cur->skip[addr] = 0;
    cur->chroma_mode[addr] = 0;
    cur->cbp[addr] = 0;
    cur->direct[addr] = 0;
  }

  // temporal direct table of the current slice (8.4.1.2.3): RefPicList0 picture ids,
  // DistScaleFactor and the "copy the co-located vector" case (td == 0 or long-term)
  static constexpr int kMaxTdir = 32;
  int tdir_n = 0;
  int tdir_id[kMaxTdir];
  int tdir_dsf[kMaxTdir];
  bool tdir_copy[kMaxTdir];

  // ------------------------------------------------------------ motion vector prediction (8.4.1.3)
  struct NbMv {
    bool avail;
    int ref;
    int mv[2];
  };
  NbMv nb_mv(int addr, int l, int xN, int yN) {
    NbMv r{false, -1, {0, 0}};
    int blk;
    int n = nb_loc(addr, xN, yN, &blk);
    if (n < 0) return r;
    r.avail = true;
    if (is_intra(n) && n != addr) return r;
    r.ref = cur->ref[l][n * 16 + blk];
    if (r.ref >= 0) {
      r.mv[0] = cur->mv[l][n * 32 + 2 * blk];
      r.mv[1] = cur->mv[l][n * 32 + 2 * blk + 1];
    }
    return r;
  }
  // x, y, w: partition geometry in samples; shape 1 16x8, 2 8x16
  void pred_mv(int addr, int l, int x, int y, int w, int shape, int part, int ref, int out[2]) {
    NbMv A = nb_mv(addr, l, x - 1, y);
    NbMv B = nb_mv(addr, l, x, y - 1);
    NbMv C = nb_mv(addr, l, x + w, y - 1);
    if (!C.avail) C = nb_mv(addr, l, x - 1, y - 1);
    if (shape == 1) {
      if (part == 0 && B.ref == ref) { out[0] = B.mv[0]; out[1] = B.mv[1]; return; }
      if (part == 1 && A.ref == ref) { out[0] = A.mv[0]; out[1] = A.mv[1]; return; }
    } else if (shape == 2) {
      if (part == 0 && A.ref == ref) { out[0] = A.mv[0]; out[1] = A.mv[1]; return; }
      if (part == 1 && C.ref == ref) { out[0] = C.mv[0]; out[1] = C.mv[1]; return; }
    }
    if (!B.avail && !C.avail && A.avail) {
      B = A;
      C = A;
    }
    int match = (A.ref == ref) + (B.ref == ref) + (C.ref == ref);
    if (match == 1) {
      const NbMv& m = A.ref == ref ? A : (B.ref == ref ? B : C);
      out[0] = m.mv[0];
      out[1] = m.mv[1];
      return;
    }
    out[0] = med3(A.mv[0], B.mv[0], C.mv[0]);
    out[1] = med3(A.mv[1], B.mv[1], C.mv[1]);
  }
  void assign(int addr, int l, int bx, int by, int w4, int h4, int ref, int mvx, int mvy) {
    if (ref >= static_cast<int>(list[l].size())) throw std::runtime_error("ref_idx beyond the reference list");
    for (int y = by; y < by + h4; ++y)
      for (int x = bx; x < bx + w4; ++x) {
        int r = x + 4 * y;
        cur->ref[l][addr * 16 + r] = static_cast<int8_t>(ref);
        cur->refpic[l][addr * 16 + r] = ref >= 0 ? list[l][ref]->id : -1;
        cur->mv[l][addr * 32 + 2 * r] = static_cast<int16_t>(mvx);
        cur->mv[l][addr * 32 + 2 * r + 1] = static_cast<int16_t>(mvy);
      }
  }
  void mark_done(int bx, int by, int w4, int h4) {
    for (int y = by; y < by + h4; ++y)
      for (int x = bx; x < bx + w4; ++x) blk_done[x + 4 * y] = 1;
  }

  // ------------------------------------------------------------ direct prediction (8.4.1.2)
  // co-located 4x4 block of raster index r in RefPicList1[0] (frames, 8.4.1.2.1)
  void colocated(int addr, int r, int* mvc, int* refc, int* refpic_col) {
    const Pic& col = *list[1][0];
    int rr = r;
    if (sp->direct_8x8_inference) {
      int x = (r & 3) < 2 ? 0 : 3, y = (r >> 2) < 2 ? 0 : 3;
      rr = x + 4 * y;
    }
    if (mbk_is_intra(col.kind[addr])) {
      mvc[0] = mvc[1] = 0;
      *refc = -1;
      *refpic_col = -1;
      return;
    }
    int l = col.ref[0][addr * 16 + rr] >= 0 ? 0 : 1;
    mvc[0] = col.mv[l][addr * 32 + 2 * rr];
    mvc[1] = col.mv[l][addr * 32 + 2 * rr + 1];
    *refc = col.ref[l][addr * 16 + rr];
    *refpic_col = col.refpic[l][addr * 16 + rr];
  }

  // direct motion of the 4x4 blocks in quadrant mask `quads` (bit q) of MB addr
  void direct_pred(int addr, int quads) {
    if (sh.direct_spatial) {
      // 8.4.1.2.2: reference indices and predictors from the MB-level neighbours A, B, C
      int refs[2], pmv[2][2] = {{0, 0}, {0, 0}};
      for (int i = 0; i < 16; ++i) blk_tmp[i] = blk_done[i];
      for (int i = 0; i < 16; ++i) blk_done[i] = 0;
      for (int l = 0; l < 2; ++l) {
        NbMv A = nb_mv(addr, l, -1, 0), B = nb_mv(addr, l, 0, -1), C = nb_mv(addr, l, 16, -1);
        if (!C.avail) C = nb_mv(addr, l, -1, -1);
        auto minpos = [](int a, int b) { return (a >= 0 && b >= 0) ? std::min(a, b) : std::max(a, b); };
        refs[l] = minpos(A.ref, minpos(B.ref, C.ref));
        if (refs[l] >= 0) pred_mv(addr, l, 0, 0, 16, 0, 0, refs[l], pmv[l]);
      }
      for (int i = 0; i < 16; ++i) blk_done[i] = blk_tmp[i];
      bool zero_pred = refs[0] < 0 && refs[1] < 0;
      const Pic& col = *list[1][0];
      // direct_8x8_inference: every 4x4 of a quadrant takes the quadrant's corner co-located
      // block, so the derivation runs once per quadrant on a 2x2 block group
      const int step = sp->direct_8x8_inference ? 2 : 1;
      for (int r = 0; r < 16; r += (step == 2 && (r & 3) == 2) ? 6 : step) {
        int q = ((r & 3) >> 1) + 2 * ((r >> 2) >> 1);
        if (!((quads >> q) & 1)) continue;
        int mvc[2], refc, rpc;
        colocated(addr, r, mvc, &refc, &rpc);
        bool col_zero = !col.long_ref && refc == 0 && std::abs(mvc[0]) <= 1 && std::abs(mvc[1]) <= 1;
        for (int l = 0; l < 2; ++l) {
          if (zero_pred) {
            assign(addr, l, r & 3, r >> 2, step, step, 0, 0, 0);
            continue;
          }
          int ref = refs[l];
          if (ref < 0) {
            assign(addr, l, r & 3, r >> 2, step, step, -1, 0, 0);
            continue;
          }
          if (ref == 0 && col_zero) assign(addr, l, r & 3, r >> 2, step, step, 0, 0, 0);
          else assign(addr, l, r & 3, r >> 2, step, step, ref, pmv[l][0], pmv[l][1]);
        }
      }
      return;
    }
    // 8.4.1.2.3 temporal
    if (sp->direct_8x8_inference && tdir_n > 0) {
      // the common case: one co-located corner block per quadrant, DistScaleFactor from the
      // slice table (the picture is found among RefPicList0's first tdir_n entries)
      const Pic& col = *list[1][0];
      const bool col_intra = mbk_is_intra(col.kind[addr]);
      for (int q = 0; q < 4; ++q) {
        if (!((quads >> q) & 1)) continue;
        const int r = (q & 1) * 2 + (q >> 1) * 8;                    // top-left 4x4 of the quadrant
        const int rr = ((q & 1) ? 3 : 0) + ((q >> 1) ? 12 : 0);      // its co-located corner
        int mvc0 = 0, mvc1 = 0, ref0 = 0;
        if (!col_intra) {
          const int l = col.ref[0][addr * 16 + rr] >= 0 ? 0 : 1;
          mvc0 = col.mv[l][addr * 32 + 2 * rr];
          mvc1 = col.mv[l][addr * 32 + 2 * rr + 1];
          if (col.ref[l][addr * 16 + rr] >= 0) {
            const int rpc = col.refpic[l][addr * 16 + rr];
            ref0 = -1;
            for (int i = 0; i < tdir_n; ++i)
              if (tdir_id[i] == rpc) {
                ref0 = i;
                break;
              }
            if (ref0 < 0) {  // beyond the table: the general path
              ref0 = -2;
            }
          }
        }
        if (ref0 == -2) {
          direct_temporal_general(addr, 1 << q);
          continue;
        }
        int m0x, m0y, m1x, m1y;
        if (tdir_copy[ref0]) {
          m0x = mvc0;
          m0y = mvc1;
          m1x = m1y = 0;
        } else {
          const int dsf = tdir_dsf[ref0];
          m0x = (dsf * mvc0 + 128) >> 8;
          m0y = (dsf * mvc1 + 128) >> 8;
          m1x = m0x - mvc0;
          m1y = m0y - mvc1;
        }
        assign2x2(addr, 0, r, ref0, tdir_id[ref0], m0x, m0y);
        assign2x2(addr, 1, r, 0, list[1][0]->id, m1x, m1y);
      }
      return;
    }
    direct_temporal_general(addr, quads);
  }

  // 2x2 group of 4x4 blocks at raster index r (top-left), list l
  void assign2x2(int addr, int l, int r, int ref, int refid, int mvx, int mvy) {
    int8_t* rf = &cur->ref[l][addr * 16 + r];
    int* rp = &cur->refpic[l][addr * 16 + r];
    int16_t* mv = &cur->mv[l][addr * 32 + 2 * r];
    rf[0] = rf[1] = rf[4] = rf[5] = static_cast<int8_t>(ref);
    rp[0] = rp[1] = rp[4] = rp[5] = refid;
    mv[0] = mv[2] = mv[8] = mv[10] = static_cast<int16_t>(mvx);
    mv[1] = mv[3] = mv[9] = mv[11] = static_cast<int16_t>(mvy);
  }

  void direct_temporal_general(int addr, int quads) {
    const Pic& p1 = *list[1][0];
    const int step = sp->direct_8x8_inference ? 2 : 1;  // as in the spatial case
    for (int r = 0; r < 16; r += (step == 2 && (r & 3) == 2) ? 6 : step) {
      int q = ((r & 3) >> 1) + 2 * ((r >> 2) >> 1);
      if (!((quads >> q) & 1)) continue;
      int mvc[2], refc, rpc;
      colocated(addr, r, mvc, &refc, &rpc);
      int ref0 = 0;
      if (refc >= 0) {
        ref0 = -1;
        for (int i = 0; i < static_cast<int>(list[0].size()); ++i)
          if (list[0][i]->id == rpc) {
            ref0 = i;
            break;
          }
        if (ref0 < 0) throw std::runtime_error("temporal direct: co-located reference not in RefPicList0");
      }
      const Pic& p0 = *list[0][ref0];
      int mv0[2], mv1[2];
      int tb = clampi(cur->poc - p0.poc, -128, 127), td = clampi(p1.poc - p0.poc, -128, 127);
      if (td == 0 || p0.long_ref) {
        mv0[0] = mvc[0];
        mv0[1] = mvc[1];
        mv1[0] = mv1[1] = 0;
      } else {
        int tx = (16384 + std::abs(td / 2)) / td;
        int dsf = clampi((tb * tx + 32) >> 6, -1024, 1023);
        for (int c = 0; c < 2; ++c) {
          mv0[c] = (dsf * mvc[c] + 128) >> 8;
          mv1[c] = mv0[c] - mvc[c];
        }
      }
      assign(addr, 0, r & 3, r >> 2, step, step, ref0, mv0[0], mv0[1]);
      assign(addr, 1, r & 3, r >> 2, step, step, 0, mv1[0], mv1[1]);
    }
  }

  void decode_skip(int addr, int qp) {
    begin_mb(addr);
    cur->skip[addr] = 1;
    cur->qp[addr] = static_cast<int8_t>(qp);
    cur->qp_dbk[addr] = static_cast<int8_t>(qp);
    if (sh.slice_type == SLICE_B) {
      cur->kind[addr] = MBK_BDIRECT;
      cur->direct[addr] = 0xF;
      direct_pred(addr, 0xF);
      mark_done(0, 0, 4, 4);
      if (parse_only) {
        cur->rec_off[addr] = static_cast<uint32_t>(cur->rec_coef.size() / 16);
        store_record(addr, MBK_BDIRECT, 0, qp, 0, 0, nullptr, 0);
        return;
      }
      inter_pred(addr);
      return;
    }
    cur->kind[addr] = MBK_PSKIP;
    int mv[2] = {0, 0};
    NbMv A = nb_mv(addr, 0, -1, 0);
    NbMv B = nb_mv(addr, 0, 0, -1);
    bool zero = !A.avail || !B.avail || (A.ref == 0 && A.mv[0] == 0 && A.mv[1] == 0) ||
                (B.ref == 0 && B.mv[0] == 0 && B.mv[1] == 0);
    if (!zero) pred_mv(addr, 0, 0, 0, 16, 0, 0, 0, mv);
    assign(addr, 0, 0, 0, 4, 4, 0, mv[0], mv[1]);
    mark_done(0, 0, 4, 4);
    if (parse_only) {
      cur->rec_off[addr] = static_cast<uint32_t>(cur->rec_coef.size() / 16);
      store_record(addr, MBK_PSKIP, 0, qp, 0, 0, nullptr, 0);
      return;
    }
    inter_pred(addr);
  }

  // parse-only: MbHeader of MB addr (levels already in the records)
  void store_record(int addr, int kind, int cbp, int qp, int i16_mode, int chroma_mode, const int* i4modes, int t8) {
    MbHeader h{};
    h.kind = static_cast<uint8_t>(kind);
    h.cbp = static_cast<uint8_t>(cbp);
    h.qp = static_cast<int8_t>(qp);
    h.i16_mode = static_cast<uint8_t>(i16_mode);
    h.chroma_mode = static_cast<uint8_t>(chroma_mode);
    h.flags = static_cast<uint8_t>(t8 ? MBF_T8x8 : 0);
    h.sub_direct = cur->direct[addr];
    h.pad0 = static_cast<uint8_t>(slice_idx);  // slice of the MB (GPU intra availability)
    // P_Skip motion is one vector for the MB, B_Skip / B_Direct_16x16 with direct_8x8_inference
    // one per quadrant: no 4x4 scan needed for them (nor for intra MBs)
    const bool known = kind == MBK_PSKIP || mbk_is_intra(kind) || (kind == MBK_BDIRECT && sp->direct_8x8_inference);
    bool quad_uniform = true;
    for (int l = 0; l < 2; ++l)
      for (int q = 0; q < 4; ++q) {
        int r0 = (q & 1) * 2 + (q >> 1) * 8;  // top-left 4x4 block of quadrant q
        const int16_t* m0 = &cur->mv[l][addr * 32 + 2 * r0];
        const int8_t* f0 = &cur->ref[l][addr * 16 + r0];
        h.mv[l][q][0] = m0[0];
        h.mv[l][q][1] = m0[1];
        h.ref[l][q] = f0[0];
        if (known) continue;
        for (int k = 1; k < 4; ++k) {
          int dr = (k & 1) + 4 * (k >> 1);
          quad_uniform = quad_uniform && f0[dr] == f0[0] && m0[2 * dr] == m0[0] && m0[2 * dr + 1] == m0[1];
        }
      }
    if (i4modes) {
      for (int b = 0; b < 16; ++b) h.i4_modes[b] = static_cast<uint8_t>(i4modes[b]);
    } else {
      std::memset(h.i4_modes, 2, 16);
    }
    if (!quad_uniform && !mbk_is_intra(kind)) {
      // motion below 8x8: the whole MB's vectors go to the side pool, i4_modes[0..3] (unused
      // by inter MBs) hold the entry index
      h.flags |= MBF_SUB4;
      uint32_t idx = static_cast<uint32_t>(cur->rec_sub.size() / kSubEntry);
      std::memcpy(h.i4_modes, &idx, 4);
      size_t b0 = cur->rec_sub.size();
      cur->rec_sub.resize(b0 + kSubEntry);
      int16_t* e = cur->rec_sub.data() + b0;
      for (int l = 0; l < 2; ++l)
        for (int r = 0; r < 16; ++r) {
          e[(l * 16 + r) * 2] = cur->mv[l][addr * 32 + 2 * r];
          e[(l * 16 + r) * 2 + 1] = cur->mv[l][addr * 32 + 2 * r + 1];
        }
      int8_t* rf = reinterpret_cast<int8_t*>(e + 64);
      for (int l = 0; l < 2; ++l)
        for (int r = 0; r < 16; ++r) rf[l * 16 + r] = cur->ref[l][addr * 16 + r];
    }
    std::memcpy(cur->rec_hdr.data() + static_cast<size_t>(addr) * sizeof(MbHeader), &h, sizeof(MbHeader));
  }

  // ------------------------------------------------------------ inter prediction (8.4.2)
  static int ref_y(const Pic& r, int x, int y) {
    return r.Y[static_cast<size_t>(clampi(y, 0, r.H - 1)) * r.W + clampi(x, 0, r.W - 1)];
  }
  static int half_h1(const Pic& r, int x, int y) {  // intermediate b1 at (x+1/2, y)
    return tap6(ref_y(r, x - 2, y), ref_y(r, x - 1, y), ref_y(r, x, y), ref_y(r, x + 1, y), ref_y(r, x + 2, y),
                ref_y(r, x + 3, y));
  }
  static int half_v1(const Pic& r, int x, int y) {  // intermediate h1 at (x, y+1/2)
    return tap6(ref_y(r, x, y - 2), ref_y(r, x, y - 1), ref_y(r, x, y), ref_y(r, x, y + 1), ref_y(r, x, y + 2),
                ref_y(r, x, y + 3));
  }
  static int luma_sample(const Pic& r, int xi, int yi, int xf, int yf, int maxv) {
    auto b = [&](int x, int y) { return clip_px((half_h1(r, x, y) + 16) >> 5, maxv); };
    auto h = [&](int x, int y) { return clip_px((half_v1(r, x, y) + 16) >> 5, maxv); };
    auto j = [&](int x, int y) {
      int j1 = tap6(half_h1(r, x, y - 2), half_h1(r, x, y - 1), half_h1(r, x, y), half_h1(r, x, y + 1),
                    half_h1(r, x, y + 2), half_h1(r, x, y + 3));
      return clip_px((j1 + 512) >> 10, maxv);
    };
    int G = ref_y(r, xi, yi);
    switch (yf * 4 + xf) {
      case 0: return G;
      case 1: return (G + b(xi, yi) + 1) >> 1;                    // a
      case 2: return b(xi, yi);                                   // b
      case 3: return (ref_y(r, xi + 1, yi) + b(xi, yi) + 1) >> 1; // c
      case 4: return (G + h(xi, yi) + 1) >> 1;                    // d
      case 5: return (b(xi, yi) + h(xi, yi) + 1) >> 1;            // e
      case 6: return (b(xi, yi) + j(xi, yi) + 1) >> 1;            // f
      case 7: return (b(xi, yi) + h(xi + 1, yi) + 1) >> 1;        // g
      case 8: return h(xi, yi);                                   // h
      case 9: return (h(xi, yi) + j(xi, yi) + 1) >> 1;            // i
      case 10: return j(xi, yi);                                  // j
      case 11: return (j(xi, yi) + h(xi + 1, yi) + 1) >> 1;       // k
      case 12: return (ref_y(r, xi, yi + 1) + h(xi, yi) + 1) >> 1; // n
      case 13: return (h(xi, yi) + b(xi, yi + 1) + 1) >> 1;       // p
      case 14: return (j(xi, yi) + b(xi, yi + 1) + 1) >> 1;       // q
      case 15: return (h(xi + 1, yi) + b(xi, yi + 1) + 1) >> 1;   // r
    }
    return 0;
  }
  static int chroma_sample(const std::vector<uint16_t>& plane, int cw, int ch, int xi, int yi, int xf, int yf) {
    auto P = [&](int x, int y) {
      return static_cast<int>(plane[static_cast<size_t>(clampi(y, 0, ch - 1)) * cw + clampi(x, 0, cw - 1)]);
    };
    return ((8 - xf) * (8 - yf) * P(xi, yi) + xf * (8 - yf) * P(xi + 1, yi) + (8 - xf) * yf * P(xi, yi + 1) +
            xf * yf * P(xi + 1, yi + 1) + 32) >>
           6;
  }
  // weighted sample prediction (8.4.2.3) from the per-list predictions
  int weigh(int comp, int r0, int r1, int p0, int p1) const {
    const bool b0 = r0 >= 0, b1 = r1 >= 0;
    const int maxv = comp ? maxC : maxY;
    if (sh.has_weights) {
      const WeightTable& w = sh.wt;
      int logwd = comp ? w.chroma_log2 : w.luma_log2;
      int w0 = 0, o0 = 0, w1 = 0, o1 = 0;
      if (b0) {
        w0 = comp ? w.cw[0][r0][comp - 1] : w.lw[0][r0];
        o0 = comp ? w.co[0][r0][comp - 1] : w.lo[0][r0];
      }
      if (b1) {
        w1 = comp ? w.cw[1][r1][comp - 1] : w.lw[1][r1];
        o1 = comp ? w.co[1][r1][comp - 1] : w.lo[1][r1];
      }
      // offsets are in units of the 8-bit range (8.4.2.3.2: o = offset * 2^(BitDepth - 8))
      const int osh = (comp ? bdC : bdY) - 8;
      o0 *= 1 << osh;
      o1 *= 1 << osh;
      if (b0 && b1) return clip_px(((p0 * w0 + p1 * w1 + (1 << logwd)) >> (logwd + 1)) + ((o0 + o1 + 1) >> 1), maxv);
      int p = b0 ? p0 : p1, ww = b0 ? w0 : w1, o = b0 ? o0 : o1;
      if (logwd >= 1) return clip_px(((p * ww + (1 << (logwd - 1))) >> logwd) + o, maxv);
      return clip_px(p * ww + o, maxv);
    }
    if (b0 && b1) {
      if (sh.slice_type == SLICE_B && pp->weighted_bipred_idc == 2) {
        int w0 = implicit_w[r0][r1][0], w1 = implicit_w[r0][r1][1];
        return clip_px((p0 * w0 + p1 * w1 + 32) >> 6, maxv);
      }
      return (p0 + p1 + 1) >> 1;
    }
    return b0 ? p0 : p1;
  }
  // predict the whole MB into the picture buffers from the per-4x4 motion
  void inter_pred(int addr) {
    int mx = addr % cur->wmb, my = addr / cur->wmb;
    int cw = cur->W / 2, ch = cur->H / 2;
    for (int r = 0; r < 16; ++r) {
      int bx = r & 3, by = r >> 2;
      int refs[2] = {cur->ref[0][addr * 16 + r], cur->ref[1][addr * 16 + r]};
      if (refs[0] < 0 && refs[1] < 0) throw std::runtime_error("inter block without prediction list");
      int ly[2][16] = {}, lu[2][4] = {}, lv[2][4] = {};
      for (int l = 0; l < 2; ++l) {
        if (refs[l] < 0) continue;
        const Pic& ref = *list[l][refs[l]];
        int mvx = cur->mv[l][addr * 32 + 2 * r], mvy = cur->mv[l][addr * 32 + 2 * r + 1];
        for (int y = 0; y < 4; ++y)
          for (int x = 0; x < 4; ++x) {
            int px = mx * 16 + bx * 4 + x, py = my * 16 + by * 4 + y;
            ly[l][y * 4 + x] = luma_sample(ref, px + (mvx >> 2), py + (mvy >> 2), mvx & 3, mvy & 3, maxY);
          }
        for (int y = 0; y < 2; ++y)
          for (int x = 0; x < 2; ++x) {
            int px = mx * 8 + bx * 2 + x, py = my * 8 + by * 2 + y;
            int xi = px + (mvx >> 3), yi = py + (mvy >> 3);
            lu[l][y * 2 + x] = chroma_sample(ref.U, cw, ch, xi, yi, mvx & 7, mvy & 7);
            lv[l][y * 2 + x] = chroma_sample(ref.V, cw, ch, xi, yi, mvx & 7, mvy & 7);
          }
      }
      for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) {
          int px = mx * 16 + bx * 4 + x, py = my * 16 + by * 4 + y;
          cur->Y[static_cast<size_t>(py) * cur->W + px] =
              static_cast<uint16_t>(weigh(0, refs[0], refs[1], ly[0][y * 4 + x], ly[1][y * 4 + x]));
        }
      for (int y = 0; y < 2; ++y)
        for (int x = 0; x < 2; ++x) {
          int px = mx * 8 + bx * 2 + x, py = my * 8 + by * 2 + y;
          cur->U[static_cast<size_t>(py) * cw + px] =
              static_cast<uint16_t>(weigh(1, refs[0], refs[1], lu[0][y * 2 + x], lu[1][y * 2 + x]));
          cur->V[static_cast<size_t>(py) * cw + px] =
              static_cast<uint16_t>(weigh(2, refs[0], refs[1], lv[0][y * 2 + x], lv[1][y * 2 + x]));
        }
    }
  }

  // ------------------------------------------------------------ CAVLC residual (9.2)
  int nc_luma(int addr, int blkidx) {
    int bx = kBlkX[blkidx], by = kBlkY[blkidx];
    int ba, bb;
    int na = nb_any(addr, bx * 4 - 1, by * 4, &ba);
    int nbk = nb_any(addr, bx * 4, by * 4 - 1, &bb);
    auto tcv = [&](int n, int b) -> int {
      if (cur->skip[n]) return 0;
      if (cur->kind[n] == MBK_IPCM) return 16;
      return cur->tc[n * 24 + kRasterToBlk[b]];
    };
    int nA = na >= 0 ? tcv(na, ba) : 0;
    int nB = nbk >= 0 ? tcv(nbk, bb) : 0;
    if (na >= 0 && nbk >= 0) return (nA + nB + 1) >> 1;
    if (na >= 0) return nA;
    if (nbk >= 0) return nB;
    return 0;
  }
  int nc_chroma(int addr, int comp, int blk) {
    int cx = blk & 1, cy = blk >> 1;
    int a = cx > 0 ? addr : mbA(addr);
    int b = cy > 0 ? addr : mbB(addr);
    int ia = 16 + comp * 4 + cy * 2 + (cx > 0 ? cx - 1 : 1);
    int ib = 16 + comp * 4 + (cy > 0 ? cy - 1 : 1) * 2 + cx;
    auto tcv = [&](int n, int i) -> int {
      if (cur->skip[n]) return 0;
      if (cur->kind[n] == MBK_IPCM) return 16;
      return cur->tc[n * 24 + i];
    };
    int nA = a >= 0 ? tcv(a, ia) : 0;
    int nB = b >= 0 ? tcv(b, ib) : 0;
    if (a >= 0 && b >= 0) return (nA + nB + 1) >> 1;
    if (a >= 0) return nA;
    if (b >= 0) return nB;
    return 0;
  }

  // residual_block_cavlc (7.3.5.3.2); writes coefficient levels into lv[start..end]
  int read_block(BitReader& br, int* lv, int start, int end, int max_num, int nc) {
    for (int i = 0; i < std::max(max_num, end + 1); ++i) lv[i] = 0;  // lv[start..end] written below
    int tc, t1;
    if (nc == -1) {
      int k = read_vlc(br, kChromaDcCoeffTokenLen, kChromaDcCoeffTokenBits, 20);
      tc = k >> 2;
      t1 = k & 3;
    } else if (nc >= 8) {
      int code = br.get(6);
      if (code == 3) {
        tc = 0;
        t1 = 0;
      } else {
        tc = (code >> 2) + 1;
        t1 = code & 3;
        if (t1 > tc) throw std::runtime_error("bad FLC coeff_token");
      }
    } else {
      int t = nc < 2 ? 0 : (nc < 4 ? 1 : 2);
      int k = read_vlc(br, kCoeffTokenLen[t], kCoeffTokenBits[t], 68);
      tc = k >> 2;
      t1 = k & 3;
    }
    if (tc == 0) return 0;
    if (tc > end - start + 1) throw std::runtime_error("TotalCoeff exceeds block size");
    int level[16], run[16];
    int suffix_len = (tc > 10 && t1 < 3) ? 1 : 0;
    for (int i = 0; i < tc; ++i) {
      if (i < t1) {
        level[i] = br.get_bit() ? -1 : 1;
        continue;
      }
      int prefix = 0;
      while (br.get_bit() == 0) {
        if (++prefix > 32) throw std::runtime_error("bad level_prefix");
      }
      int code = (std::min(15, prefix) << suffix_len);
      int ssize = suffix_len;
      if (prefix == 14 && suffix_len == 0) ssize = 4;
      if (prefix >= 15) ssize = prefix - 3;
      if (suffix_len > 0 || prefix >= 14) {
        if (ssize > 0) code += static_cast<int>(br.get(ssize));
      }
      if (prefix >= 15 && suffix_len == 0) code += 15;
      if (prefix >= 16) code += (1 << (prefix - 3)) - 4096;
      if (i == t1 && t1 < 3) code += 2;
      level[i] = (code % 2 == 0) ? (code + 2) >> 1 : (-code - 1) >> 1;
      if (suffix_len == 0) suffix_len = 1;
      if (std::abs(level[i]) > (3 << (suffix_len - 1)) && suffix_len < 6) ++suffix_len;
    }
    int zeros_left = 0;
    if (tc < end - start + 1) {
      if (max_num == 4) {
        zeros_left = read_vlc(br, kChromaDcTotalZerosLen[tc - 1], kChromaDcTotalZerosBits[tc - 1], 4);
      } else {
        zeros_left = read_vlc(br, kTotalZerosLen[tc - 1], kTotalZerosBits[tc - 1], 16);
      }
    }
    for (int i = 0; i < tc - 1; ++i) {
      if (zeros_left > 0) {
        int t = std::min(zeros_left, 7) - 1;
        run[i] = read_vlc(br, kRunBeforeLen[t], kRunBeforeBits[t], 15);
        if (run[i] > zeros_left) throw std::runtime_error("run_before exceeds zerosLeft");
      } else {
        run[i] = 0;
      }
      zeros_left -= run[i];
    }
    run[tc - 1] = zeros_left;
    int pos = -1;
    for (int i = tc - 1; i >= 0; --i) {
      pos += run[i] + 1;
      if (start + pos > end) throw std::runtime_error("coefficient index out of range");
      lv[start + pos] = level[i];
    }
    return tc;
  }

  // ------------------------------------------------------------ CABAC syntax (9.3.2, 9.3.3.1)
  bool cabac_skip_flag(int addr) {
    int a = mbA(addr), b = mbB(addr);
    int inc = (a >= 0 && !cur->skip[a]) + (b >= 0 && !cur->skip[b]);
    return cab.decision((sh.slice_type == SLICE_B ? 24 : 11) + inc) != 0;
  }
  // I mb_type (prefix-less in I slices, suffix in P/B); returns the I mb_type value 0..25
  int cabac_mb_type_i(int addr, bool islice) {
    int b0;
    if (islice) {
      int a = mbA(addr), b = mbB(addr);
      auto ct = [&](int n) { return n >= 0 && cur->kind[n] != MBK_I4x4 && cur->kind[n] != MBK_I8x8; };
      b0 = cab.decision(3 + ct(a) + ct(b));
    } else {
      b0 = cab.decision(sh.slice_type == SLICE_B ? 32 : 17);
    }
    if (!b0) return 0;
    if (cab.terminate()) return 25;
    int cl, cc, pm;
    if (islice) {
      cl = cab.decision(3 + 3);
      cc = cab.decision(3 + 4);
      if (cc) cc += cab.decision(3 + 5);
      pm = cab.decision(3 + 6) << 1;
      pm |= cab.decision(3 + 7);
    } else {
      int off = sh.slice_type == SLICE_B ? 32 : 17;
      cl = cab.decision(off + 1);
      cc = cab.decision(off + 2);
      if (cc) cc += cab.decision(off + 2);
      pm = cab.decision(off + 3) << 1;
      pm |= cab.decision(off + 3);
    }
    return 1 + pm + 4 * cc + 12 * cl;
  }
  int cabac_mb_type_b(int addr) {
    int a = mbA(addr), b = mbB(addr);
    auto ct = [&](int n) { return n >= 0 && !cur->skip[n] && cur->kind[n] != MBK_BDIRECT; };
    if (!cab.decision(27 + ct(a) + ct(b))) return 0;
    if (!cab.decision(27 + 3)) return 1 + cab.decision(27 + 5);
    int bits = cab.decision(27 + 4) << 3;
    bits |= cab.decision(27 + 5) << 2;
    bits |= cab.decision(27 + 5) << 1;
    bits |= cab.decision(27 + 5);
    if (bits < 8) return bits + 3;
    if (bits == 13) return 23 + cabac_mb_type_i(addr, false);
    if (bits == 14) return 11;
    if (bits == 15) return 22;
    bits = (bits << 1) | cab.decision(27 + 5);
    return bits - 4;
  }
  int cabac_sub_b() {
    if (!cab.decision(36)) return 0;
    if (!cab.decision(37)) return 1 + cab.decision(39);
    int t = 3;
    if (cab.decision(38)) {
      if (cab.decision(39)) return 11 + cab.decision(39);
      t += 4;
    }
    t += 2 * cab.decision(39);
    t += cab.decision(39);
    return t;
  }
  int cabac_sub_p() {
    if (cab.decision(21)) return 0;
    if (!cab.decision(22)) return 1;
    return cab.decision(23) ? 2 : 3;
  }
  int cabac_ref_idx(int addr, int l, int x4, int y4) {
    auto cond = [&](int xN, int yN) {
      int blk;
      int n = nb_any(addr, xN, yN, &blk);
      if (n < 0) return 0;
      if (n != addr && (cur->skip[n] || is_intra(n))) return 0;
      int q = ((blk & 3) >> 1) + 2 * ((blk >> 2) >> 1);
      if ((cur->direct[n] >> q) & 1) return 0;
      return cur->ref[l][n * 16 + blk] > 0 ? 1 : 0;
    };
    int inc = cond(x4 * 4 - 1, y4 * 4) + 2 * cond(x4 * 4, y4 * 4 - 1);
    if (!cab.decision(54 + inc)) return 0;
    int v = 1;
    int ctx = 58;
    while (cab.decision(ctx)) {
      ++v;
      ctx = 59;
      if (v > 32) throw std::runtime_error("CABAC: ref_idx too large");
    }
    return v;
  }
  int cabac_mvd(int addr, int l, int comp, int x4, int y4) {
    auto absn = [&](int xN, int yN) {
      int blk;
      int n = nb_any(addr, xN, yN, &blk);
      if (n < 0) return 0;
      return static_cast<int>(cur->mvd[l][n * 32 + 2 * blk + comp]);
    };
    int sum = absn(x4 * 4 - 1, y4 * 4) + absn(x4 * 4, y4 * 4 - 1);
    int base = comp ? 47 : 40;
    int inc = sum < 3 ? 0 : (sum > 32 ? 2 : 1);
    if (!cab.decision(base + inc)) return 0;
    int v = 1;
    while (v < 9 && cab.decision(base + (v < 4 ? v + 2 : 6))) ++v;
    if (v >= 9) v += cab.eg(3);
    return cab.bypass() ? -v : v;
  }
  int cabac_cbp(int addr) {
    int a = mbA(addr), b = mbB(addr);
    auto lcbp = [&](int n) { return n < 0 ? 0x0F : (cur->kind[n] == MBK_IPCM ? 0x2F : (cur->skip[n] ? 0 : cur->cbp[n])); };
    int la = lcbp(a), lb = lcbp(b);
    int cbp = 0;
    for (int b8 = 0; b8 < 4; ++b8) {
      int ca = (b8 & 1) ? ((cbp >> (b8 - 1)) & 1) : ((la >> (b8 + 1)) & 1);
      int cb = (b8 & 2) ? ((cbp >> (b8 - 2)) & 1) : ((lb >> (b8 + 2)) & 1);
      cbp |= cab.decision(73 + (ca ? 0 : 1) + 2 * (cb ? 0 : 1)) << b8;
    }
    auto ccbp = [&](int n) { return n < 0 ? 0 : (cur->kind[n] == MBK_IPCM ? 2 : (cur->skip[n] ? 0 : cur->cbp[n] >> 4)); };
    int ca = ccbp(a), cb = ccbp(b);
    if (cab.decision(77 + (ca > 0) + 2 * (cb > 0))) {
      int c2 = cab.decision(77 + 4 + (ca == 2) + 2 * (cb == 2));
      cbp |= (1 + c2) << 4;
    }
    return cbp;
  }
  int cabac_qp_delta() {
    if (!cab.decision(60 + (prev_qp_delta_nz ? 1 : 0))) return 0;
    int m = 1;
    int ctx = 62;
    while (cab.decision(ctx)) {
      ++m;
      ctx = 63;
      if (m > 104) throw std::runtime_error("CABAC: mb_qp_delta too large");
    }
    return (m & 1) ? (m + 1) / 2 : -(m / 2);
  }
  int cabac_chroma_mode(int addr) {
    int a = mbA(addr), b = mbB(addr);
    auto ct = [&](int n) { return n >= 0 && is_intra(n) && cur->kind[n] != MBK_IPCM && cur->chroma_mode[n] != 0; };
    if (!cab.decision(64 + ct(a) + ct(b))) return 0;
    if (!cab.decision(67)) return 1;
    return cab.decision(67) ? 3 : 2;
  }
  int cabac_intra_mode() {  // -1: prev_intra_pred_mode_flag, else rem_intra_pred_mode
    if (cab.decision(68)) return -1;
    int r = cab.decision(69);
    r |= cab.decision(69) << 1;
    r |= cab.decision(69) << 2;
    return r;
  }
  int cabac_t8x8(int addr) {
    int a = mbA(addr), b = mbB(addr);
    return cab.decision(399 + (a >= 0 && cur->t8x8[a]) + (b >= 0 && cur->t8x8[b]));
  }
  // residual_block_cabac: n coefficients in levelListIdx order
  void cabac_block(int* c, int n, int cat, int cbf_inc) {
    for (int i = 0; i < n; ++i) c[i] = 0;
    if (cbf_inc >= 0) {
      if (!cab.decision(85 + kCbfCatOffset[cat] + cbf_inc)) return;
    }
    int sigpos[64];
    int ns = 0;
    int last = n - 1;
    for (int i = 0; i < n - 1; ++i) {
      int sctx, lctx;
      if (cat == 5) {
        sctx = 402 + kSig8x8Frame[i];
        lctx = 417 + kLast8x8Frame[i];
      } else {
        int inc = cat == 3 ? std::min(i, 2) : i;
        sctx = 105 + kSigCatOffset[cat] + inc;
        lctx = 166 + kSigCatOffset[cat] + inc;
      }
      if (cab.decision(sctx)) {
        sigpos[ns++] = i;
        if (cab.decision(lctx)) {
          last = i;
          break;
        }
      }
    }
    if (ns == 0 || sigpos[ns - 1] != last) sigpos[ns++] = last;  // reached the end: last coefficient significant
    int abase = cat == 5 ? 426 : 227 + kAbsCatOffset[cat];
    int gmax = cat == 3 ? 3 : 4;
    int ngt1 = 0, neq1 = 0;
    for (int k = ns - 1; k >= 0; --k) {
      int a1;
      if (!cab.decision(abase + (ngt1 ? 0 : std::min(4, neq1 + 1)))) {
        a1 = 0;
      } else {
        int ctx1 = abase + 5 + std::min(gmax, ngt1);
        a1 = 1;
        while (a1 < 14 && cab.decision(ctx1)) ++a1;
        if (a1 >= 14) a1 += cab.eg(0);
      }
      if (a1 == 0) ++neq1;
      else ++ngt1;
      int v = a1 + 1;
      c[sigpos[k]] = cab.bypass() ? -v : v;
    }
  }

  // ------------------------------------------------------------ intra prediction (8.3)
  int intra_avail(int addr, int xN, int yN) {
    int blk;
    int n = nb_loc(addr, xN, yN, &blk);
    if (n < 0) return 0;
    if (n != addr && pp->constrained_intra_pred && !is_intra(n)) return 0;
    return 1;
  }

  void pred4x4(int addr, int blkidx, int mode, uint16_t* pred) {
    int mx = addr % cur->wmb, my = addr / cur->wmb;
    int bx = kBlkX[blkidx] * 4, by = kBlkY[blkidx] * 4;
    int X0 = mx * 16 + bx, Y0 = my * 16 + by;
    int top[8], left[4], tl = 0;
    bool has_top = intra_avail(addr, bx, by - 1);
    bool has_left = intra_avail(addr, bx - 1, by);
    bool has_tl = intra_avail(addr, bx - 1, by - 1);
    bool has_tr = intra_avail(addr, bx + 4, by - 1);
    if (has_top)
      for (int x = 0; x < 4; ++x) top[x] = cur->px(X0 + x, Y0 - 1);
    if (has_top) {
      if (has_tr)
        for (int x = 4; x < 8; ++x) top[x] = cur->px(X0 + x, Y0 - 1);
      else
        for (int x = 4; x < 8; ++x) top[x] = top[3];
    }
    if (has_left)
      for (int y = 0; y < 4; ++y) left[y] = cur->px(X0 - 1, Y0 + y);
    if (has_tl) tl = cur->px(X0 - 1, Y0 - 1);
    auto P = [&](int x, int y) -> int {  // p[x,y] with x,y in -1..7
      if (y == -1 && x == -1) return tl;
      if (y == -1) return top[x];
      return left[y];
    };
    auto need = [&](bool c) {
      if (!c) throw std::runtime_error("intra 4x4 mode uses unavailable samples");
    };
    for (int y = 0; y < 4; ++y)
      for (int x = 0; x < 4; ++x) {
        int v = 0;
        switch (mode) {
          case 0: need(has_top); v = P(x, -1); break;
          case 1: need(has_left); v = P(-1, y); break;
          case 2: {
            if (has_top && has_left) v = (top[0] + top[1] + top[2] + top[3] + left[0] + left[1] + left[2] + left[3] + 4) >> 3;
            else if (has_left) v = (left[0] + left[1] + left[2] + left[3] + 2) >> 2;
            else if (has_top) v = (top[0] + top[1] + top[2] + top[3] + 2) >> 2;
            else v = 1 << (bdY - 1);
            break;
          }
          case 3:
            need(has_top);
            if (x == 3 && y == 3) v = (P(6, -1) + 3 * P(7, -1) + 2) >> 2;
            else v = (P(x + y, -1) + 2 * P(x + y + 1, -1) + P(x + y + 2, -1) + 2) >> 2;
            break;
          case 4:
            need(has_top && has_left && has_tl);
            if (x > y) v = (P(x - y - 2, -1) + 2 * P(x - y - 1, -1) + P(x - y, -1) + 2) >> 2;
            else if (x < y) v = (P(-1, y - x - 2) + 2 * P(-1, y - x - 1) + P(-1, y - x) + 2) >> 2;
            else v = (P(0, -1) + 2 * P(-1, -1) + P(-1, 0) + 2) >> 2;
            break;
          case 5: {
            need(has_top && has_left && has_tl);
            int z = 2 * x - y;
            if (z >= 0 && (z & 1) == 0) v = (P(x - (y >> 1) - 1, -1) + P(x - (y >> 1), -1) + 1) >> 1;
            else if (z >= 0) v = (P(x - (y >> 1) - 2, -1) + 2 * P(x - (y >> 1) - 1, -1) + P(x - (y >> 1), -1) + 2) >> 2;
            else if (z == -1) v = (P(-1, 0) + 2 * P(-1, -1) + P(0, -1) + 2) >> 2;
            else v = (P(-1, y - 1) + 2 * P(-1, y - 2) + P(-1, y - 3) + 2) >> 2;
            break;
          }
          case 6: {
            need(has_top && has_left && has_tl);
            int z = 2 * y - x;
            if (z >= 0 && (z & 1) == 0) v = (P(-1, y - (x >> 1) - 1) + P(-1, y - (x >> 1)) + 1) >> 1;
            else if (z >= 0) v = (P(-1, y - (x >> 1) - 2) + 2 * P(-1, y - (x >> 1) - 1) + P(-1, y - (x >> 1)) + 2) >> 2;
            else if (z == -1) v = (P(-1, 0) + 2 * P(-1, -1) + P(0, -1) + 2) >> 2;
            else v = (P(x - 1, -1) + 2 * P(x - 2, -1) + P(x - 3, -1) + 2) >> 2;
            break;
          }
          case 7:
            need(has_top);
            if ((y & 1) == 0) v = (P(x + (y >> 1), -1) + P(x + (y >> 1) + 1, -1) + 1) >> 1;
            else v = (P(x + (y >> 1), -1) + 2 * P(x + (y >> 1) + 1, -1) + P(x + (y >> 1) + 2, -1) + 2) >> 2;
            break;
          case 8: {
            need(has_left);
            int z = x + 2 * y;
            if (z < 5 && (z & 1) == 0) v = (P(-1, y + (x >> 1)) + P(-1, y + (x >> 1) + 1) + 1) >> 1;
            else if (z < 5) v = (P(-1, y + (x >> 1)) + 2 * P(-1, y + (x >> 1) + 1) + P(-1, y + (x >> 1) + 2) + 2) >> 2;
            else if (z == 5) v = (P(-1, 2) + 3 * P(-1, 3) + 2) >> 2;
            else v = P(-1, 3);
            break;
          }
          default: throw std::runtime_error("bad intra4x4 mode");
        }
        pred[y * 4 + x] = static_cast<uint16_t>(v);
      }
  }

  // Intra_8x8 (8.3.2) with reference sample filtering (8.3.2.2.1)
  void pred8x8(int addr, int b8, int mode, uint16_t* pred) {
    int mx = addr % cur->wmb, my = addr / cur->wmb;
    int bx = (b8 & 1) * 8, by = (b8 >> 1) * 8;
    int X0 = mx * 16 + bx, Y0 = my * 16 + by;
    bool has_top = intra_avail(addr, bx, by - 1);
    bool has_left = intra_avail(addr, bx - 1, by);
    bool has_tl = intra_avail(addr, bx - 1, by - 1);
    bool has_tr = intra_avail(addr, bx + 8, by - 1);
    int t[16] = {}, l[8] = {}, tl = 0;
    if (has_top) {
      for (int x = 0; x < 8; ++x) t[x] = cur->px(X0 + x, Y0 - 1);
      for (int x = 8; x < 16; ++x) t[x] = has_tr ? cur->px(X0 + x, Y0 - 1) : t[7];
    }
    if (has_left)
      for (int y = 0; y < 8; ++y) l[y] = cur->px(X0 - 1, Y0 + y);
    if (has_tl) tl = cur->px(X0 - 1, Y0 - 1);
    int ft[16] = {}, fl[8] = {}, ftl = 0;
    if (has_top) {
      ft[0] = has_tl ? (tl + 2 * t[0] + t[1] + 2) >> 2 : (3 * t[0] + t[1] + 2) >> 2;
      for (int x = 1; x < 15; ++x) ft[x] = (t[x - 1] + 2 * t[x] + t[x + 1] + 2) >> 2;
      ft[15] = (t[14] + 3 * t[15] + 2) >> 2;
    }
    if (has_tl) {
      if (has_top && has_left) ftl = (t[0] + 2 * tl + l[0] + 2) >> 2;
      else if (has_top) ftl = (3 * tl + t[0] + 2) >> 2;
      else if (has_left) ftl = (3 * tl + l[0] + 2) >> 2;
      else ftl = tl;
    }
    if (has_left) {
      fl[0] = has_tl ? (tl + 2 * l[0] + l[1] + 2) >> 2 : (3 * l[0] + l[1] + 2) >> 2;
      for (int y = 1; y < 7; ++y) fl[y] = (l[y - 1] + 2 * l[y] + l[y + 1] + 2) >> 2;
      fl[7] = (l[6] + 3 * l[7] + 2) >> 2;
    }
    auto T = [&](int x) { return x < 0 ? ftl : ft[x]; };
    auto L = [&](int y) { return y < 0 ? ftl : fl[y]; };
    if ((mode == 0 || mode == 3 || mode == 7) && !has_top) throw std::runtime_error("intra 8x8 mode needs top samples");
    if ((mode == 1 || mode == 8) && !has_left) throw std::runtime_error("intra 8x8 mode needs left samples");
    if ((mode == 4 || mode == 5 || mode == 6) && !(has_top && has_left && has_tl))
      throw std::runtime_error("intra 8x8 mode needs top, left and top-left samples");
    if (mode < 0 || mode > 8) throw std::runtime_error("bad intra8x8 mode");
    int dc = 1 << (bdY - 1);
    if (mode == 2) {
      int st = 0, sl = 0;
      for (int i = 0; i < 8; ++i) {
        st += ft[i];
        sl += fl[i];
      }
      if (has_top && has_left) dc = (st + sl + 8) >> 4;
      else if (has_left) dc = (sl + 4) >> 3;
      else if (has_top) dc = (st + 4) >> 3;
    }
    for (int y = 0; y < 8; ++y)
      for (int x = 0; x < 8; ++x) {
        int v = 0;
        switch (mode) {
          case 0: v = ft[x]; break;
          case 1: v = fl[y]; break;
          case 2: v = dc; break;
          case 3:
            if (x == 7 && y == 7) v = (ft[14] + 3 * ft[15] + 2) >> 2;
            else v = (T(x + y) + 2 * T(x + y + 1) + T(x + y + 2) + 2) >> 2;
            break;
          case 4:
            if (x > y) v = (T(x - y - 2) + 2 * T(x - y - 1) + T(x - y) + 2) >> 2;
            else if (x < y) v = (L(y - x - 2) + 2 * L(y - x - 1) + L(y - x) + 2) >> 2;
            else v = (T(0) + 2 * ftl + L(0) + 2) >> 2;
            break;
          case 5: {
            int z = 2 * x - y;
            if (z >= 0 && (z & 1) == 0) v = (T(x - (y >> 1) - 1) + T(x - (y >> 1)) + 1) >> 1;
            else if (z >= 0) v = (T(x - (y >> 1) - 2) + 2 * T(x - (y >> 1) - 1) + T(x - (y >> 1)) + 2) >> 2;
            else if (z == -1) v = (L(0) + 2 * ftl + T(0) + 2) >> 2;
            else v = (L(y - 2 * x - 1) + 2 * L(y - 2 * x - 2) + L(y - 2 * x - 3) + 2) >> 2;
            break;
          }
          case 6: {
            int z = 2 * y - x;
            if (z >= 0 && (z & 1) == 0) v = (L(y - (x >> 1) - 1) + L(y - (x >> 1)) + 1) >> 1;
            else if (z >= 0) v = (L(y - (x >> 1) - 2) + 2 * L(y - (x >> 1) - 1) + L(y - (x >> 1)) + 2) >> 2;
            else if (z == -1) v = (L(0) + 2 * ftl + T(0) + 2) >> 2;
            else v = (T(x - 2 * y - 1) + 2 * T(x - 2 * y - 2) + T(x - 2 * y - 3) + 2) >> 2;
            break;
          }
          case 7:
            if ((y & 1) == 0) v = (T(x + (y >> 1)) + T(x + (y >> 1) + 1) + 1) >> 1;
            else v = (T(x + (y >> 1)) + 2 * T(x + (y >> 1) + 1) + T(x + (y >> 1) + 2) + 2) >> 2;
            break;
          case 8: {
            int z = x + 2 * y;
            if (z < 13 && (z & 1) == 0) v = (L(y + (x >> 1)) + L(y + (x >> 1) + 1) + 1) >> 1;
            else if (z < 13) v = (L(y + (x >> 1)) + 2 * L(y + (x >> 1) + 1) + L(y + (x >> 1) + 2) + 2) >> 2;
            else if (z == 13) v = (L(6) + 3 * L(7) + 2) >> 2;
            else v = L(7);
            break;
          }
        }
        pred[y * 8 + x] = static_cast<uint16_t>(v);
      }
  }

  void pred16x16(int addr, int mode, uint16_t* pred) {
    int mx = addr % cur->wmb, my = addr / cur->wmb;
    int X0 = mx * 16, Y0 = my * 16;
    bool has_top = intra_avail(addr, 0, -1), has_left = intra_avail(addr, -1, 0), has_tl = intra_avail(addr, -1, -1);
    int top[16], left[16], tl = has_tl ? cur->px(X0 - 1, Y0 - 1) : 0;
    for (int i = 0; i < 16; ++i) {
      top[i] = has_top ? cur->px(X0 + i, Y0 - 1) : 0;
      left[i] = has_left ? cur->px(X0 - 1, Y0 + i) : 0;
    }
    if (mode == 0 && !has_top) throw std::runtime_error("I16 V without top");
    if (mode == 1 && !has_left) throw std::runtime_error("I16 H without left");
    if (mode == 3 && !(has_top && has_left && has_tl)) throw std::runtime_error("I16 plane without neighbours");
    int dc = 1 << (bdY - 1);
    if (mode == 2) {
      int st = 0, sl = 0;
      for (int i = 0; i < 16; ++i) {
        st += top[i];
        sl += left[i];
      }
      if (has_top && has_left) dc = (st + sl + 16) >> 5;
      else if (has_left) dc = (sl + 8) >> 4;
      else if (has_top) dc = (st + 8) >> 4;
    }
    int a = 0, b = 0, c = 0;
    if (mode == 3) {
      int H = 0, V = 0;
      for (int i = 0; i < 8; ++i) {
        H += (i + 1) * (top[8 + i] - (6 - i >= 0 ? top[6 - i] : tl));
        V += (i + 1) * (left[8 + i] - (6 - i >= 0 ? left[6 - i] : tl));
      }
      a = 16 * (left[15] + top[15]);
      b = (5 * H + 32) >> 6;
      c = (5 * V + 32) >> 6;
    }
    for (int y = 0; y < 16; ++y)
      for (int x = 0; x < 16; ++x) {
        int v;
        switch (mode) {
          case 0: v = top[x]; break;
          case 1: v = left[y]; break;
          case 2: v = dc; break;
          default: v = clipY((a + b * (x - 7) + c * (y - 7) + 16) >> 5); break;
        }
        pred[y * 16 + x] = static_cast<uint16_t>(v);
      }
  }

  void pred_chroma(int addr, int mode, const std::vector<uint16_t>& plane, uint16_t* pred) {
    int mx = addr % cur->wmb, my = addr / cur->wmb;
    int cw = cur->W / 2;
    int X0 = mx * 8, Y0 = my * 8;
    bool has_top = intra_avail(addr, 0, -1), has_left = intra_avail(addr, -1, 0), has_tl = intra_avail(addr, -1, -1);
    auto C = [&](int x, int y) { return static_cast<int>(plane[static_cast<size_t>(y) * cw + x]); };
    int top[8], left[8], tl = has_tl ? C(X0 - 1, Y0 - 1) : 0;
    for (int i = 0; i < 8; ++i) {
      top[i] = has_top ? C(X0 + i, Y0 - 1) : 0;
      left[i] = has_left ? C(X0 - 1, Y0 + i) : 0;
    }
    if (mode == 0) {
      for (int blk = 0; blk < 4; ++blk) {
        int xo = (blk & 1) * 4, yo = (blk >> 1) * 4;
        int st = 0, sl = 0;
        for (int i = 0; i < 4; ++i) {
          st += top[xo + i];
          sl += left[yo + i];
        }
        int dc;
        if ((xo == 0 && yo == 0) || (xo > 0 && yo > 0)) {
          if (has_top && has_left) dc = (st + sl + 4) >> 3;
          else if (has_left) dc = (sl + 2) >> 2;
          else if (has_top) dc = (st + 2) >> 2;
          else dc = 1 << (bdC - 1);
        } else if (xo > 0 && yo == 0) {
          if (has_top) dc = (st + 2) >> 2;
          else if (has_left) dc = (sl + 2) >> 2;
          else dc = 1 << (bdC - 1);
        } else {
          if (has_left) dc = (sl + 2) >> 2;
          else if (has_top) dc = (st + 2) >> 2;
          else dc = 1 << (bdC - 1);
        }
        for (int y = 0; y < 4; ++y)
          for (int x = 0; x < 4; ++x) pred[(yo + y) * 8 + xo + x] = static_cast<uint16_t>(dc);
      }
      return;
    }
    if (mode == 1 && !has_left) throw std::runtime_error("chroma H without left");
    if (mode == 2 && !has_top) throw std::runtime_error("chroma V without top");
    if (mode == 3 && !(has_top && has_left && has_tl)) throw std::runtime_error("chroma plane without neighbours");
    int a = 0, b = 0, c = 0;
    if (mode == 3) {
      int H = 0, V = 0;
      for (int i = 0; i < 4; ++i) {
        H += (i + 1) * (top[4 + i] - (2 - i >= 0 ? top[2 - i] : tl));
        V += (i + 1) * (left[4 + i] - (2 - i >= 0 ? left[2 - i] : tl));
      }
      a = 16 * (left[7] + top[7]);
      b = (34 * H + 32) >> 6;
      c = (34 * V + 32) >> 6;
    }
    for (int y = 0; y < 8; ++y)
      for (int x = 0; x < 8; ++x) {
        int v;
        if (mode == 1) v = left[y];
        else if (mode == 2) v = top[x];
        else v = clipC((a + b * (x - 3) + c * (y - 3) + 16) >> 5);
        pred[y * 8 + x] = static_cast<uint16_t>(v);
      }
  }

  // predIntraNxNPredMode of the block whose top-left sample is (bx, by) (8.3.1.1 / 8.3.2.1)
  int pred_intra_mode(int addr, int bx, int by) {
    int ba, bb;
    int na = nb_any(addr, bx - 1, by, &ba);
    int nb = nb_any(addr, bx, by - 1, &bb);
    bool dcpred = na < 0 || nb < 0 || (na != addr && pp->constrained_intra_pred && !is_intra(na)) ||
                  (nb != addr && pp->constrained_intra_pred && !is_intra(nb));
    if (dcpred) return 2;
    auto md = [&](int n, int b) {
      int k = cur->kind[n];
      return (k == MBK_I4x4 || k == MBK_I8x8) ? static_cast<int>(cur->i4[n * 16 + b]) : 2;
    };
    return std::min(md(na, ba), md(nb, bb));
  }

  // ------------------------------------------------------------ macroblock layer (7.3.5)
  void decode_mb(BitReader& br, int addr, int& qp) {
    begin_mb(addr);
    MbSyn s;
    const int st = sh.slice_type;
    // ---- mb_type
    int ptype = -1;  // P mb_type 0..4 (4 = P_8x8ref0)
    int itype = -1;  // I mb_type 0..25
    if (cabac) {
      if (st == SLICE_I) {
        itype = cabac_mb_type_i(addr, true);
      } else if (st == SLICE_P) {
        if (!cab.decision(14)) {
          if (!cab.decision(15)) ptype = cab.decision(16) ? 3 : 0;
          else ptype = cab.decision(17) ? 1 : 2;
        } else {
          itype = cabac_mb_type_i(addr, false);
        }
      } else {
        int bt = cabac_mb_type_b(addr);
        if (bt >= 23) itype = bt - 23;
        else s.btype = bt;
      }
    } else {
      const int mb_type = br.get_ue_max(48, "mb_type");
      if (st == SLICE_P) {
        if (mb_type < 5) ptype = mb_type;
        else itype = mb_type - 5;
      } else if (st == SLICE_B) {
        if (mb_type < 23) s.btype = mb_type;
        else itype = mb_type - 23;
      } else {
        itype = mb_type;
      }
    }
    const bool p8x8ref0 = ptype == 4;
    int kind;
    if (itype >= 0) {
      if (itype > 25) throw std::runtime_error("bad I mb_type");
      if (itype == 0) kind = MBK_I4x4;
      else if (itype == 25) kind = MBK_IPCM;
      else {
        kind = MBK_I16x16;
        s.i16_mode = (itype - 1) % 4;
        s.cbp = ((((itype - 1) / 4) % 3) << 4) | ((itype >= 13) ? 15 : 0);
      }
    } else if (st == SLICE_P) {
      kind = ptype == 0 ? MBK_P16x16 : ptype == 1 ? MBK_P16x8 : ptype == 2 ? MBK_P8x16 : MBK_P8x8;
    } else {
      kind = s.btype == 0 ? MBK_BDIRECT : s.btype == 22 ? MBK_B8x8
             : kBType[s.btype].shape == 0 ? MBK_B16x16 : kBType[s.btype].shape == 1 ? MBK_B16x8 : MBK_B8x16;
    }
    cur->kind[addr] = static_cast<int8_t>(kind);
    int mx = addr % cur->wmb, my = addr / cur->wmb;
    int cw = cur->W / 2;
    if (kind == MBK_IPCM) {
      // pcm_alignment_zero_bits + samples; CABAC restarts its engine afterwards (9.3.1.2)
      while (!br.byte_aligned()) {
        if (br.get_bit()) throw std::runtime_error("pcm_alignment_zero_bit is 1");
      }
      int16_t pcm[384];
      for (int i = 0; i < 384; ++i) pcm[i] = static_cast<int16_t>(br.get(i < 256 ? bdY : bdC));
      if (!parse_only) {
        for (int y = 0; y < 16; ++y)
          for (int x = 0; x < 16; ++x) cur->Y[static_cast<size_t>(my * 16 + y) * cur->W + mx * 16 + x] = pcm[y * 16 + x];
        for (int y = 0; y < 8; ++y)
          for (int x = 0; x < 8; ++x) {
            cur->U[static_cast<size_t>(my * 8 + y) * cw + mx * 8 + x] = pcm[256 + y * 8 + x];
            cur->V[static_cast<size_t>(my * 8 + y) * cw + mx * 8 + x] = pcm[320 + y * 8 + x];
          }
      }
      for (int i = 0; i < 24; ++i) cur->tc[addr * 24 + i] = 16;
      for (int i = 0; i < 16; ++i) cur->nz[addr * 16 + i] = 1;
      cur->cbp[addr] = 0x2F;
      cur->cbf_luma[addr] = 0xFFFF;
      cur->cbf_dc[addr] = 7;
      cur->cbf_cac0[addr] = cur->cbf_cac1[addr] = 15;
      cur->qp[addr] = static_cast<int8_t>(qp);
      cur->qp_dbk[addr] = 0;
      for (int i = 0; i < 16; ++i) blk_done[i] = 1;
      if (cabac) cab.init_engine();
      prev_qp_delta_nz = 0;
      if (parse_only) {
        // the GPU copies the samples from the level pool: 24 chunks of 16 (luma raster, then
        // Cb, Cr); QP 0 is the macroblock's deblocking QP (8.7.2.2, qPp of I_PCM)
        cur->rec_off[addr] = static_cast<uint32_t>(cur->rec_coef.size() / 16);
        cur->rec_mask[addr] = 0;
        cur->rec_coef.insert(cur->rec_coef.end(), pcm, pcm + 384);
        store_record(addr, MBK_IPCM, 0x2F, 0, 0, 0, nullptr, 0);
      }
      return;
    }
    const bool intra = mbk_is_intra(kind);
    // ---- prediction syntax
    const bool sub8 = kind == MBK_P8x8 || kind == MBK_B8x8;
    bool no_sub_lt8 = true;
    if (sub8) {
      // sub_mb_pred (7.3.5.2)
      for (int q = 0; q < 4; ++q) {
        if (st == SLICE_P) s.sub[q] = cabac ? cabac_sub_p() : br.get_ue_max(3, "sub_mb_type");
        else s.sub[q] = cabac ? cabac_sub_b() : br.get_ue_max(12, "sub_mb_type");
        if (s.sub[q] < 0 || s.sub[q] > (st == SLICE_P ? 3 : 12)) throw std::runtime_error("bad sub_mb_type");
        const SubInfo& si = st == SLICE_P ? kPSub[s.sub[q]] : kBSub[s.sub[q]];
        if (st == SLICE_B && s.sub[q] == 0) {
          if (!sp->direct_8x8_inference) no_sub_lt8 = false;
          cur->direct[addr] |= static_cast<uint8_t>(1 << q);
        } else if (si.nparts > 1) {
          no_sub_lt8 = false;
        }
      }
      for (int l = 0; l < 2; ++l) {
        int nref = l ? sh.num_ref_idx_l1_active : sh.num_ref_idx_l0_active;
        for (int q = 0; q < 4; ++q) {
          s.refidx[l][q] = -1;
          const SubInfo& si = st == SLICE_P ? kPSub[s.sub[q]] : kBSub[s.sub[q]];
          if ((cur->direct[addr] >> q) & 1) continue;
          if (!((si.pred >> l) & 1)) continue;
          int v = 0;
          if (nref > 1 && !p8x8ref0)
            v = cabac ? cabac_ref_idx(addr, l, (q & 1) * 2, (q >> 1) * 2) : static_cast<int>(br.get_te(nref - 1));
          if (v >= nref) throw std::runtime_error("ref_idx out of range");
          s.refidx[l][q] = v;
          for (int k = 0; k < 4; ++k)  // visible to the next ref_idx contexts
            cur->ref[l][addr * 16 + (q & 1) * 2 + (k & 1) + 4 * ((q >> 1) * 2 + (k >> 1))] = static_cast<int8_t>(v);
        }
      }
      for (int l = 0; l < 2; ++l)
        for (int q = 0; q < 4; ++q) {
          if ((cur->direct[addr] >> q) & 1) continue;
          const SubInfo& si = st == SLICE_P ? kPSub[s.sub[q]] : kBSub[s.sub[q]];
          if (!((si.pred >> l) & 1)) continue;
          for (int k = 0; k < si.nparts; ++k) {
            int x4 = (q & 1) * 2 + (si.w4 == 1 ? (k & 1) : 0);
            int y4 = (q >> 1) * 2 + (si.h4 == 1 ? (si.w4 == 1 ? (k >> 1) : k) : 0);
            int d0, d1;
            if (cabac) {
              d0 = cabac_mvd(addr, l, 0, x4, y4);
              d1 = cabac_mvd(addr, l, 1, x4, y4);
            } else {
              d0 = br.get_se_range(-32768, 32767, "mvd_l0");
              d1 = br.get_se_range(-32768, 32767, "mvd_l1");
            }
            s.mvd[l][q][k][0] = d0;
            s.mvd[l][q][k][1] = d1;
            for (int yy = y4; yy < y4 + si.h4; ++yy)
              for (int xx = x4; xx < x4 + si.w4; ++xx) {
                cur->mvd[l][addr * 32 + 2 * (xx + 4 * yy)] = static_cast<uint8_t>(std::min(255, std::abs(d0)));
                cur->mvd[l][addr * 32 + 2 * (xx + 4 * yy) + 1] = static_cast<uint8_t>(std::min(255, std::abs(d1)));
              }
          }
        }
    } else if (intra) {
      if (pp->transform_8x8_mode && kind == MBK_I4x4) {
        s.t8x8 = cabac ? cabac_t8x8(addr) : static_cast<int>(br.get_bit());
        if (s.t8x8) {
          kind = MBK_I8x8;
          cur->kind[addr] = MBK_I8x8;
        }
        cur->t8x8[addr] = static_cast<int8_t>(s.t8x8);
      }
      if (kind == MBK_I4x4 || kind == MBK_I8x8) {
        int nblk = kind == MBK_I4x4 ? 16 : 4;
        for (int i = 0; i < nblk; ++i) {
          int rem;
          if (cabac) rem = cabac_intra_mode();
          else rem = br.get_bit() ? -1 : static_cast<int>(br.get(3));
          int bx = kind == MBK_I4x4 ? kBlkX[i] * 4 : (i & 1) * 8;
          int by = kind == MBK_I4x4 ? kBlkY[i] * 4 : (i >> 1) * 8;
          int pred = pred_intra_mode(addr, bx, by);
          int mode = rem < 0 ? pred : (rem < pred ? rem : rem + 1);
          if (kind == MBK_I4x4) {
            s.i4[i] = mode;
            cur->i4[addr * 16 + (bx >> 2) + 4 * (by >> 2)] = static_cast<uint8_t>(mode);
          } else {
            for (int k = 0; k < 4; ++k) {
              s.i4[i * 4 + k] = mode;
              cur->i4[addr * 16 + (bx >> 2) + (k & 1) + 4 * ((by >> 2) + (k >> 1))] = static_cast<uint8_t>(mode);
            }
          }
        }
      }
      s.chroma_mode = cabac ? cabac_chroma_mode(addr) : br.get_ue_max(3, "intra_chroma_pred_mode");
      if (s.chroma_mode > 3) throw std::runtime_error("bad intra_chroma_pred_mode");
      cur->chroma_mode[addr] = static_cast<int8_t>(s.chroma_mode);
    } else if (kind != MBK_BDIRECT) {
      // mb_pred for 16x16 / 16x8 / 8x16 inter partitions
      int np = (kind == MBK_P16x16 || kind == MBK_B16x16) ? 1 : 2;
      int shape = (kind == MBK_P16x8 || kind == MBK_B16x8) ? 1 : ((kind == MBK_P8x16 || kind == MBK_B8x16) ? 2 : 0);
      auto pred_of = [&](int p) -> int {
        if (st == SLICE_P) return 1;
        return p == 0 ? kBType[s.btype].p0 : kBType[s.btype].p1;
      };
      for (int l = 0; l < 2; ++l) {
        int nref = l ? sh.num_ref_idx_l1_active : sh.num_ref_idx_l0_active;
        for (int p = 0; p < np; ++p) {
          s.refidx[l][p] = -1;
          if (!((pred_of(p) >> l) & 1)) continue;
          int x4 = shape == 2 ? p * 2 : 0, y4 = shape == 1 ? p * 2 : 0;
          int w4 = shape == 2 ? 2 : 4, h4 = shape == 1 ? 2 : 4;
          int v = 0;
          if (nref > 1) v = cabac ? cabac_ref_idx(addr, l, x4, y4) : static_cast<int>(br.get_te(nref - 1));
          if (v >= nref) throw std::runtime_error("ref_idx out of range");
          s.refidx[l][p] = v;
          for (int yy = y4; yy < y4 + h4; ++yy)
            for (int xx = x4; xx < x4 + w4; ++xx) cur->ref[l][addr * 16 + xx + 4 * yy] = static_cast<int8_t>(v);
        }
      }
      for (int l = 0; l < 2; ++l)
        for (int p = 0; p < np; ++p) {
          if (!((pred_of(p) >> l) & 1)) continue;
          int x4 = shape == 2 ? p * 2 : 0, y4 = shape == 1 ? p * 2 : 0;
          int w4 = shape == 2 ? 2 : 4, h4 = shape == 1 ? 2 : 4;
          int d0, d1;
          if (cabac) {
            d0 = cabac_mvd(addr, l, 0, x4, y4);
            d1 = cabac_mvd(addr, l, 1, x4, y4);
          } else {
            d0 = br.get_se_range(-32768, 32767, "mvd");
            d1 = br.get_se_range(-32768, 32767, "mvd");
          }
          s.mvd[l][p][0][0] = d0;
          s.mvd[l][p][0][1] = d1;
          for (int yy = y4; yy < y4 + h4; ++yy)
            for (int xx = x4; xx < x4 + w4; ++xx) {
              cur->mvd[l][addr * 32 + 2 * (xx + 4 * yy)] = static_cast<uint8_t>(std::min(255, std::abs(d0)));
              cur->mvd[l][addr * 32 + 2 * (xx + 4 * yy) + 1] = static_cast<uint8_t>(std::min(255, std::abs(d1)));
            }
        }
    } else {
      cur->direct[addr] = 0xF;
    }
    // ---- motion derivation (partition order)
    if (!intra) derive_motion(addr, kind, s);
    // ---- coded_block_pattern / transform size / qp delta
    if (kind != MBK_I16x16) {
      if (cabac) {
        s.cbp = cabac_cbp(addr);
      } else {
        const int code = br.get_ue_max(47, "coded_block_pattern");
        s.cbp = intra ? kGolombToIntraCbp[code] : kGolombToInterCbp[code];
      }
      if ((s.cbp & 15) && pp->transform_8x8_mode && !intra && no_sub_lt8 &&
          (kind != MBK_BDIRECT || sp->direct_8x8_inference)) {
        s.t8x8 = cabac ? cabac_t8x8(addr) : static_cast<int>(br.get_bit());
        cur->t8x8[addr] = static_cast<int8_t>(s.t8x8);
      }
    }
    cur->cbp[addr] = static_cast<uint8_t>(s.cbp);
    int cbp_luma = s.cbp & 15, cbp_chroma = s.cbp >> 4;
    if (cbp_luma || cbp_chroma || kind == MBK_I16x16) {
      const int dlo = -(26 + qpbdY / 2), dhi = 25 + qpbdY / 2;
      const int d = cabac ? cabac_qp_delta() : br.get_se_range(dlo, dhi, "mb_qp_delta");
      if (d < dlo || d > dhi) throw std::runtime_error("mb_qp_delta out of range");
      qp = ((qp + d + 52 + 2 * qpbdY) % (52 + qpbdY)) - qpbdY;
      prev_qp_delta_nz = d != 0;
    } else {
      prev_qp_delta_nz = 0;
    }
    cur->qp[addr] = static_cast<int8_t>(qp);
    cur->qp_dbk[addr] = static_cast<int8_t>(qp);
    // ---- residual syntax
    if (!parse_only) {
      // the parse-only path reads only the blocks the coded_block_pattern codes (every coded
      // block is written whole by the residual parse), so it skips these 2.6 KB of clears
      std::memset(s.lum, 0, sizeof(s.lum));
      std::memset(s.lum8, 0, sizeof(s.lum8));
      std::memset(s.lumdc, 0, sizeof(s.lumdc));
      std::memset(s.cdc, 0, sizeof(s.cdc));
      std::memset(s.cac, 0, sizeof(s.cac));
    }
    for (int i = 0; i < 16; ++i) blk_done[i] = 1;  // for neighbour lookups inside the MB
    if (cabac) parse_residual_cabac(addr, kind, s);
    else parse_residual_cavlc(br, addr, kind, s);
    // non-zero flags for deblocking (per 4x4; 8x8 transform blocks mark their four 4x4s)
    if (s.t8x8) {
      for (int b8 = 0; b8 < 4; ++b8) {
        bool any = false;
        if (cbp_luma & (1 << b8))
          for (int i = 0; i < 64; ++i) any |= s.lum8[b8][i] != 0;
        for (int k = 0; k < 4; ++k) cur->nz[addr * 16 + (b8 & 1) * 2 + (k & 1) + 4 * ((b8 >> 1) * 2 + (k >> 1))] = any;
      }
    } else {
      for (int blk = 0; blk < 16; ++blk) {
        bool any = false;
        if (cbp_luma & (1 << (blk >> 2)))
          for (int i = 0; i < 16; ++i) any |= s.lum[blk][i] != 0;
        if (kind == MBK_I16x16) any |= s.lumdc[blk] != 0;  // not used for bS (intra), informative
        cur->nz[addr * 16 + kBlkX[blk] + 4 * kBlkY[blk]] = any;
      }
    }
    if (parse_only) {
      store_parsed(addr, kind, s, qp);
      for (int i = 0; i < 16; ++i) blk_done[i] = 1;
      return;
    }
    for (int i = 0; i < 16; ++i) blk_done[i] = 0;
    reconstruct(addr, kind, s, qp);
    for (int i = 0; i < 16; ++i) blk_done[i] = 1;
  }

  void derive_motion(int addr, int kind, const MbSyn& s) {
    const int st = sh.slice_type;
    for (int i = 0; i < 16; ++i) blk_done[i] = 0;
    // the partitions' ref_idx were written for the parse contexts; re-derive everything
    for (int l = 0; l < 2; ++l)
      for (int i = 0; i < 16; ++i) cur->ref[l][addr * 16 + i] = -1;
    if (kind == MBK_BDIRECT) {
      direct_pred(addr, 0xF);
      mark_done(0, 0, 4, 4);
      return;
    }
    if (kind == MBK_P8x8 || kind == MBK_B8x8) {
      for (int q = 0; q < 4; ++q) {
        int qx = (q & 1) * 2, qy = (q >> 1) * 2;
        if (st == SLICE_B && s.sub[q] == 0) {
          direct_pred(addr, 1 << q);
          mark_done(qx, qy, 2, 2);
          continue;
        }
        const SubInfo& si = st == SLICE_P ? kPSub[s.sub[q]] : kBSub[s.sub[q]];
        for (int k = 0; k < si.nparts; ++k) {
          int x4 = qx + (si.w4 == 1 ? (k & 1) : 0);
          int y4 = qy + (si.h4 == 1 ? (si.w4 == 1 ? (k >> 1) : k) : 0);
          for (int l = 0; l < 2; ++l) {
            if (!((si.pred >> l) & 1)) continue;
            int ref = s.refidx[l][q];
            int pm[2];
            pred_mv(addr, l, x4 * 4, y4 * 4, si.w4 * 4, 0, 0, ref, pm);
            assign(addr, l, x4, y4, si.w4, si.h4, ref, pm[0] + s.mvd[l][q][k][0], pm[1] + s.mvd[l][q][k][1]);
          }
          mark_done(x4, y4, si.w4, si.h4);
        }
      }
      return;
    }
    int np = (kind == MBK_P16x16 || kind == MBK_B16x16) ? 1 : 2;
    int shape = (kind == MBK_P16x8 || kind == MBK_B16x8) ? 1 : ((kind == MBK_P8x16 || kind == MBK_B8x16) ? 2 : 0);
    for (int p = 0; p < np; ++p) {
      int x4 = shape == 2 ? p * 2 : 0, y4 = shape == 1 ? p * 2 : 0;
      int w4 = shape == 2 ? 2 : 4, h4 = shape == 1 ? 2 : 4;
      int pred = st == SLICE_P ? 1 : (p == 0 ? kBType[s.btype].p0 : kBType[s.btype].p1);
      for (int l = 0; l < 2; ++l) {
        if (!((pred >> l) & 1)) continue;
        int ref = s.refidx[l][p];
        int pm[2];
        pred_mv(addr, l, x4 * 4, y4 * 4, w4 * 4, shape, p, ref, pm);
        assign(addr, l, x4, y4, w4, h4, ref, pm[0] + s.mvd[l][p][0][0], pm[1] + s.mvd[l][p][0][1]);
      }
      mark_done(x4, y4, w4, h4);
    }
  }

  void parse_residual_cavlc(BitReader& br, int addr, int kind, MbSyn& s) {
    int cbp_luma = s.cbp & 15, cbp_chroma = s.cbp >> 4;
    if (kind == MBK_I16x16) read_block(br, s.lumdc, 0, 15, 16, nc_luma(addr, 0));
    for (int b8 = 0; b8 < 4; ++b8)
      for (int b4 = 0; b4 < 4; ++b4) {
        int blk = b8 * 4 + b4;
        if (!(cbp_luma & (1 << b8))) continue;
        int nc = nc_luma(addr, blk);
        int t = kind == MBK_I16x16 ? read_block(br, s.lum[blk], 1, 15, 15, nc) : read_block(br, s.lum[blk], 0, 15, 16, nc);
        cur->tc[addr * 24 + blk] = static_cast<uint8_t>(t);
        if (s.t8x8)  // 8x8 levels arrive as four interleaved 4x4 blocks (7.3.5.3.2)
          for (int i = 0; i < 16; ++i) s.lum8[b8][4 * i + b4] = s.lum[blk][i];
      }
    if (s.t8x8) std::memset(s.lum, 0, sizeof(s.lum));
    if (cbp_chroma)
      for (int c = 0; c < 2; ++c) read_block(br, s.cdc[c], 0, 3, 4, -1);
    if (cbp_chroma & 2)
      for (int c = 0; c < 2; ++c)
        for (int b = 0; b < 4; ++b) {
          int t = read_block(br, s.cac[c][b], 1, 15, 15, nc_chroma(addr, c, b));
          cur->tc[addr * 24 + 16 + c * 4 + b] = static_cast<uint8_t>(t);
        }
  }

  void parse_residual_cabac(int addr, int kind, MbSyn& s) {
    const bool intra = mbk_is_intra(kind);
    int cbp_luma = s.cbp & 15, cbp_chroma = s.cbp >> 4;
    int a = mbA(addr), b = mbB(addr);
    if (kind == MBK_I16x16) {
      auto cond = [&](int n) {
        if (n < 0) return 1;  // the current MB is intra
        if (cur->kind[n] == MBK_IPCM) return 1;
        if (cur->kind[n] != MBK_I16x16) return 0;
        return cur->cbf_dc[n] & 1;
      };
      cabac_block(s.lumdc, 16, 0, cond(a) + 2 * cond(b));
      bool any = false;
      for (int i = 0; i < 16; ++i) any |= s.lumdc[i] != 0;
      if (any) cur->cbf_dc[addr] |= 1;
    }
    for (int b8 = 0; b8 < 4; ++b8) {
      if (!(cbp_luma & (1 << b8))) continue;
      if (s.t8x8) {
        cabac_block(s.lum8[b8], 64, 5, -1);
        int x4 = (b8 & 1) * 2, y4 = (b8 >> 1) * 2;
        cur->cbf_luma[addr] |= static_cast<uint16_t>(0x33u << (x4 + 4 * y4));
        continue;
      }
      for (int b4 = 0; b4 < 4; ++b4) {
        int blk = b8 * 4 + b4;
        int x4 = kBlkX[blk], y4 = kBlkY[blk];
        auto cond = [&](int xN, int yN) {
          int nb;
          int n = nb_any(addr, xN, yN, &nb);
          if (n < 0) return intra ? 1 : 0;
          if (cur->kind[n] == MBK_IPCM) return 1;
          if (n != addr && cur->skip[n]) return 0;
          return (cur->cbf_luma[n] >> nb) & 1;
        };
        int inc = cond(x4 * 4 - 1, y4 * 4) + 2 * cond(x4 * 4, y4 * 4 - 1);
        int tmp[16];
        bool any = false;
        if (kind == MBK_I16x16) {
          cabac_block(tmp, 15, 1, inc);
          s.lum[blk][0] = 0;
          for (int i = 0; i < 15; ++i) {
            s.lum[blk][i + 1] = tmp[i];
            any |= tmp[i] != 0;
          }
        } else {
          cabac_block(tmp, 16, 2, inc);
          for (int i = 0; i < 16; ++i) {
            s.lum[blk][i] = tmp[i];
            any |= tmp[i] != 0;
          }
        }
        if (any) cur->cbf_luma[addr] |= static_cast<uint16_t>(1u << (x4 + 4 * y4));
      }
    }
    if (cbp_chroma) {
      for (int c = 0; c < 2; ++c) {
        auto cond = [&](int n) {
          if (n < 0) return intra ? 1 : 0;
          if (cur->kind[n] == MBK_IPCM) return 1;
          if (cur->skip[n] || (cur->cbp[n] >> 4) == 0) return 0;
          return (cur->cbf_dc[n] >> (1 + c)) & 1;
        };
        cabac_block(s.cdc[c], 4, 3, cond(a) + 2 * cond(b));
        bool any = false;
        for (int i = 0; i < 4; ++i) any |= s.cdc[c][i] != 0;
        if (any) cur->cbf_dc[addr] |= static_cast<uint8_t>(2 << c);
      }
    }
    if (cbp_chroma & 2) {
      for (int c = 0; c < 2; ++c)
        for (int bb = 0; bb < 4; ++bb) {
          int cx = bb & 1, cy = bb >> 1;
          auto cond = [&](int n, int blk) {
            if (n < 0) return intra ? 1 : 0;
            if (cur->kind[n] == MBK_IPCM) return 1;
            if (n != addr && (cur->skip[n] || (cur->cbp[n] >> 4) != 2)) return 0;
            return ((c ? cur->cbf_cac1[n] : cur->cbf_cac0[n]) >> blk) & 1;
          };
          int ca = cx > 0 ? cond(addr, cy * 2) : cond(a, cy * 2 + 1);
          int cb = cy > 0 ? cond(addr, cx) : cond(b, 2 + cx);
          int tmp[15];
          cabac_block(tmp, 15, 4, ca + 2 * cb);
          bool any = false;
          s.cac[c][bb][0] = 0;
          for (int i = 0; i < 15; ++i) {
            s.cac[c][bb][i + 1] = tmp[i];
            any |= tmp[i] != 0;
          }
          if (any) {
            if (c) cur->cbf_cac1[addr] |= static_cast<uint8_t>(1 << bb);
            else cur->cbf_cac0[addr] |= static_cast<uint8_t>(1 << bb);
          }
        }
    }
  }

  // parse-only records (the GPU decode path's layout)
  void store_parsed(int addr, int kind, const MbSyn& s, int qp) {
    uint32_t mask = 0;
    cur->rec_off[addr] = static_cast<uint32_t>(cur->rec_coef.size() / 16);
    auto put = [&](int bit, const int* v, int n, const int* v2) {
      bool any = false;
      for (int i = 0; i < n; ++i) any |= v[i] != 0 || (v2 && v2[i] != 0);
      if (!any) return;
      mask |= 1u << bit;
      size_t b = cur->rec_coef.size();
      cur->rec_coef.resize(b + 16, 0);
      for (int i = 0; i < n; ++i) cur->rec_coef[b + i] = static_cast<int16_t>(v[i]);
      if (v2)
        for (int i = 0; i < n; ++i) cur->rec_coef[b + n + i] = static_cast<int16_t>(v2[i]);
    };
    // only the blocks the coded_block_pattern codes are read (decode_mb leaves the others
    // uncleared in parse-only mode)
    const int cbp_luma = s.cbp & 15, cbp_chroma = s.cbp >> 4;
    if (s.t8x8) {
      // 8x8 levels as 16-level chunks: chunk blk = b8 * 4 + k holds levels 16k..16k+15 of
      // 8x8 block b8, i.e. the record layout (COEF_LUMA + b8 * 64).  The GPU path reads
      // 8x8 transform (decode.hip inverse8x8).
      for (int blk = 0; blk < 16; ++blk)
        if (cbp_luma & (1 << (blk >> 2))) put(blk, s.lum8[blk >> 2] + 16 * (blk & 3), 16, nullptr);
    } else {
      for (int blk = 0; blk < 16; ++blk)
        if (cbp_luma & (1 << (blk >> 2))) put(blk, s.lum[blk], 16, nullptr);
    }
    if (kind == MBK_I16x16) put(16, s.lumdc, 16, nullptr);
    if (cbp_chroma) put(17, s.cdc[0], 4, s.cdc[1]);
    if (cbp_chroma & 2)
      for (int cc = 0; cc < 2; ++cc)
        for (int b = 0; b < 4; ++b) put(18 + cc * 4 + b, s.cac[cc][b], 16, nullptr);
    cur->rec_mask[addr] = mask;
    store_record(addr, kind, s.cbp, qp, s.i16_mode, s.chroma_mode, (kind == MBK_I4x4 || kind == MBK_I8x8) ? s.i4 : nullptr,
                 s.t8x8);
  }

  // ------------------------------------------------------------ reconstruction
  void add_residual4(int addr, int bx, int by, const int* lv, int qp, bool dc_given, int dcv, const uint8_t* w4) {
    int X0 = (addr % cur->wmb) * 16, Y0 = (addr / cur->wmb) * 16;
    int d[16];
    for (int i = 0; i < 16; ++i) d[i] = 0;
    for (int i = dc_given ? 1 : 0; i < 16; ++i) {
      int r = kZigzag4x4[i];
      d[r] = scale4(lv[i], qp, r & 3, r >> 2, w4);
    }
    if (dc_given) d[0] = dcv;
    idct4(d);
    for (int y = 0; y < 4; ++y)
      for (int x = 0; x < 4; ++x) {
        uint16_t& o = cur->Y[static_cast<size_t>(Y0 + by + y) * cur->W + X0 + bx + x];
        o = static_cast<uint16_t>(clipY(o + d[y * 4 + x]));
      }
  }
  void add_residual8(int addr, int b8, const int* lv, int qp, const uint8_t* w8) {
    int X0 = (addr % cur->wmb) * 16 + (b8 & 1) * 8, Y0 = (addr / cur->wmb) * 16 + (b8 >> 1) * 8;
    int d[64];
    for (int i = 0; i < 64; ++i) d[i] = 0;
    for (int i = 0; i < 64; ++i) {
      int r = kZigzag8x8[i];
      d[r] = scale8(lv[i], qp, r & 7, r >> 3, w8);
    }
    idct8(d);
    for (int y = 0; y < 8; ++y)
      for (int x = 0; x < 8; ++x) {
        uint16_t& o = cur->Y[static_cast<size_t>(Y0 + y) * cur->W + X0 + x];
        o = static_cast<uint16_t>(clipY(o + d[y * 8 + x]));
      }
  }

  void reconstruct(int addr, int kind, const MbSyn& s, int qp_y) {
    const int qp = qp_y + qpbdY;  // QP'Y (8.5.12.1)
    int mx = addr % cur->wmb, my = addr / cur->wmb;
    int cw = cur->W / 2;
    int X0 = mx * 16, Y0 = my * 16;
    int cbp_luma = s.cbp & 15, cbp_chroma = s.cbp >> 4;
    // the picture's scaling lists (8.5.9): intra Y / Cb / Cr, inter Y / Cb / Cr; 8x8 intra / inter
    const int li = mbk_is_intra(kind) ? 0 : 3;
    const uint8_t* wy4 = pp->sl4[li];
    const uint8_t* wy8 = pp->sl8[li ? 1 : 0];
    if (kind == MBK_I4x4) {
      for (int blk = 0; blk < 16; ++blk) {
        uint16_t pred[16];
        pred4x4(addr, blk, s.i4[blk], pred);
        int bx = kBlkX[blk] * 4, by = kBlkY[blk] * 4;
        for (int y = 0; y < 4; ++y)
          for (int x = 0; x < 4; ++x) cur->Y[static_cast<size_t>(Y0 + by + y) * cur->W + X0 + bx + x] = pred[y * 4 + x];
        add_residual4(addr, bx, by, s.lum[blk], qp, false, 0, wy4);
        blk_done[kBlkX[blk] + 4 * kBlkY[blk]] = 1;
      }
    } else if (kind == MBK_I8x8) {
      for (int b8 = 0; b8 < 4; ++b8) {
        uint16_t pred[64];
        pred8x8(addr, b8, s.i4[b8 * 4], pred);
        int bx = (b8 & 1) * 8, by = (b8 >> 1) * 8;
        for (int y = 0; y < 8; ++y)
          for (int x = 0; x < 8; ++x) cur->Y[static_cast<size_t>(Y0 + by + y) * cur->W + X0 + bx + x] = pred[y * 8 + x];
        if (cbp_luma & (1 << b8)) add_residual8(addr, b8, s.lum8[b8], qp, wy8);
        mark_done(bx >> 2, by >> 2, 2, 2);
      }
    } else if (kind == MBK_I16x16) {
      uint16_t pred[256];
      pred16x16(addr, s.i16_mode, pred);
      for (int y = 0; y < 16; ++y)
        for (int x = 0; x < 16; ++x) cur->Y[static_cast<size_t>(Y0 + y) * cur->W + X0 + x] = pred[y * 16 + x];
      // luma DC: inverse scan into 4x4 (block geometry), Hadamard, scale (8.5.10)
      int c[16], f[16], tmp[16];
      for (int i = 0; i < 16; ++i) c[kZigzag4x4[i]] = s.lumdc[i];
      for (int y = 0; y < 4; ++y) {
        int* q = c + 4 * y;
        tmp[4 * y + 0] = q[0] + q[1] + q[2] + q[3];
        tmp[4 * y + 1] = q[0] + q[1] - q[2] - q[3];
        tmp[4 * y + 2] = q[0] - q[1] - q[2] + q[3];
        tmp[4 * y + 3] = q[0] - q[1] + q[2] - q[3];
      }
      for (int x = 0; x < 4; ++x) {
        int s0 = tmp[x], s1 = tmp[4 + x], s2 = tmp[8 + x], s3 = tmp[12 + x];
        f[x] = s0 + s1 + s2 + s3;
        f[4 + x] = s0 + s1 - s2 - s3;
        f[8 + x] = s0 - s1 - s2 + s3;
        f[12 + x] = s0 - s1 + s2 - s3;
      }
      int ls = level_scale(qp % 6, 0, 0, wy4[0]);
      for (int blk = 0; blk < 16; ++blk) {
        int bx = kBlkX[blk], by = kBlkY[blk];
        int fv = f[bx + 4 * by];
        int dcv = qp >= 36 ? (fv * ls) << (qp / 6 - 6) : (fv * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
        add_residual4(addr, bx * 4, by * 4, s.lum[blk], qp, true, dcv, wy4);
      }
    } else {
      inter_pred(addr);
      if (s.t8x8) {
        for (int b8 = 0; b8 < 4; ++b8)
          if (cbp_luma & (1 << b8)) add_residual8(addr, b8, s.lum8[b8], qp, wy8);
      } else {
        for (int blk = 0; blk < 16; ++blk) {
          if (!(cbp_luma & (1 << (blk >> 2)))) continue;
          add_residual4(addr, kBlkX[blk] * 4, kBlkY[blk] * 4, s.lum[blk], qp, false, 0, wy4);
        }
      }
    }
    // chroma
    const bool intra = mbk_is_intra(kind);
    for (int comp = 0; comp < 2; ++comp) {
      std::vector<uint16_t>& plane = comp == 0 ? cur->U : cur->V;
      uint16_t pred[64];
      if (intra) {
        pred_chroma(addr, s.chroma_mode, plane, pred);
      } else {
        for (int y = 0; y < 8; ++y)
          for (int x = 0; x < 8; ++x) pred[y * 8 + x] = plane[static_cast<size_t>(my * 8 + y) * cw + mx * 8 + x];
      }
      const int qpc = qpc_of(qp_y, comp == 0 ? pp->chroma_qp_index_offset : pp->second_chroma_qp_index_offset) + qpbdC;
      int c0 = s.cdc[comp][0], c1 = s.cdc[comp][1], c2 = s.cdc[comp][2], c3 = s.cdc[comp][3];
      int f[4] = {c0 + c1 + c2 + c3, c0 - c1 + c2 - c3, c0 + c1 - c2 - c3, c0 - c1 - c2 + c3};
      const uint8_t* wc4 = pp->sl4[li + 1 + comp];
      int ls = level_scale(qpc % 6, 0, 0, wc4[0]);
      for (int b = 0; b < 4; ++b) {
        int d[16];
        for (int i = 0; i < 16; ++i) d[i] = 0;
        if (cbp_chroma & 2)
          for (int i = 1; i < 16; ++i) {
            int r = kZigzag4x4[i];
            d[r] = scale4(s.cac[comp][b][i], qpc, r & 3, r >> 2, wc4);
          }
        d[0] = ((f[b] * ls) << (qpc / 6)) >> 5;
        bool any = cbp_chroma != 0;
        if (any) idct4(d);
        int xo = (b & 1) * 4, yo = (b >> 1) * 4;
        for (int y = 0; y < 4; ++y)
          for (int x = 0; x < 4; ++x) {
            int v = pred[(yo + y) * 8 + xo + x] + (any ? d[y * 4 + x] : 0);
            plane[static_cast<size_t>(my * 8 + yo + y) * cw + mx * 8 + xo + x] = static_cast<uint16_t>(clipC(v));
          }
      }
    }
  }

  // parse-only: the slice's reference lists (picture ids) and weighted-prediction table
  void record_lists_and_weights() {
    // a later slice of the picture must use the same lists and weights (one table per
    // picture on the GPU): compare with the first slice's
    std::vector<int32_t> prev_ids;
    std::vector<int16_t> prev_wp;
    if (cur->nslices > 1) {
      prev_ids.swap(cur->list_ids);
      prev_wp.swap(cur->wp);
    }
    cur->list_ids.assign(64, -1);
    for (int l = 0; l < 2; ++l)
      for (size_t i = 0; i < list[l].size() && i < 32; ++i) cur->list_ids[l * 32 + i] = list[l][i]->id;
    cur->wp.assign(kWpEntries, 0);
    int16_t* w = cur->wp.data();
    // the picture's scaling lists (raster weights, 8.5.6) and constrained_intra_pred_flag ride
    // in the same per-picture table
    for (int i = 0; i < 6; ++i)
      for (int j = 0; j < 16; ++j) w[kWpScale + i * 16 + j] = pp->sl4[i][j];
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 64; ++j) w[kWpScale + 96 + i * 64 + j] = pp->sl8[i][j];
    w[kWpFlags] = static_cast<int16_t>(pp->constrained_intra_pred ? 1 : 0);
    if (sh.has_weights) {
      w[0] = 1;
      w[1] = static_cast<int16_t>(sh.wt.luma_log2);
      w[2] = static_cast<int16_t>(sh.wt.chroma_log2);
      for (int l = 0; l < 2; ++l)
        for (int i = 0; i < 32; ++i) {
          w[kWpLw + l * 32 + i] = static_cast<int16_t>(sh.wt.lw[l][i]);
          w[kWpLo + l * 32 + i] = static_cast<int16_t>(sh.wt.lo[l][i]);
          for (int c = 0; c < 2; ++c) {
            w[kWpCw + (l * 32 + i) * 2 + c] = static_cast<int16_t>(sh.wt.cw[l][i][c]);
            w[kWpCo + (l * 32 + i) * 2 + c] = static_cast<int16_t>(sh.wt.co[l][i][c]);
          }
        }
    } else if (sh.slice_type == SLICE_B && pp->weighted_bipred_idc == 2) {
      w[0] = 2;
      if (sh.num_ref_idx_l0_active > 8 || sh.num_ref_idx_l1_active > 8) cur->gpu_ok = false;
      for (int i = 0; i < 8 && i < sh.num_ref_idx_l0_active; ++i)
        for (int j = 0; j < 8 && j < sh.num_ref_idx_l1_active; ++j) {
          w[kWpImp + (i * 8 + j) * 2] = static_cast<int16_t>(implicit_w[i][j][0]);
          w[kWpImp + (i * 8 + j) * 2 + 1] = static_cast<int16_t>(implicit_w[i][j][1]);
        }
    }
    if (cur->nslices > 1 && (prev_ids != cur->list_ids || prev_wp != cur->wp)) cur->gpu_ok = false;
  }

  // parse-only: boundary strength of every filtered edge segment (deblock.hip reads these
  // instead of deriving them, so reference identity across lists / multi-reference and
  // 8x8-transform edges follow the decoder exactly); 0 = not filtered.  Packed 4 bits per
  // segment: [mb][16] bytes, segment i = dir * 16 + edge * 4 + k in byte i / 2 (low nibble
  // for even i).
  std::vector<uint8_t> boundary_strengths() {
    int nmb = cur->wmb * cur->hmb;
    std::vector<uint8_t> out(static_cast<size_t>(nmb) * 16, 0);
    flat_.resize(nmb);
    for (int a = 0; a < nmb; ++a) flat_[a] = !is_intra(a) && no_nz(a) && one_motion(a);
    for (int addr = 0; addr < nmb; ++addr) {
      if (cur->slice[addr] < 0) continue;
      const SliceParams& spar = slices[cur->slice[addr]];
      if (spar.disable_idc == 1) continue;
      int mx = addr % cur->wmb, my = addr / cur->wmb;
      bool left = mx > 0 && !(spar.disable_idc == 2 && cur->slice[addr - 1] != cur->slice[addr]);
      bool top = my > 0 && !(spar.disable_idc == 2 && cur->slice[addr - cur->wmb] != cur->slice[addr]);
      bool t8 = cur->t8x8[addr] != 0;
      const bool iq = is_intra(addr);
      // internal edges of an inter MB with one motion for all 16 blocks and no coded luma
      // block have bS 0 (8.7.2.1), as do the 4 segments of an MB edge between two such MBs
      // with the same motion
      const bool flat_q = flat_[addr] != 0;
      uint8_t* o = &out[static_cast<size_t>(addr) * 16];
      auto put = [&](int i, int v) { o[i >> 1] |= static_cast<uint8_t>(v << ((i & 1) * 4)); };
      for (int dir = 0; dir < 2; ++dir)
        for (int e = 0; e < 4; ++e) {
          if (e == 0 && !(dir == 0 ? left : top)) continue;
          if (t8 && (e & 1)) continue;
          if (e > 0 && flat_q) continue;
          const int base = dir * 16 + e * 4;
          int mbp = e == 0 ? (dir == 0 ? addr - 1 : addr - cur->wmb) : addr;
          if (iq || (e == 0 && is_intra(mbp))) {
            for (int k = 0; k < 4; ++k) put(base + k, e == 0 ? 4 : 3);
            continue;
          }
          if (e == 0 && flat_q && flat_[mbp]) {
            // two flat MBs: every segment of the edge compares the same two motions
            if (same_motion(mbp, addr)) continue;
            const int v = bs_inter(mbp, dir == 0 ? 3 : 12, addr, 0);
            for (int k = 0; k < 4; ++k) put(base + k, v);
            continue;
          }
          for (int k = 0; k < 4; ++k) {
            int blkq = dir == 0 ? (e + 4 * k) : (k + 4 * e);
            int blkp = dir == 0 ? (e == 0 ? 3 + 4 * k : e - 1 + 4 * k) : (e == 0 ? k + 12 : k + 4 * (e - 1));
            put(base + k, bs_inter(mbp, blkp, addr, blkq));
          }
        }
    }
    return out;
  }
  // bs_of for two inter MBs (the callers above have taken the intra cases)
  int bs_inter(int mbp, int blkp, int mbq, int blkq) const {
    if (cur->nz[mbp * 16 + blkp] | cur->nz[mbq * 16 + blkq]) return 2;
    const int p0 = cur->refpic[0][mbp * 16 + blkp], p1 = cur->refpic[1][mbp * 16 + blkp];
    const int q0 = cur->refpic[0][mbq * 16 + blkq], q1 = cur->refpic[1][mbq * 16 + blkq];
    const int np = (p0 >= 0) + (p1 >= 0), nq = (q0 >= 0) + (q1 >= 0);
    if (np != nq) return 1;
    const int16_t* mp0 = &cur->mv[0][mbp * 32 + 2 * blkp];
    const int16_t* mp1 = &cur->mv[1][mbp * 32 + 2 * blkp];
    const int16_t* mq0 = &cur->mv[0][mbq * 32 + 2 * blkq];
    const int16_t* mq1 = &cur->mv[1][mbq * 32 + 2 * blkq];
    auto far = [](const int16_t* a, const int16_t* b) { return std::abs(a[0] - b[0]) >= 4 || std::abs(a[1] - b[1]) >= 4; };
    if (np == 1) {
      const int pp = p0 >= 0 ? p0 : p1, qq = q0 >= 0 ? q0 : q1;
      if (pp != qq) return 1;
      return far(p0 >= 0 ? mp0 : mp1, q0 >= 0 ? mq0 : mq1) ? 1 : 0;
    }
    if (!((p0 == q0 && p1 == q1) || (p0 == q1 && p1 == q0))) return 1;
    if (p0 != p1) {
      if (p0 == q0) return (far(mp0, mq0) || far(mp1, mq1)) ? 1 : 0;
      return (far(mp0, mq1) || far(mp1, mq0)) ? 1 : 0;
    }
    return ((far(mp0, mq0) || far(mp1, mq1)) && (far(mp0, mq1) || far(mp1, mq0))) ? 1 : 0;
  }
  std::vector<uint8_t> flat_;  // boundary_strengths: inter MB, no coded luma, one motion
  bool no_nz(int a) const {
    uint64_t w0, w1;
    std::memcpy(&w0, &cur->nz[a * 16], 8);
    std::memcpy(&w1, &cur->nz[a * 16 + 8], 8);
    return (w0 | w1) == 0;
  }
  // all 16 blocks share each list's picture and vector
  bool one_motion(int a) const {
    // every entry equals its successor (pictures) / the pair after it (vectors)
    for (int l = 0; l < 2; ++l) {
      const int* rp = &cur->refpic[l][a * 16];
      const int16_t* m = &cur->mv[l][a * 32];
      if (std::memcmp(rp, rp + 1, 15 * sizeof(int)) != 0 || std::memcmp(m, m + 2, 30 * sizeof(int16_t)) != 0) return false;
    }
    return true;
  }
  // block 0 of MBs a and b reference the same pictures with the same vectors, per list
  bool same_motion(int a, int b) const {
    for (int l = 0; l < 2; ++l) {
      if (cur->refpic[l][a * 16] != cur->refpic[l][b * 16]) return false;
      if (cur->refpic[l][a * 16] < 0) continue;
      if (cur->mv[l][a * 32] != cur->mv[l][b * 32] || cur->mv[l][a * 32 + 1] != cur->mv[l][b * 32 + 1]) return false;
    }
    return true;
  }

  // ------------------------------------------------------------ deblocking (8.7)
  int bs_of(int mbp, int blkp, int mbq, int blkq, bool mb_edge) {
    bool ip = is_intra(mbp), iq = is_intra(mbq);
    if (mb_edge && (ip || iq)) return 4;
    if (ip || iq) return 3;
    if (cur->nz[mbp * 16 + blkp] || cur->nz[mbq * 16 + blkq]) return 2;
    // different reference pictures / numbers of motion vectors, or MV differences (8.7.2.1)
    int P[2] = {cur->refpic[0][mbp * 16 + blkp], cur->refpic[1][mbp * 16 + blkp]};
    int Q[2] = {cur->refpic[0][mbq * 16 + blkq], cur->refpic[1][mbq * 16 + blkq]};
    int np = (P[0] >= 0) + (P[1] >= 0), nq = (Q[0] >= 0) + (Q[1] >= 0);
    if (np != nq) return 1;
    auto far = [&](int lp, int lq) {
      return std::abs(cur->mv[lp][mbp * 32 + 2 * blkp] - cur->mv[lq][mbq * 32 + 2 * blkq]) >= 4 ||
             std::abs(cur->mv[lp][mbp * 32 + 2 * blkp + 1] - cur->mv[lq][mbq * 32 + 2 * blkq + 1]) >= 4;
    };
    if (np == 1) {
      int lp = P[0] >= 0 ? 0 : 1, lq = Q[0] >= 0 ? 0 : 1;
      if (P[lp] != Q[lq]) return 1;
      return far(lp, lq) ? 1 : 0;
    }
    if (!((P[0] == Q[0] && P[1] == Q[1]) || (P[0] == Q[1] && P[1] == Q[0]))) return 1;
    if (P[0] != P[1]) {
      if (P[0] == Q[0]) return (far(0, 0) || far(1, 1)) ? 1 : 0;
      return (far(0, 1) || far(1, 0)) ? 1 : 0;
    }
    return ((far(0, 0) || far(1, 1)) && (far(0, 1) || far(1, 0))) ? 1 : 0;
  }

  // filter one line of samples across an edge; q0p points to q0, step = distance p0 -> q0
  static void filter_line(uint16_t* q0p, int step, int bs, int alpha, int beta, int tc0, bool chroma, int maxv) {
    int p0 = q0p[-step], p1 = q0p[-2 * step], q0 = q0p[0], q1 = q0p[step];
    if (!(std::abs(p0 - q0) < alpha && std::abs(p1 - p0) < beta && std::abs(q1 - q0) < beta)) return;
    int p2 = chroma ? 0 : q0p[-3 * step], q2 = chroma ? 0 : q0p[2 * step];
    int ap = std::abs(p2 - p0), aq = std::abs(q2 - q0);
    if (bs < 4) {
      int tc = chroma ? tc0 + 1 : tc0 + (ap < beta) + (aq < beta);
      int delta = clampi((((q0 - p0) << 2) + (p1 - q1) + 4) >> 3, -tc, tc);
      q0p[-step] = static_cast<uint16_t>(clip_px(p0 + delta, maxv));
      q0p[0] = static_cast<uint16_t>(clip_px(q0 - delta, maxv));
      if (!chroma) {
        if (ap < beta) q0p[-2 * step] = static_cast<uint16_t>(p1 + clampi((p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1, -tc0, tc0));
        if (aq < beta) q0p[step] = static_cast<uint16_t>(q1 + clampi((q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1, -tc0, tc0));
      }
    } else {
      if (!chroma && ap < beta && std::abs(p0 - q0) < ((alpha >> 2) + 2)) {
        int p3 = q0p[-4 * step];
        q0p[-step] = static_cast<uint16_t>((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
        q0p[-2 * step] = static_cast<uint16_t>((p2 + p1 + p0 + q0 + 2) >> 2);
        q0p[-3 * step] = static_cast<uint16_t>((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
      } else {
        q0p[-step] = static_cast<uint16_t>((2 * p1 + p0 + q1 + 2) >> 2);
      }
      if (!chroma && aq < beta && std::abs(p0 - q0) < ((alpha >> 2) + 2)) {
        int q3 = q0p[3 * step];
        q0p[0] = static_cast<uint16_t>((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
        q0p[step] = static_cast<uint16_t>((p0 + q0 + q1 + q2 + 2) >> 2);
        q0p[2 * step] = static_cast<uint16_t>((2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3);
      } else {
        q0p[0] = static_cast<uint16_t>((2 * q1 + q0 + p1 + 2) >> 2);
      }
    }
  }

  void deblock_picture() {
    int W = cur->W, cw = W / 2;
    int nmb = cur->wmb * cur->hmb;
    for (int addr = 0; addr < nmb; ++addr) {
      if (cur->slice[addr] < 0) continue;
      const SliceParams& spar = slices[cur->slice[addr]];
      if (spar.disable_idc == 1) continue;
      int mx = addr % cur->wmb, my = addr / cur->wmb;
      bool left = mx > 0 && !(spar.disable_idc == 2 && cur->slice[addr - 1] != cur->slice[addr]);
      bool top = my > 0 && !(spar.disable_idc == 2 && cur->slice[addr - cur->wmb] != cur->slice[addr]);
      bool t8 = cur->t8x8[addr] != 0;
      for (int dir = 0; dir < 2; ++dir) {  // 0: vertical edges, 1: horizontal edges
        for (int e = 0; e < 4; ++e) {
          if (e == 0 && !(dir == 0 ? left : top)) continue;
          if (t8 && (e & 1)) continue;  // 8x8 transform: no luma 4-sample edges, no chroma edge there
          int mbp = e == 0 ? (dir == 0 ? addr - 1 : addr - cur->wmb) : addr;
          int bS[4];
          for (int k = 0; k < 4; ++k) {
            int blkq = dir == 0 ? (e + 4 * k) : (k + 4 * e);
            int blkp = dir == 0 ? (e == 0 ? 3 + 4 * k : e - 1 + 4 * k) : (e == 0 ? k + 12 : k + 4 * (e - 1));
            bS[k] = bs_of(mbp, blkp, addr, blkq, e == 0);
          }
          // luma
          int qpav = (cur->qp_dbk[mbp] + cur->qp_dbk[addr] + 1) >> 1;
          int ia = clampi(qpav + spar.alpha_off, 0, 51), ib = clampi(qpav + spar.beta_off, 0, 51);
          const int sy = 1 << (bdY - 8);
          int alpha = kAlpha[ia] * sy, beta = kBeta[ib] * sy;
          for (int i = 0; i < 16; ++i) {
            int bs = bS[i >> 2];
            if (!bs) continue;
            int tc0 = bs < 4 ? kTc0[ia][bs - 1] * sy : 0;
            uint16_t* q0;
            int step;
            if (dir == 0) {
              q0 = &cur->Y[static_cast<size_t>(my * 16 + i) * W + mx * 16 + e * 4];
              step = 1;
            } else {
              q0 = &cur->Y[static_cast<size_t>(my * 16 + e * 4) * W + mx * 16 + i];
              step = W;
            }
            filter_line(q0, step, bs, alpha, beta, tc0, false, maxY);
          }
          // chroma: edges 0 and 2 (luma) map to chroma edges 0 and 4
          if (e == 0 || e == 2) {
            int ce = e / 2;
            for (int comp = 0; comp < 2; ++comp) {
              int off = comp == 0 ? spar.cb_off : spar.cr_off;
              int qpp = cur->kind[mbp] == MBK_IPCM ? qpc_of(0, off) : qpc_of(cur->qp_dbk[mbp], off);
              int qpq = cur->kind[addr] == MBK_IPCM ? qpc_of(0, off) : qpc_of(cur->qp_dbk[addr], off);
              int qa = (qpp + qpq + 1) >> 1;
              int iac = clampi(qa + spar.alpha_off, 0, 51), ibc = clampi(qa + spar.beta_off, 0, 51);
              const int sc = 1 << (bdC - 8);
              int ac = kAlpha[iac] * sc, bc = kBeta[ibc] * sc;
              std::vector<uint16_t>& pl = comp == 0 ? cur->U : cur->V;
              for (int i = 0; i < 8; ++i) {
                int bs = bS[i >> 1];
                if (!bs) continue;
                int tc0 = bs < 4 ? kTc0[iac][bs - 1] * sc : 0;
                uint16_t* q0;
                int step;
                if (dir == 0) {
                  q0 = &pl[static_cast<size_t>(my * 8 + i) * cw + mx * 8 + ce * 4];
                  step = 1;
                } else {
                  q0 = &pl[static_cast<size_t>(my * 8 + ce * 4) * cw + mx * 8 + i];
                  step = cw;
                }
                filter_line(q0, step, bs, ac, bc, tc0, true, maxC);
              }
            }
          }
        }
      }
    }
  }
};

Decoder::Decoder() : impl_(new Impl) {}
Decoder::~Decoder() = default;

void Decoder::decode(const uint8_t* data, size_t n) {
  impl_->skip_deblock = skip_deblock_;
  impl_->out_ = &out_;
  std::vector<NalUnit> nals = parse_annexb(data, n);
  for (NalUnit& u : nals) {
    switch (u.nal_unit_type) {
      case NAL_SPS: {
        BitReader br(u.rbsp.data(), u.rbsp.size());
        SPS s = parse_sps(br);
        impl_->sps[s.sps_id] = s;
        impl_->have_sps[s.sps_id] = true;
        break;
      }
      case NAL_PPS: {
        BitReader br(u.rbsp.data(), u.rbsp.size());
        PPS p = parse_pps(br, impl_->sps);
        impl_->pps[p.pps_id] = p;
        impl_->have_pps[p.pps_id] = true;
        break;
      }
      case NAL_SLICE:
      case NAL_IDR:
        impl_->decode_slice(u, out_);
        break;
      case NAL_AUD:
        impl_->finish_picture(out_);
        break;
      default:
        break;
    }
  }
}

void Decoder::flush() {
  impl_->finish_picture(out_);
  impl_->out_ = &out_;
  if (!impl_->parse_only) impl_->output_ready(true);
}

void Decoder::set_parse_only(bool v) { impl_->parse_only = v; }

void Decoder::pps_scaling(int pps_id, uint8_t* sl4, uint8_t* sl8) const {
  if (pps_id < 0 || pps_id > 255 || !impl_->have_pps[pps_id]) throw std::runtime_error("pps_scaling: unknown PPS");
  std::memcpy(sl4, impl_->pps[pps_id].sl4, sizeof(impl_->pps[pps_id].sl4));
  std::memcpy(sl8, impl_->pps[pps_id].sl8, sizeof(impl_->pps[pps_id].sl8));
}

}  // namespace h264
}  // namespace mivc
