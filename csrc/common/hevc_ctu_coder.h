// HEVC CABAC slice-data coder (ITU-T H.265 7.3.8, 9.3) of the encoder's decision records:
// one implementation shared by the host writer (csrc/host/hevc_writer.cc, host threads over
// the WPP substreams) and the GPU entropy kernel (csrc/kernels/hevc_entropy.hip, one lane per
// WPP substream, one workgroup per picture), so the two produce the same bytes by construction.
//
// The coder reads CtuInfo / CuInfo records and quantised levels (packed non-zero 4x4 blocks,
// or level planes + the per-CTB sub-block maps), keeps the picture-wide state of coded CUs
// (depth, skip, prediction, intra modes, motion, QpY per 8x8 granule) in caller-owned arrays,
// and writes bins through an arithmetic engine templated on its bit sink (host BitWriter, or
// the device's bounded byte buffer).  Invalid records set `err` (a CoderError) instead of
// throwing, so device code can report them; the host wrapper turns them into exceptions.
#pragma once
#include <cstdint>
#include <cstring>

#include "../host/hevc_ctx_tables.h"
#include "hevc_tables.h"

// the slice coder's member functions: host + device without forced inlining, the large ones
// kept out of line on the device (one call site each in the kernel instead of copies)
#if defined(__HIPCC__)
#define HV_FN __host__ __device__
#define HV_BIG __host__ __device__ __attribute__((noinline))
#define HV_CYCLES() __builtin_readcyclecounter()
#else
#define HV_FN inline
#define HV_BIG inline
#define HV_CYCLES() __builtin_ia32_rdtsc()
#endif

// On the device the coder object, its contexts, tables and sink live in LDS: telling the
// compiler lets it use LDS instructions and exclude aliasing with global stores
#if defined(__HIP_DEVICE_COMPILE__)
#define HV_LDS(p) __builtin_assume(__builtin_amdgcn_is_shared(reinterpret_cast<const void*>(p)))
#define HV_GLOBAL(p)                                                                 \
  __builtin_assume(!__builtin_amdgcn_is_shared(reinterpret_cast<const void*>(p)) && \
                   !__builtin_amdgcn_is_private(reinterpret_cast<const void*>(p)))
#else
#define HV_LDS(p) ((void)0)
#define HV_GLOBAL(p) ((void)0)
#endif

namespace mivc {
namespace hevc {

struct CtxState {
  uint8_t state = 0;
  uint8_t mps = 0;
};

// writer context index -> index in the spec initValue table (hevc_ctx_tables.h, dec::DCtx)
struct WriterCtxMap {
  uint8_t m[kNumCtx];
  constexpr void run(int w, int d, int n) {
    for (int i = 0; i < n; ++i) m[w + i] = static_cast<uint8_t>(d + i);
  }
  constexpr WriterCtxMap() : m() {
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
  }
};
static constexpr WriterCtxMap kWriterCtxMap{};

// 9.3.2.2 initialisation; init_type 0 = I, 1 = P, 2 = B (cabac_init_flag 0)
MIVC_HD void init_contexts(CtxState* ctx, int init_type, int slice_qp) {
  const int qp = slice_qp < 0 ? 0 : (slice_qp > 51 ? 51 : slice_qp);
  for (int i = 0; i < kNumCtx; ++i) {
    const int v = dec::kInit[init_type][kWriterCtxMap.m[i]];
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

// one word per (state, quarter of the range): rangeTabLps | next state after an LPS << 8 |
// next state after an MPS << 16 -- a single table read per bin (the GPU coder keeps it in LDS)
struct CabacStepTable {
  uint32_t t[256];
  constexpr CabacStepTable() : t() {
    for (int s = 0; s < 64; ++s)
      for (int q = 0; q < 4; ++q)
        t[(s << 2) | q] = static_cast<uint32_t>(kRangeLps[s][q]) | (static_cast<uint32_t>(kTransIdxLps[s]) << 8) |
                          (static_cast<uint32_t>(s < 62 ? s + 1 : s) << 16);
  }
};
static constexpr CabacStepTable kCabacStep{};

MIVC_HD int hv_clz32(uint32_t v) { return __builtin_clz(v); }

// Arithmetic encoder (9.3.4.3): low / range with deferred carry (outstanding 0xFF bytes).
// Sink: put(value, nbits) of up to 24 bits, MSB first.
template <class Sink>
struct CabacEngine {
  Sink* out = nullptr;
  const uint32_t* step = kCabacStep.t;  // CabacStepTable (or a copy of it in faster memory)
  uint32_t low_ = 0, range_ = 510;
  int bits_left_ = 23;
  int num_buffered_ = 0;
  uint32_t buffered_ = 0xFF;
  uint64_t bins_ = 0;

  MIVC_HD void start() {
    low_ = 0;
    range_ = 510;
    bits_left_ = 23;
    num_buffered_ = 0;
    buffered_ = 0xFF;
    bins_ = 0;
  }

  // branch-free regular bin (9.3.4.3.2): the LPS / MPS choice selects range and low with
  // conditional moves, the renormalisation shift is a count of leading zeros, and the
  // state transition is one table entry
  MIVC_HD void encode(int bin, CtxState& c) {
    HV_LDS(&c);
    HV_LDS(step);
    const uint32_t s = c.state, mps = c.mps;
    uint32_t range = range_, low = low_;
    const uint32_t ent = step[(s << 2) | ((range >> 6) & 3)];
    const uint32_t lps = ent & 0xFFu;
    const uint32_t rmps = range - lps;
    const bool is_lps = static_cast<uint32_t>(bin) != mps;
    const uint32_t r = is_lps ? lps : rmps;
    low += is_lps ? rmps : 0u;
    const int nb = hv_clz32(r) - 23;  // r in [2, 510]: shifts until r >= 256
    const int left = bits_left_ - nb;
    range_ = r << nb;
    low_ = low << nb;
    bits_left_ = left;
    ++bins_;
    c.mps = static_cast<uint8_t>(mps ^ static_cast<uint32_t>(is_lps && s == 0));
    c.state = static_cast<uint8_t>((ent >> (is_lps ? 8 : 16)) & 63u);
    if (left < 12) write_out();
  }

  MIVC_HD void bypass(int bin) {
    ++bins_;
    low_ <<= 1;
    if (bin) low_ += range_;
    if (--bits_left_ < 12) write_out();
  }

  // n bypass bins, most significant first
  MIVC_HD void bypass_bits(uint32_t v, int n) {
    while (n > 8) {
      n -= 8;
      bypass_chunk((v >> n) & 255u, 8);
    }
    if (n > 0) bypass_chunk(v & ((1u << n) - 1u), n);
  }

  MIVC_HD void terminate(int bin) {
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

  // flush after a terminating bin equal to 1
  MIVC_HD void finish() {
    if ((low_ >> (32 - bits_left_)) != 0) {
      out->put(buffered_ + 1, 8);
      while (num_buffered_ > 1) {
        out->put(0x00, 8);
        --num_buffered_;
      }
      low_ -= 1u << (32 - bits_left_);
    } else {
      if (num_buffered_ > 0) out->put(buffered_, 8);
      while (num_buffered_ > 1) {
        out->put(0xFF, 8);
        --num_buffered_;
      }
    }
    out->put(low_ >> 8, 24 - bits_left_);
  }

  MIVC_HD uint64_t bins() const { return bins_; }

  MIVC_HD void bypass_chunk(uint32_t v, int n) {
    bins_ += n;
    low_ <<= n;
    low_ += range_ * v;
    bits_left_ -= n;
    if (bits_left_ < 12) write_out();
  }
  MIVC_HD void write_out() {
    HV_LDS(out);
    const uint32_t lead = low_ >> (24 - bits_left_);
    bits_left_ += 8;
    low_ &= 0xFFFFFFFFu >> bits_left_;
    if (lead == 0xFF) {
      ++num_buffered_;
    } else if (num_buffered_ > 0) {
      const uint32_t carry = lead >> 8;
      out->put(buffered_ + carry, 8);
      buffered_ = lead & 0xFF;
      const uint32_t fill = (0xFF + carry) & 0xFF;
      while (num_buffered_ > 1) {
        out->put(fill, 8);
        --num_buffered_;
      }
    } else {
      num_buffered_ = 1;
      buffered_ = lead;
    }
  }
};

// ------------------------------------------------------------------ coder inputs and state
struct Mv {
  int16_t x, y;
  MIVC_HD bool operator==(const Mv& o) const { return x == o.x && y == o.y; }
};
// motion of a PU: direction (bit 0 list 0, bit 1 list 1), refIdx and vector per used list
struct Motion {
  uint8_t dir;
  int8_t r[2];
  uint8_t pad;
  Mv m[2];
  MIVC_HD bool operator==(const Motion& o) const {
    return dir == o.dir && (!(dir & 1) || (m[0] == o.m[0] && r[0] == o.r[0])) &&
           (!(dir & 2) || (m[1] == o.m[1] && r[1] == o.r[1]));
  }
};
MIVC_HD Motion motion_none() {
  Motion m;
  m.dir = 0;
  m.r[0] = m.r[1] = 0;
  m.pad = 0;
  m.m[0] = Mv{0, 0};
  m.m[1] = Mv{0, 0};
  return m;
}
static_assert(sizeof(Motion) == 12, "Motion is 12 bytes");

// what the coder needs of HevcConfig / HevcFrameParams (plain data: a GPU kernel argument)
struct CoderPic {
  int W, H;         // coded size (multiples of 32)
  int wctb, hctb;   // 32x32 record blocks
  int wctu, hctu;   // CTUs (64x64 with ctu64)
  int L;            // CtbLog2SizeY
  int ctu64, sao, max_merge, tmvp, cu_qp_delta, bit_depth, tu_inter_depth, sdh, wpp;
  int slice_type, qp, poc;
  int ref_poc[2], num_ref[2], list_poc[2][4];
  // collocated picture (8.5.3.2.8): records (null: intra / none), POC and its lists' POCs
  int col_set, col_poc, col_ref_poc[2], col_list_poc[2][4];
};

// level source: packed non-zero 4x4 blocks (levels != null), else coefficient planes;
// nzmap: per CTB (raster) luma sub-block bits (by * 8 + bx), then Cb bits 0-15 / Cr 16-31
struct CoderLevels {
  const uint64_t* nzmap = nullptr;
  const uint32_t* ctb_off = nullptr;
  const int16_t* levels = nullptr;
  size_t nblocks = 0;
  const int16_t* plane[3] = {nullptr, nullptr, nullptr};
  // staged per CTU (GPU): `levels` holds the first `nblocks` non-zero blocks of the current CTU
  // (its 32x32 blocks in z-order, each in packed order), the rest are read from the planes
  int stage_ctu = 0;
};

// picture-wide state of coded CUs, one entry per 8x8 granule (mode4: per 4x4 block); shared by
// the substream coders of one picture (a WPP row only reads granules its 2-CTU lag makes final)
struct CoderState {
  int8_t* depth;
  int8_t* skip;
  int8_t* pred;
  int8_t* mode4;
  Motion* mot;
  uint8_t* coded;
  int8_t* qpy;
};

enum CoderError : int {
  CE_NONE = 0,
  CE_ALL_ZERO_BLOCK,
  CE_PACKED_RANGE,
  CE_SAO_OFFSET,
  CE_SAO_EDGE_SIGN,
  CE_DIRECTION,
  CE_REFIDX,
  CE_COL_REFIDX,
  CE_INTRA_MODE,
  CE_INTER_SPLIT,
  CE_CBF_LUMA,
  CE_QP_DELTA,
  CE_SDH_PARITY,
  CE_OVERFLOW,
  CE_TIMEOUT,
  CE_COUNT
};
inline const char* coder_error_text(int e) {
  switch (e) {
    case CE_ALL_ZERO_BLOCK: return "residual_coding of an all-zero block";
    case CE_PACKED_RANGE: return "HEVC packed levels: block index out of range";
    case CE_SAO_OFFSET: return "SAO offset out of range";
    case CE_SAO_EDGE_SIGN: return "edge-offset signs violate 7.4.9.3.2";
    case CE_DIRECTION: return "HEVC: inter CU direction not allowed in this slice";
    case CE_REFIDX: return "HEVC: inter CU refIdx outside the active list";
    case CE_COL_REFIDX: return "HEVC: collocated refIdx out of range";
    case CE_INTRA_MODE: return "intra mode out of range";
    case CE_INTER_SPLIT: return "HEVC: inter TU split needs depth 1 and a 16x16+ CU";
    case CE_CBF_LUMA: return "inter TU: cbf_luma inferred 1 but the luma block is empty";
    case CE_QP_DELTA: return "HEVC: CuQpDeltaVal out of range";
    case CE_SDH_PARITY: return "HEVC: sign data hiding parity does not match the hidden sign";
    case CE_OVERFLOW: return "HEVC entropy: substream buffer overflow";
    case CE_TIMEOUT: return "HEVC GPU entropy: wavefront progress timeout";
    default: return "HEVC slice coder error";
  }
}

struct CoderStats {
  int intra_cus = 0, inter_cus = 0, skip_cus = 0, merge_cus = 0;
};

// optional cycle accounting of the coder's parts (diagnostics): slot k of `acc` gets the cycles
// spent inside the scope (cycle counter of the CPU / the GPU's s_memtime)
enum CoderProf : int { CP_RESIDUAL = 0, CP_MERGE, CP_AMVP, CP_CU, CP_SAO, CP_CTU, CP_SCAN, CP_N };
struct ProfScope {
  uint64_t* acc;
  uint64_t t0;
  MIVC_HD ProfScope(uint64_t* a, int k) : acc(a ? a + k : nullptr), t0(a ? HV_CYCLES() : 0) {}
  MIVC_HD ~ProfScope() {
    if (acc) *acc += HV_CYCLES() - t0;
  }
};

// ------------------------------------------------------------------ constant tables
// scan orders (6.5.3-6.5.5): [scan_idx][log2 of the grid side 0..3][position] -> x | y << 4
constexpr int scan_pos_c(int scan_idx, int log2size, int p) {
  const int n = 1 << log2size;
  if (scan_idx == 1) return (p % n) | ((p / n) << 8);
  if (scan_idx == 2) return (p / n) | ((p % n) << 8);
  int i = 0;
  for (int d = 0; d < 2 * n - 1; ++d)
    for (int y = d; y >= 0; --y) {
      const int x = d - y;
      if (x < n && y < n) {
        if (i == p) return x | (y << 8);
        ++i;
      }
    }
  return 0;
}
struct ScanTables {
  uint8_t t[3][4][64];
  constexpr ScanTables() : t() {
    for (int s = 0; s < 3; ++s)
      for (int l = 0; l < 4; ++l)
        for (int i = 0; i < (1 << (2 * l)); ++i) {
          const int p = scan_pos_c(s, l, i);
          t[s][l][i] = static_cast<uint8_t>((p & 255) | ((p >> 8) << 4));
        }
  }
};
static constexpr ScanTables kScans{};

// significance context (9.3.4.2.5) of coefficient (xc, yc) of a (1 << log2)^2 TU
constexpr int sig_ctx_c(int xc, int yc, int log2, int cidx, int scan_idx, int prev_csbf, int xs, int ys) {
  constexpr uint8_t map4[16] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8};
  int s = 0;
  if (log2 == 2) {
    s = map4[(yc << 2) + xc];
  } else if (xc + yc == 0) {
    s = 0;
  } else {
    const int xp = xc & 3, yp = yc & 3;
    if (prev_csbf == 0) s = (xp + yp == 0) ? 2 : (xp + yp < 3) ? 1 : 0;
    else if (prev_csbf == 1) s = (yp == 0) ? 2 : (yp == 1) ? 1 : 0;
    else if (prev_csbf == 2) s = (xp == 0) ? 2 : (xp == 1) ? 1 : 0;
    else s = 2;
    if (cidx == 0) {
      if (xs + ys > 0) s += 3;
      s += log2 == 3 ? (scan_idx == 0 ? 9 : 15) : 21;
    } else {
      s += log2 == 3 ? 9 : 12;
    }
  }
  return cidx == 0 ? s : 27 + s;
}
// per (TU size, component, scan, neighbouring coded sub-block flags, first sub-block or not,
// position in the sub-block's scan): a table lookup per coefficient instead of the derivation
struct SigTables {
  uint8_t t[4][2][3][4][2][16];
  constexpr SigTables() : t() {
    for (int l = 0; l < 4; ++l)
      for (int c = 0; c < 2; ++c)
        for (int sc = 0; sc < 3; ++sc)
          for (int pc = 0; pc < 4; ++pc)
            for (int g0 = 0; g0 < 2; ++g0)
              for (int p = 0; p < 16; ++p) {
                const int q = kScans.t[sc][2][p];
                // any sub-block other than the first (a 4x4 TU has only the first: the g0 = 0
                // entries of l = 0 are never read, keep them in range)
                const int xs = (g0 || l == 0) ? 0 : 1;
                t[l][c][sc][pc][g0][p] =
                    static_cast<uint8_t>(sig_ctx_c(xs * 4 + (q & 15), (q >> 4), l + 2, c, sc, pc, xs, 0));
              }
  }
};
static constexpr SigTables kSig{};

static constexpr int8_t kLastGroup[32] = {0, 1, 2, 3, 4, 4, 5, 5, 6, 6, 6, 6, 7, 7, 7, 7,
                                          8, 8, 8, 8, 8, 8, 8, 8, 9, 9, 9, 9, 9, 9, 9, 9};
static constexpr int8_t kLastGroupMin[10] = {0, 1, 2, 3, 4, 6, 8, 12, 16, 24};
static constexpr int8_t kCombL0[12] = {0, 1, 0, 2, 1, 2, 0, 3, 1, 3, 2, 3};
static constexpr int8_t kCombL1[12] = {1, 0, 2, 0, 2, 1, 3, 0, 3, 1, 3, 2};

MIVC_HD int hv_min(int a, int b) { return a < b ? a : b; }
MIVC_HD int hv_max(int a, int b) { return a > b ? a : b; }
MIVC_HD int hv_abs(int a) { return a < 0 ? -a : a; }
MIVC_HD int hv_clamp(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// ------------------------------------------------------------------ the coder
template <class Sink>
struct CtuCoder {
  const CoderPic* P;
  const CtuInfo* ctu;
  const CuInfo* cu;
  const CuInfo* col_cu;  // the collocated picture's records (null: none / intra)
  CoderLevels lv;
  CoderState S;
  CabacEngine<Sink> e;
  CtxState* ctx;  // kNumCtx entries (host: a member array; device: LDS)
  CoderStats st;
  int err = CE_NONE;
  int W, H, wctb, w8, L;
  bool inter_slice, bslice, tmvp, col_l1, no_backward;
  // cu_qp_delta state (7.4.9.14, 8.6.1): qPY_PREV of the next quantization group (the slice
  // QP at the start of the slice and, with WPP, of every CTB row), whether the current
  // quantization group coded its delta, and its qPY_PRED
  int qp_prev = 0, qp_ctb = 0, qp_pred_cur = 0;
  bool qp_coded = false;
  // non-zero 4x4 sub-blocks of the current 32x32 block
  uint64_t nz_luma = 0;
  uint32_t nz_chroma[2] = {0, 0};
  uint32_t ctb_base = 0;
  int cu64_midx = -1;
  Motion cu64_mot;
  uint64_t* prof = nullptr;  // CP_N cycle counters (diagnostics), or null
  // constant tables (kScans, kSig) or copies of them in faster memory (GPU LDS)
  const uint8_t* scans_tab = &kScans.t[0][0][0];
  const uint8_t* sig_tab = &kSig.t[0][0][0][0][0][0];

  HV_FN void fail(int code) __restrict__ {
    if (err == CE_NONE) err = code;
  }

  // contexts initialised, engine started on `sink`
  HV_BIG void begin(const CoderPic* pic, const CtuInfo* ct, const CuInfo* cu_, const CuInfo* col, const CoderLevels& l,
                     const CoderState& s, CtxState* ctx_mem, Sink* sink, const uint32_t* step_tab = nullptr,
                     const uint8_t* scans = nullptr, const uint8_t* sig = nullptr) __restrict__ {
    HV_LDS(this);
    HV_LDS(ctx);
    HV_LDS(P);
    P = pic;
    ctu = ct;
    cu = cu_;
    col_cu = col;
    lv = l;
    S = s;
    ctx = ctx_mem;
    e.out = sink;
    e.step = step_tab ? step_tab : kCabacStep.t;
    scans_tab = scans ? scans : &kScans.t[0][0][0];
    sig_tab = sig ? sig : &kSig.t[0][0][0][0][0][0];
    e.start();
    // every field set here: a coder may sit in raw (unconstructed) memory, e.g. GPU LDS
    err = CE_NONE;
    st = CoderStats();
    qp_ctb = qp_pred_cur = 0;
    qp_coded = false;
    nz_luma = 0;
    nz_chroma[0] = nz_chroma[1] = 0;
    ctb_base = 0;
    cu64_midx = -1;
    cu_stage = nullptr;
    stage_cx = stage_cy = -1;
    prof = nullptr;
    W = P->W;
    H = P->H;
    wctb = P->wctb;
    w8 = W / 8;
    L = P->L;
    inter_slice = P->slice_type != 2;
    bslice = P->slice_type == 0;
    tmvp = inter_slice && P->tmvp;
    col_l1 = bslice;
    no_backward = true;  // NoBackwardPredFlag: no picture of either list follows the current one
    for (int l = 0; l < (bslice ? 2 : 1); ++l)
      for (int i = 0; i < nref(l); ++i) no_backward = no_backward && list_poc(l, i) <= P->poc;
    init_contexts(ctx, bslice ? 2 : (inter_slice ? 1 : 0), P->qp);
    qp_prev = P->qp;
    cu64_mot = motion_none();
  }

  HV_FN size_t g(int x, int y) const __restrict__ { return static_cast<size_t>(y >> 3) * w8 + (x >> 3); }
  HV_FN size_t g4(int x, int y) const __restrict__ { return static_cast<size_t>(y >> 2) * (2 * w8) + (x >> 2); }
  HV_FN bool inside(int x, int y) const __restrict__ { return x >= 0 && y >= 0 && x < W && y < H; }
  // 6.4.1 z-scan availability at 8x8 granularity (the granule is coded iff already visited)
  HV_FN bool avail(int x, int y) const __restrict__ {
    HV_GLOBAL(S.coded);
    return inside(x, y) && S.coded[g(x, y)];
  }

  // records of the current CTU staged in faster memory (GPU): [4 blocks in z-order][16 granules]
  const CuInfo* cu_stage = nullptr;
  int stage_cx = -1, stage_cy = -1;
  HV_FN const CuInfo& cu_at(int x, int y) const __restrict__ {
    if (cu_stage && (x >> L) == stage_cx && (y >> L) == stage_cy) {
      HV_LDS(cu_stage);
      const int q = L == 6 ? ((((y >> 5) & 1) << 1) | ((x >> 5) & 1)) : 0;
      return cu_stage[q * kCusPerCtb + zorder8((x & (kCtb - 1)) >> 3, (y & (kCtb - 1)) >> 3)];
    }
    const int ci = (y >> kCtbLog2) * wctb + (x >> kCtbLog2);
    return cu[static_cast<size_t>(ci) * kCusPerCtb + zorder8((x & (kCtb - 1)) >> 3, (y & (kCtb - 1)) >> 3)];
  }

  // ---------------------------------------------------------------- SAO (7.3.8.3)
  HV_FN static bool same_sao(const CtuInfo& a, const CtuInfo& b) {
    for (int k = 0; k < 2; ++k)
      if (a.sao_type[k] != b.sao_type[k] || (a.sao_type[k] == 2 && a.sao_class[k] != b.sao_class[k])) return false;
    for (int ci = 0; ci < 3; ++ci) {
      const int t = a.sao_type[ci ? 1 : 0];
      if (t == 0) continue;
      if (t == 1 && a.sao_band[ci] != b.sao_band[ci]) return false;
      for (int i = 0; i < 4; ++i)
        if (a.sao_off[ci][i] != b.sao_off[ci][i]) return false;
    }
    return true;
  }

  // SAO parameters of CTU (cx, cy): those of its first 32x32 record block
  HV_FN const CtuInfo& ctu_sao(int cx, int cy) const __restrict__ {
    const int k = P->ctu64 ? 1 : 0;
    return ctu[(cy << k) * wctb + (cx << k)];
  }
  HV_BIG void write_sao(int rx, int ry) __restrict__ {
    HV_LDS(this);
    HV_LDS(ctx);
    HV_LDS(P);
    const ProfScope prof_scope(prof, CP_SAO);
    const CtuInfo& t = ctu_sao(rx, ry);
    if (rx > 0 && same_sao(t, ctu_sao(rx - 1, ry))) {
      e.encode(1, ctx[CTX_SAO_MERGE]);
      return;
    }
    if (rx > 0) e.encode(0, ctx[CTX_SAO_MERGE]);
    if (ry > 0 && same_sao(t, ctu_sao(rx, ry - 1))) {
      e.encode(1, ctx[CTX_SAO_MERGE]);
      return;
    }
    if (ry > 0) e.encode(0, ctx[CTX_SAO_MERGE]);
    const int cmax = (1 << (hv_min(P->bit_depth, 10) - 5)) - 1;
    for (int ci = 0; ci < 3; ++ci) {
      const int type = t.sao_type[ci ? 1 : 0];
      if (ci < 2) {  // sao_type_idx_luma / _chroma: TR cMax 2, first bin context coded
        if (type == 0) {
          e.encode(0, ctx[CTX_SAO_TYPE]);
        } else {
          e.encode(1, ctx[CTX_SAO_TYPE]);
          e.bypass(type == 2);
        }
      }
      if (type == 0) continue;
      for (int i = 0; i < 4; ++i) {
        int a = hv_abs(static_cast<int>(t.sao_off[ci][i]));
        if (a > cmax) {
          fail(CE_SAO_OFFSET);
          a = cmax;
        }
        for (int k = 0; k < a; ++k) e.bypass(1);  // TR, bypass
        if (a < cmax) e.bypass(0);
      }
      if (type == 1) {
        for (int i = 0; i < 4; ++i)
          if (t.sao_off[ci][i] != 0) e.bypass(t.sao_off[ci][i] < 0);
        e.bypass_bits(t.sao_band[ci] & 31, 5);
      } else {
        if (t.sao_off[ci][0] < 0 || t.sao_off[ci][1] < 0 || t.sao_off[ci][2] > 0 || t.sao_off[ci][3] > 0)
          fail(CE_SAO_EDGE_SIGN);
        if (ci < 2) e.bypass_bits(t.sao_class[ci] & 3, 2);
      }
    }
  }

  // ---------------------------------------------------------------- residual coding (7.3.8.11)
  template <class En>
  HV_FN static void write_last(En& en, CtxState* cx, int v, int log2, int cidx, int ctx_base) {
    const int prefix = kLastGroup[v];
    const int cmax = (log2 << 1) - 1;
    int off, shift;
    if (cidx == 0) {
      off = 3 * (log2 - 2) + ((log2 - 1) >> 2);
      shift = (log2 + 1) >> 2;
    } else {
      off = 15;
      shift = log2 - 2;
    }
    for (int i = 0; i < prefix; ++i) en.encode(1, cx[ctx_base + off + (i >> shift)]);
    if (prefix < cmax) en.encode(0, cx[ctx_base + off + (prefix >> shift)]);
  }
  template <class En>
  HV_FN static void write_last_suffix(En& en, int v) {
    const int prefix = kLastGroup[v];
    if (prefix > 3) en.bypass_bits(v - kLastGroupMin[prefix], (prefix >> 1) - 1);
  }

  template <class En>
  HV_FN static void write_remaining(En& en, int v, int rice) {
    if (v < (3 << rice)) {
      const int len = v >> rice;
      en.bypass_bits((1u << (len + 1)) - 2, len + 1);
      en.bypass_bits(v & ((1 << rice) - 1), rice);
    } else {
      int len = rice;
      int s = v - (3 << rice);
      while (s >= (1 << len)) {
        s -= 1 << len;
        ++len;
      }
      const int ones = 3 + len + 1 - rice;
      // ones-1 ones and a zero, then len bits
      for (int i = 0; i < ones - 1; ++i) en.bypass(1);
      en.bypass(0);
      en.bypass_bits(static_cast<uint32_t>(s), len);
    }
  }

  // levels of the 4x4 block at plane position (px, py) of component cidx (in the current CTB)
  HV_FN void load4x4(int cidx, int px, int py, int16_t (&rows)[4][4]) __restrict__ {
    if (lv.levels) {
      const int side = cidx ? 4 : 8, m = cidx ? 15 : 31;
      const int bit = ((py & m) >> 2) * side + ((px & m) >> 2);
      uint32_t rank;
      if (cidx == 0) {
        rank = static_cast<uint32_t>(__builtin_popcountll(nz_luma & ((1ull << bit) - 1ull)));
      } else {
        rank = static_cast<uint32_t>(__builtin_popcountll(nz_luma));
        if (cidx == 2) rank += static_cast<uint32_t>(__builtin_popcount(nz_chroma[0]));
        rank += static_cast<uint32_t>(__builtin_popcount(nz_chroma[cidx - 1] & ((1u << bit) - 1u)));
      }
      const size_t at = static_cast<size_t>(ctb_base) + rank;
      if (at < lv.nblocks) {
        HV_LDS(lv.levels);  // the device stages the CTU's blocks in LDS
        memcpy(rows, lv.levels + at * 16, 32);
        return;
      }
      if (!lv.plane[0]) {
        fail(CE_PACKED_RANGE);
        memset(rows, 0, 32);
        return;
      }
    }
    const int stride = cidx ? W / 2 : W;
    const int16_t* b = lv.plane[cidx] + static_cast<size_t>(py) * stride + px;
    for (int r = 0; r < 4; ++r) memcpy(rows[r], b + static_cast<size_t>(r) * stride, sizeof(rows[r]));
  }

  HV_FN static bool any_row(const int16_t (&rows)[4][4]) {
    uint64_t a = 0;
    for (int r = 0; r < 4; ++r) {
      uint64_t w;
      memcpy(&w, rows[r], 8);
      a |= w;
    }
    return a != 0;
  }

  // residual_coding of the (1 << log2)^2 block of component cidx at plane position (bx0, by0);
  // gmask: bit (ys * nsb + xs) set for every non-zero 4x4 sub-block of the TU (from the CTB's
  // sub-block map), so all-zero sub-blocks are never loaded
  HV_BIG void write_residual(int cidx, int bx0, int by0, int log2, int scan_idx, uint64_t gmask) __restrict__ {
    HV_LDS(this);
    HV_LDS(ctx);
    HV_LDS(P);
    const ProfScope prof_scope(prof, CP_RESIDUAL);
    const int log2sb = log2 - 2, nsb = 1 << log2sb, nsbsq = nsb * nsb;
    const uint8_t* sbs = scans_tab + (scan_idx * 4 + log2sb) * 64;
    const uint8_t* ps = scans_tab + (scan_idx * 4 + 2) * 64;
    // last significant group / position
    int last_i = -1, last_p = -1;
    int16_t lvx[16];
    for (int i = nsbsq - 1; i >= 0 && last_i < 0; --i) {
      if (!((gmask >> ((sbs[i] >> 4) * nsb + (sbs[i] & 15))) & 1u)) continue;
      int16_t rows[4][4];
      load4x4(cidx, bx0 + (sbs[i] & 15) * 4, by0 + (sbs[i] >> 4) * 4, rows);
      if (!any_row(rows)) continue;
      for (int p = 0; p < 16; ++p) lvx[p] = rows[ps[p] >> 4][ps[p] & 15];
      for (int p = 15; p >= 0; --p)
        if (lvx[p] != 0) {
          last_i = i;
          last_p = p;
          break;
        }
    }
    if (last_i < 0) {
      fail(CE_ALL_ZERO_BLOCK);
      return;
    }
    // the engine state in locals for the block (registers on the device; the member lives in
    // memory because the coder's address crosses the out-of-line calls)
    CabacEngine<Sink> en = e;
    CtxState* const cx = ctx;  // a local: stores through the contexts cannot move it
    HV_LDS(cx);
    HV_LDS(sig_tab);
    HV_LDS(scans_tab);
    HV_LDS(en.out);
    int lx = (sbs[last_i] & 15) * 4 + (ps[last_p] & 15), ly = (sbs[last_i] >> 4) * 4 + (ps[last_p] >> 4);
    if (scan_idx == 2) {
      const int t = lx;
      lx = ly;
      ly = t;
    }
    write_last(en, cx, lx, log2, cidx, CTX_LAST_X);
    write_last(en, cx, ly, log2, cidx, CTX_LAST_Y);
    write_last_suffix(en, lx);
    write_last_suffix(en, ly);

    uint8_t csbf[8][8];
    memset(csbf, 0, sizeof(csbf));
    int c1 = 1;
    bool first_sb = true;
    for (int i = last_i; i >= 0; --i) {
      const int xs = sbs[i] & 15, ys = sbs[i] >> 4;
      int16_t lvl[16];
      bool nonzero;
      if (i == last_i) {
        memcpy(lvl, lvx, sizeof(lvl));
        nonzero = true;
      } else if (!((gmask >> (ys * nsb + xs)) & 1u)) {
        nonzero = false;
      } else {
        int16_t rows[4][4];
        load4x4(cidx, bx0 + xs * 4, by0 + ys * 4, rows);
        nonzero = any_row(rows);
        if (nonzero)
          for (int p = 0; p < 16; ++p) lvl[p] = rows[ps[p] >> 4][ps[p] & 15];
      }
      bool infer_dc = false;
      if (i < last_i && i > 0) {
        int cs = 0;
        if (xs < nsb - 1) cs += csbf[xs + 1][ys];
        if (ys < nsb - 1) cs += csbf[xs][ys + 1];
        en.encode(nonzero, cx[CTX_CSBF + hv_min(cs, 1) + (cidx ? 2 : 0)]);
        csbf[xs][ys] = nonzero;
        infer_dc = true;
      } else {
        csbf[xs][ys] = 1;
        if (!nonzero) memset(lvl, 0, sizeof(lvl));  // DC group of a block: coded even if empty
      }
      if (!csbf[xs][ys]) continue;
      int prev_csbf = 0;
      if (xs < nsb - 1) prev_csbf += csbf[xs + 1][ys];
      if (ys < nsb - 1) prev_csbf += csbf[xs][ys + 1] << 1;
      // significance
      int vals[16], nsig = 0;
      if (i == last_i) vals[nsig++] = lvl[last_p];
      const uint8_t* sct = sig_tab + ((((log2 - 2) * 2 + (cidx ? 1 : 0)) * 3 + scan_idx) * 4 + prev_csbf) * 32 +
                           (xs + ys == 0 ? 16 : 0);
      CtxState* sctx = cx + CTX_SIG;
      for (int p = (i == last_i ? last_p - 1 : 15); p >= 0; --p) {
        const int v = lvl[p];
        if (p > 0 || !infer_dc) {
          en.encode(v != 0, sctx[sct[p]]);
          if (v != 0) infer_dc = false;
        }
        if (v != 0) vals[nsig++] = v;
      }
      // greater1 / greater2
      int ctx_set = (i == 0 || cidx > 0) ? 0 : 2;
      if (!first_sb && c1 == 0) ++ctx_set;
      first_sb = false;
      c1 = 1;
      int g1_first = -1;
      int g1[16];
      for (int k = 0; k < 16; ++k) g1[k] = 0;
      for (int k = 0; k < nsig && k < 8; ++k) {
        const int a = hv_abs(vals[k]);
        g1[k] = a > 1;
        en.encode(g1[k], cx[CTX_GT1 + (cidx ? 16 : 0) + ctx_set * 4 + c1]);
        if (g1[k]) {
          c1 = 0;
          if (g1_first < 0) g1_first = k;
        } else if (c1 > 0 && c1 < 3) {
          ++c1;
        }
      }
      int g2 = 0;
      if (g1_first >= 0) {
        g2 = hv_abs(vals[g1_first]) > 2;
        en.encode(g2, cx[CTX_GT2 + (cidx ? 4 : 0) + ctx_set]);
      }
      uint32_t signs = 0;
      for (int k = 0; k < nsig; ++k) signs = (signs << 1) | (vals[k] < 0);
      // sign data hiding: vals[nsig - 1] is the first significant coefficient in scan order
      int first_p = -1, last_p_g = -1;
      for (int p = 0; p < 16; ++p)
        if (lvl[p] != 0) {
          if (first_p < 0) first_p = p;
          last_p_g = p;
        }
      if (P->sdh && first_p >= 0 && last_p_g - first_p > 3) {
        int sum = 0;
        for (int k = 0; k < nsig; ++k) sum += hv_abs(vals[k]);
        if ((sum & 1) != (vals[nsig - 1] < 0 ? 1 : 0)) fail(CE_SDH_PARITY);
        en.bypass_bits(signs >> 1, nsig - 1);
      } else {
        en.bypass_bits(signs, nsig);
      }
      int rice = 0;
      for (int k = 0; k < nsig; ++k) {
        const int a = hv_abs(vals[k]);
        const int base = 1 + (k < 8 ? g1[k] : 0) + (k == g1_first ? g2 : 0);
        const int thr = k < 8 ? (k == g1_first ? 3 : 2) : 1;
        if (base == thr) {
          write_remaining(en, a - base, rice);
          if (a > 3 * (1 << rice)) rice = hv_min(rice + 1, 4);
        }
      }
    }
    e = en;
  }

  HV_FN static int mdcs(int mode) { return (mode >= 6 && mode <= 14) ? 2 : ((mode >= 22 && mode <= 30) ? 1 : 0); }

  HV_BIG void scan_ctb_nz(int x0, int y0) __restrict__ {
    HV_LDS(this);
    HV_LDS(ctx);
    HV_LDS(P);
    const ProfScope prof_scope(prof, CP_SCAN);
    const size_t ci = static_cast<size_t>(y0 / kCtb) * wctb + x0 / kCtb;
    if (lv.nzmap) {
      nz_luma = lv.nzmap[2 * ci];
      nz_chroma[0] = static_cast<uint32_t>(lv.nzmap[2 * ci + 1] & 0xFFFFu);
      nz_chroma[1] = static_cast<uint32_t>((lv.nzmap[2 * ci + 1] >> 16) & 0xFFFFu);
      ctb_base = lv.ctb_off ? lv.ctb_off[ci] : 0;
      if (lv.stage_ctu && P->ctu64) {  // blocks of the CTU's earlier 32x32 blocks (z-order)
        const int bx = x0 / kCtb, by = y0 / kCtb, q = ((by & 1) << 1) | (bx & 1);
        ctb_base = 0;
        for (int k = 0; k < q; ++k) {
          const int qx = (bx & ~1) + (k & 1), qy = (by & ~1) + (k >> 1);
          if (qx * kCtb >= W || qy * kCtb >= H) continue;
          const size_t cj = static_cast<size_t>(qy) * wctb + qx;
          ctb_base += static_cast<uint32_t>(__builtin_popcountll(lv.nzmap[2 * cj]) +
                                            __builtin_popcountll(lv.nzmap[2 * cj + 1] & 0xFFFFFFFFull));
        }
      }
      return;
    }
    nz_luma = 0;
    for (int by = 0; by < 8; ++by)
      for (int bx = 0; bx < 8; ++bx) {
        const int16_t* p = lv.plane[0] + static_cast<size_t>(y0 + by * 4) * W + x0 + bx * 4;
        uint64_t a = 0;
        for (int r = 0; r < 4; ++r) {
          uint64_t w;
          memcpy(&w, p + static_cast<size_t>(r) * W, 8);
          a |= w;
        }
        nz_luma |= static_cast<uint64_t>(a != 0) << (by * 8 + bx);
      }
    const int cw = W / 2;
    for (int c = 0; c < 2; ++c) {
      nz_chroma[c] = 0;
      for (int by = 0; by < 4; ++by)
        for (int bx = 0; bx < 4; ++bx) {
          const int16_t* p = lv.plane[1 + c] + static_cast<size_t>(y0 / 2 + by * 4) * cw + x0 / 2 + bx * 4;
          uint64_t a = 0;
          for (int r = 0; r < 4; ++r) {
            uint64_t w;
            memcpy(&w, p + static_cast<size_t>(r) * cw, 8);
            a |= w;
          }
          nz_chroma[c] |= static_cast<uint32_t>(a != 0) << (by * 4 + bx);
        }
    }
  }
  // sub-block mask of an n x n block at plane position (x, y) inside the current CTB, in
  // the block's own raster order (bit ys * (n / 4) + xs)
  HV_FN uint64_t block_mask(int cidx, int x, int y, int n) const __restrict__ {
    const int side = cidx ? 4 : 8, m = cidx ? 15 : 31;
    const uint64_t src = cidx ? nz_chroma[cidx - 1] : nz_luma;
    const int bx0 = (x & m) >> 2, by0 = (y & m) >> 2, nb = n >> 2;
    uint64_t out = 0;
    for (int r = 0; r < nb; ++r) out |= ((src >> ((by0 + r) * side + bx0)) & ((1ull << nb) - 1ull)) << (r * nb);
    return out;
  }
  HV_FN bool any_nonzero(int cidx, int x, int y, int n) const __restrict__ { return block_mask(cidx, x, y, n) != 0; }

  // ---------------------------------------------------------------- inter prediction helpers
  // A PU's motion is its direction (bit 0 list 0, bit 1 list 1) and a refIdx + vector per used
  // list; RefPicListX holds num_ref[X] pictures (POC list_poc(X, i)).
  HV_FN bool inter_avail(int x, int y) const __restrict__ {
    HV_GLOBAL(S.pred);
    return avail(x, y) && S.pred[g(x, y)] == CU_INTER;
  }
  HV_FN const Motion& mot_at(int x, int y) const __restrict__ {
    HV_GLOBAL(S.mot);
    return S.mot[g(x, y)];
  }
  // a neighbour granule's inter availability and motion, loaded unconditionally (coordinates
  // clamped into the picture): the probes of a candidate list issue together instead of one
  // dependent load after another (the motion is meaningful only where `inter`)
  struct Nb {
    bool inter;
    Motion m;
  };
  // neighbour flag probes with unconditional (clamped) loads, so a context's two probes
  // overlap: skip flag of a coded neighbour, depth of a coded neighbour deeper than d
  HV_FN int nb_skip(int xn, int yn) const __restrict__ {
    const size_t k = g(hv_clamp(xn, 0, W - 1), hv_clamp(yn, 0, H - 1));
    const uint8_t cd = S.coded[k];
    const int8_t sk = S.skip[k];
    return (inside(xn, yn) && cd && sk) ? 1 : 0;
  }
  HV_FN int nb_deeper(int xn, int yn, int d) const __restrict__ {
    const size_t k = g(hv_clamp(xn, 0, W - 1), hv_clamp(yn, 0, H - 1));
    const uint8_t cd = S.coded[k];
    const int8_t dp = S.depth[k];
    return (inside(xn, yn) && cd && dp > d) ? 1 : 0;
  }
  HV_FN Nb probe(int xn, int yn) const __restrict__ {
    const bool in = inside(xn, yn);
    const size_t k = g(hv_clamp(xn, 0, W - 1), hv_clamp(yn, 0, H - 1));
    const uint8_t cd = S.coded[k];
    const int8_t pr = S.pred[k];
    Nb r;
    r.m = S.mot[k];
    r.inter = in && cd && pr == CU_INTER;
    return r;
  }
  HV_FN int ref_poc(int l) const __restrict__ {
    return l == 0 ? (P->ref_poc[0] >= 0 ? P->ref_poc[0] : P->poc - 1) : P->ref_poc[1];
  }
  HV_FN int nref(int l) const __restrict__ { return hv_max(1, P->num_ref[l]); }
  HV_FN int list_poc(int l, int i) const __restrict__ { return i == 0 ? ref_poc(l) : P->list_poc[l][i]; }

  HV_FN static Mv scale_mv(Mv v, int td0, int tb0) {  // 8.5.3.2.8 (8-209 .. 8-213)
    const int td = hv_clamp(td0, -128, 127), tb = hv_clamp(tb0, -128, 127);
    const int tx = (16384 + (hv_abs(td) >> 1)) / td;
    const int dsf = hv_clamp((tb * tx + 32) >> 6, -4096, 4095);
    const int px = dsf * v.x, py = dsf * v.y;
    const int sx = hv_clamp((px < 0 ? -1 : 1) * ((hv_abs(px) + 127) >> 8), -32768, 32767);
    const int sy = hv_clamp((py < 0 ? -1 : 1) * ((hv_abs(py) + 127) >> 8), -32768, 32767);
    return Mv{static_cast<int16_t>(sx), static_cast<int16_t>(sy)};
  }

  // 8.5.3.2.8 / 8.5.3.2.9 temporal vector of list X (target refIdx ri) for the PU (x, y, n x n)
  // the collocated records of a PU (8.5.3.2.8): bottom-right and centre candidates, both loaded
  // up front (one memory latency for the pair, shared by the L0 and L1 derivations)
  struct ColPair {
    CuInfo br, ce;
    bool br_ok, ce_ok;
  };
  HV_FN const CuInfo& col_rec(int xc, int yc) const __restrict__ {
    const int ci = (yc >> kCtbLog2) * wctb + (xc >> kCtbLog2);
    return col_cu[static_cast<size_t>(ci) * kCusPerCtb + zorder8((xc & (kCtb - 1)) >> 3, (yc & (kCtb - 1)) >> 3)];
  }
  HV_FN ColPair col_pair(int x, int y, int n) const __restrict__ {
    ColPair c;
    const int xbr = ((x + n) >> 4) << 4, ybr = ((y + n) >> 4) << 4;
    const int xce = ((x + (n >> 1)) >> 4) << 4, yce = ((y + (n >> 1)) >> 4) << 4;
    c.br_ok = tmvp && col_cu && (y >> L) == ((y + n) >> L) && y + n < H && x + n < W && xbr < W && ybr < H;
    c.ce_ok = tmvp && col_cu && xce < W && yce < H;
    if (col_cu) {
      c.br = col_rec(hv_min(xbr, W - 1), hv_min(ybr, H - 1));
      c.ce = col_rec(hv_min(xce, W - 1), hv_min(yce, H - 1));
    }
    return c;
  }
  // 8.5.3.2.9 temporal vector of list X (target refIdx ri) from a collocated record
  HV_FN bool col_mv(const CuInfo& cc, int X, int ri, Mv* out) __restrict__ {
    if (cc.pred != CU_INTER) return false;
    const int dir = cu_dir(cc);
    int list;
    if (!(dir & 1)) list = 1;
    else if (dir == DIR_L0) list = 0;
    else list = no_backward ? X : (col_l1 ? 0 : 1);  // N = collocated_from_l0_flag
    Mv v = list == 0 ? Mv{cc.mv[0], cc.mv[1]} : Mv{cc.mv1[0], cc.mv1[1]};
    int cr = cc.pad[list];
    if (cr >= 4) {
      fail(CE_COL_REFIDX);
      cr = 0;
    }
    const int col_diff = P->col_poc - (cr == 0 ? P->col_ref_poc[list] : P->col_list_poc[list][cr]);
    const int cur_diff = P->poc - list_poc(X, ri);
    if (col_diff != cur_diff && col_diff != 0) v = scale_mv(v, col_diff, cur_diff);
    *out = v;
    return true;
  }
  HV_FN bool temporal(const ColPair& c, int X, int ri, Mv* out) __restrict__ {
    if (c.br_ok && col_mv(c.br, X, ri, out)) return true;
    return c.ce_ok && col_mv(c.ce, X, ri, out);
  }

  // 8.5.3.2.2-8.5.3.2.5 merge candidates of a 2Nx2N PU (MaxNumMergeCand entries)
  HV_BIG int merge_list(int x, int y, int n, Motion* out) __restrict__ {
    HV_LDS(this);
    HV_LDS(ctx);
    HV_LDS(P);
    const ProfScope prof_scope(prof, CP_MERGE);
    Motion cand[8];
    int k = 0;
    const Motion none = motion_none();
    const Nb na1 = probe(x - 1, y + n - 1), nb1 = probe(x + n - 1, y - 1), nb0 = probe(x + n, y - 1);
    const Nb na0 = probe(x - 1, y + n), nb2 = probe(x - 1, y - 1);
    const bool a1 = na1.inter, av_b1 = nb1.inter;
    const Motion ma1 = a1 ? na1.m : none, mb1 = av_b1 ? nb1.m : none;
    const bool b1 = av_b1 && !(a1 && ma1 == mb1);
    bool b0 = nb0.inter, a0 = na0.inter, b2 = nb2.inter;
    const Motion mb0 = b0 ? nb0.m : none, ma0 = a0 ? na0.m : none;
    const Motion mb2 = b2 ? nb2.m : none;
    if (b0 && av_b1 && mb1 == mb0) b0 = false;
    if (a0 && a1 && ma1 == ma0) a0 = false;
    if (b2 && ((a1 && ma1 == mb2) || (av_b1 && mb1 == mb2))) b2 = false;
    if (a0 + a1 + b0 + b1 == 4) b2 = false;
    if (a1) cand[k++] = ma1;
    if (b1) cand[k++] = mb1;
    if (b0) cand[k++] = mb0;
    if (a0) cand[k++] = ma0;
    if (b2) cand[k++] = mb2;
    if (k < P->max_merge && tmvp) {
      Motion t = none;
      const ColPair cp = col_pair(x, y, n);
      if (temporal(cp, 0, 0, &t.m[0])) t.dir |= DIR_L0;  // refIdx 0 (8.5.3.2.8 merge: refIdxLXCol 0)
      if (bslice && temporal(cp, 1, 0, &t.m[1])) t.dir |= DIR_L1;
      if (t.dir) cand[k++] = t;
    }
    const int orig = k;
    if (bslice && orig > 1 && orig < P->max_merge) {  // combined bi-predictive candidates
      for (int comb = 0; comb < orig * (orig - 1) && k < P->max_merge; ++comb) {
        const Motion c0 = cand[kCombL0[comb]], c1 = cand[kCombL1[comb]];
        if ((c0.dir & DIR_L0) && (c1.dir & DIR_L1) &&
            (list_poc(0, c0.r[0]) != list_poc(1, c1.r[1]) || !(c0.m[0] == c1.m[1]))) {
          Motion m = none;
          m.dir = DIR_BI;
          m.r[0] = c0.r[0];
          m.r[1] = c1.r[1];
          m.m[0] = c0.m[0];
          m.m[1] = c1.m[1];
          cand[k++] = m;
        }
      }
    }
    // zero candidates (8.5.3.2.5): refIdx 0, 1, .. up to the active list size, then 0
    const int nzr = bslice ? hv_min(nref(0), nref(1)) : nref(0);
    for (int zi = 0; k < P->max_merge; ++zi) {
      const int8_t r = static_cast<int8_t>(zi < nzr ? zi : 0);
      Motion m = none;
      m.dir = static_cast<uint8_t>(bslice ? DIR_BI : DIR_L0);
      m.r[0] = m.r[1] = r;
      cand[k++] = m;
    }
    const int nm = hv_min(k, P->max_merge);
    for (int i = 0; i < nm; ++i) out[i] = cand[i];
    return nm;
  }

  // a neighbour vector pointing at the target picture (8.5.3.2.7, no scaling)
  HV_FN bool amvp_same(const Motion& m, int X, int tgt, Mv* v) const __restrict__ {
    const int Y = 1 - X;
    if ((m.dir >> X) & 1 && list_poc(X, m.r[X]) == tgt) {
      *v = m.m[X];
      return true;
    }
    if ((m.dir >> Y) & 1 && list_poc(Y, m.r[Y]) == tgt) {
      *v = m.m[Y];
      return true;
    }
    return false;
  }
  // any vector of the neighbour, scaled by the POC distances
  HV_FN bool amvp_scaled(const Motion& m, int X, int tgt, Mv* v) const __restrict__ {
    for (int j = 0; j < 2; ++j) {
      const int Lx = j == 0 ? X : 1 - X;
      if (!((m.dir >> Lx) & 1)) continue;
      const int td = P->poc - list_poc(Lx, m.r[Lx]), tb = P->poc - tgt;
      *v = (td != tb && td != 0) ? scale_mv(m.m[Lx], td, tb) : m.m[Lx];
      return true;
    }
    return false;
  }

  // 8.5.3.2.6-8.5.3.2.7 AMVP candidates of list X, refIdx ri
  HV_BIG void amvp_list(int x, int y, int n, int X, int ri, Mv* out) __restrict__ {
    HV_LDS(this);
    HV_LDS(ctx);
    HV_LDS(P);
    const ProfScope prof_scope(prof, CP_AMVP);
    const int tgt = list_poc(X, ri);
    const ColPair cp = col_pair(x, y, n);  // issued with the spatial probes
    const Nb pa[2] = {probe(x - 1, y + n), probe(x - 1, y + n - 1)};
    const Nb pb[3] = {probe(x + n, y - 1), probe(x + n - 1, y - 1), probe(x - 1, y - 1)};
    const bool is_scaled = pa[0].inter || pa[1].inter;
    bool fa = false, fb = false;
    Mv ma{0, 0}, mb{0, 0};
    for (int k = 0; k < 2 && !fa; ++k)
      if (pa[k].inter) fa = amvp_same(pa[k].m, X, tgt, &ma);
    for (int k = 0; k < 2 && !fa; ++k)
      if (pa[k].inter) fa = amvp_scaled(pa[k].m, X, tgt, &ma);
    for (int k = 0; k < 3 && !fb; ++k)
      if (pb[k].inter) fb = amvp_same(pb[k].m, X, tgt, &mb);
    if (!is_scaled && fb) {
      ma = mb;
      fa = true;
    }
    if (!is_scaled) {
      fb = false;
      for (int k = 0; k < 3 && !fb; ++k)
        if (pb[k].inter) fb = amvp_scaled(pb[k].m, X, tgt, &mb);
    }
    int k = 0;
    if (fa) out[k++] = ma;
    if (fb && !(fa && ma == mb)) out[k++] = mb;
    if (k < 2) {
      Mv t{0, 0};
      if (temporal(cp, X, ri, &t)) out[k++] = t;
    }
    while (k < 2) out[k++] = Mv{0, 0};
  }

  // ---------------------------------------------------------------- coding unit (7.3.8.5)
  HV_FN void mark(int x, int y, int n, int d, int sk, int pm, int md, const Motion& mv) __restrict__ {
    HV_GLOBAL(S.depth);
    HV_GLOBAL(S.skip);
    HV_GLOBAL(S.pred);
    HV_GLOBAL(S.mode4);
    HV_GLOBAL(S.mot);
    HV_GLOBAL(S.coded);
    for (int yy = y; yy < y + n; yy += 8)
      for (int xx = x; xx < x + n; xx += 8) {
        const size_t k = g(xx, yy);
        S.depth[k] = static_cast<int8_t>(d);
        S.skip[k] = static_cast<int8_t>(sk);
        S.pred[k] = static_cast<int8_t>(pm);
        for (int q = 0; q < 4; ++q) S.mode4[g4(xx + (q & 1) * 4, yy + (q >> 1) * 4)] = static_cast<int8_t>(md);
        S.mot[k] = mv;
        S.coded[k] = 1;
      }
  }

  // inter_pred_idc (9.3.3.7, 2Nx2N PU of a CU at depth d): PRED_BI "1", PRED_L0 "00", PRED_L1 "01"
  HV_FN void write_inter_pred_idc(int dir, int d) __restrict__ {
    e.encode(dir == DIR_BI, ctx[CTX_INTER_PRED + d]);
    if (dir != DIR_BI) e.encode(dir == DIR_L1, ctx[CTX_INTER_PRED + 4]);
  }

  // a CU, then the QpY of its granules (8.6.1: the quantization group's prediction until a
  // cu_qp_delta has been coded, the coded QP from then on)
  HV_FN void write_cu(int x, int y, int log2, int d) __restrict__ {
    write_cu_body(x, y, log2, d);
    const int q = qp_coded ? qp_ctb : qp_pred_cur, n = 1 << log2;
    for (int yy = y; yy < y + n; yy += 8)
      for (int xx = x; xx < x + n; xx += 8) S.qpy[g(xx, yy)] = static_cast<int8_t>(q);
  }

  HV_FN Motion cu_motion(const CuInfo& ci) const __restrict__ {
    Motion mv = motion_none();
    mv.dir = static_cast<uint8_t>(cu_dir(ci));
    mv.r[0] = static_cast<int8_t>(ci.pad[0]);
    mv.r[1] = static_cast<int8_t>(ci.pad[1]);
    mv.m[0] = Mv{ci.mv[0], ci.mv[1]};
    mv.m[1] = Mv{ci.mv1[0], ci.mv1[1]};
    return mv;
  }

  HV_BIG void write_cu_body(int x, int y, int log2, int d) __restrict__ {
    HV_LDS(this);
    HV_LDS(ctx);
    HV_LDS(P);
    const ProfScope prof_scope(prof, CP_CU);
    const int n = 1 << log2;
    const CuInfo& ci = cu_at(x, y);
    const bool cb_y = any_nonzero(0, x, y, n);
    const bool cb_cb = any_nonzero(1, x / 2, y / 2, n / 2), cb_cr = any_nonzero(2, x / 2, y / 2, n / 2);
    const bool intra = ci.pred == CU_INTRA || !inter_slice;
    Motion mv = cu_motion(ci);
    if (!intra && (mv.dir & ~3 || (!bslice && mv.dir != DIR_L0))) fail(CE_DIRECTION);
    if (!intra && (((mv.dir & DIR_L0) && (mv.r[0] < 0 || mv.r[0] >= nref(0))) ||
                   ((mv.dir & DIR_L1) && (mv.r[1] < 0 || mv.r[1] >= nref(1)))))
      fail(CE_REFIDX);
    for (int X = 0; X < 2; ++X)
      if (!((mv.dir >> X) & 1)) {
        mv.m[X] = Mv{0, 0};
        mv.r[X] = 0;
      }
    if (inter_slice) {
      const int skip_ctx = nb_skip(x - 1, y) + nb_skip(x, y - 1);
      int midx = -1;
      if (!intra) {
        Motion ml[5];
        const int nm = merge_list(x, y, n, ml);
        for (int k = 0; k < nm; ++k)
          if (ml[k] == mv) {
            midx = k;
            break;
          }
      }
      const bool is_skip = !intra && midx >= 0 && !cb_y && !cb_cb && !cb_cr;
      e.encode(is_skip, ctx[CTX_CU_SKIP + skip_ctx]);
      if (is_skip) {
        write_merge_idx(midx);
        mark(x, y, n, d, 1, CU_INTER, 1, mv);
        ++st.skip_cus;
        return;
      }
      e.encode(intra, ctx[CTX_PRED_MODE]);
      if (!intra) {
        e.encode(1, ctx[CTX_PART_MODE]);  // PART_2Nx2N
        const bool merge = midx >= 0;
        e.encode(merge, ctx[CTX_MERGE_FLAG]);
        if (merge) {
          write_merge_idx(midx);
          ++st.merge_cus;
        } else {
          if (bslice) write_inter_pred_idc(mv.dir, d);
          for (int X = 0; X < 2; ++X) {
            if (!((mv.dir >> X) & 1)) continue;
            if (nref(X) > 1) write_ref_idx(mv.r[X], nref(X) - 1);
            Mv ap[2];
            amvp_list(x, y, n, X, mv.r[X], ap);
            const Mv v = mv.m[X];
            const int c0 = hv_abs(v.x - ap[0].x) + hv_abs(v.y - ap[0].y);
            const int c1 = hv_abs(v.x - ap[1].x) + hv_abs(v.y - ap[1].y);
            const int idx = c1 < c0 ? 1 : 0;
            write_mvd_pair(v.x - ap[idx].x, v.y - ap[idx].y);  // (mvd_l1_zero_flag 0)
            e.encode(idx, ctx[CTX_MVP_IDX]);
          }
        }
        const bool root = cb_y || cb_cb || cb_cr;
        if (!merge) e.encode(root, ctx[CTX_RQT_ROOT_CBF]);
        mark(x, y, n, d, 0, CU_INTER, 1, mv);
        ++st.inter_cus;
        if (root) {
          if (ci.flags & 16) write_tu_inter_split(x, y, log2, cb_cb, cb_cr);
          else write_tu(x, y, log2, false, 0, cb_y, cb_cb, cb_cr);
        }
        return;
      }
    }
    // intra CU: PART_2Nx2N, or PART_NxN at the minimum CB size (four 4x4 PUs, CuInfo flags
    // bit 3, PU modes in the bytes of the unused motion vector)
    const bool nxn = log2 == kMinCbLog2 && (ci.flags & 8);
    if (log2 == kMinCbLog2) e.encode(nxn ? 0 : 1, ctx[CTX_PART_MODE]);
    const int npu = nxn ? 4 : 1, h = nxn ? n / 2 : n;
    int m[4] = {0, 0, 0, 0}, mpm[4] = {-1, -1, -1, -1}, rem[4] = {0, 0, 0, 0};
    for (int k = 0; k < npu; ++k) {
      m[k] = nxn ? reinterpret_cast<const uint8_t*>(ci.mv)[k] : ci.mode;
      if (m[k] > 34) {
        fail(CE_INTRA_MODE);
        m[k] = 1;
      }
      const int xk = x + (k & 1) * h, yk = y + (k >> 1) * h;
      // 8.4.2 most probable modes; an NxN PU's left / above neighbour may be an earlier PU
      const int ca = mpm_cand(x, y, h, m, xk - 1, yk, yk, false);
      const int cb = mpm_cand(x, y, h, m, xk, yk - 1, yk, true);
      int cand[3];
      if (ca == cb) {
        if (ca < 2) {
          cand[0] = 0;
          cand[1] = 1;
          cand[2] = 26;
        } else {
          cand[0] = ca;
          cand[1] = 2 + ((ca + 29) % 32);
          cand[2] = 2 + ((ca - 2 + 1) % 32);
        }
      } else {
        cand[0] = ca;
        cand[1] = cb;
        cand[2] = (ca != 0 && cb != 0) ? 0 : ((ca != 1 && cb != 1) ? 1 : 26);
      }
      mpm[k] = -1;
      for (int j = 0; j < 3; ++j)
        if (cand[j] == m[k]) mpm[k] = j;
      // ascending order of the three candidates
      if (cand[0] > cand[1]) { const int t = cand[0]; cand[0] = cand[1]; cand[1] = t; }
      if (cand[1] > cand[2]) { const int t = cand[1]; cand[1] = cand[2]; cand[2] = t; }
      if (cand[0] > cand[1]) { const int t = cand[0]; cand[0] = cand[1]; cand[1] = t; }
      rem[k] = m[k];
      for (int j = 2; j >= 0; --j)
        if (rem[k] > cand[j]) --rem[k];
    }
    for (int k = 0; k < npu; ++k) e.encode(mpm[k] >= 0, ctx[CTX_PREV_INTRA]);
    for (int k = 0; k < npu; ++k) {
      if (mpm[k] >= 0) {
        e.bypass(mpm[k] > 0);
        if (mpm[k] > 0) e.bypass(mpm[k] > 1);
      } else {
        e.bypass_bits(rem[k], 5);
      }
    }
    e.encode(0, ctx[CTX_CHROMA_MODE]);  // intra_chroma_pred_mode = 4 (DM: the mode of PU 0)
    mark(x, y, n, d, 0, CU_INTRA, m[0], motion_none());
    if (nxn)
      for (int k = 1; k < 4; ++k) S.mode4[g4(x + (k & 1) * h, y + (k >> 1) * h)] = static_cast<int8_t>(m[k]);
    ++st.intra_cus;
    if (nxn) write_tu_nxn(x, y, m, cb_cb, cb_cr);
    else write_tu(x, y, log2, true, m[0], cb_y, cb_cb, cb_cr);
  }

  // MPM candidate (8.4.2) from the neighbour (xn, yn) of the PU at row yk of the CU at (x, y)
  // with PUs of size h and modes m
  HV_FN int mpm_cand(int x, int y, int h, const int* m, int xn, int yn, int yk, bool above) const __restrict__ {
    if (xn >= x && yn >= y) return m[(xn - x >= h) + 2 * (yn - y >= h)];
    // the three loads unconditional (clamped), then the availability logic
    const int xc = hv_clamp(xn, 0, W - 1), yc = hv_clamp(yn, 0, H - 1);
    const uint8_t cd = S.coded[g(xc, yc)];
    const int8_t pr = S.pred[g(xc, yc)];
    const int md = S.mode4[g4(xc, yc)];
    if (!inside(xn, yn) || !cd || pr != CU_INTRA) return 1;
    if (above && (yn >> L) != (yk >> L)) return 1;
    return md;
  }

  // transform_tree of an intra PART_NxN CU (7.3.8.8 / 7.3.8.10): chroma cbfs at depth 0,
  // split_transform_flag inferred (IntraSplitFlag), four 4x4 luma TUs with cbf_luma at
  // depth 1; cbfChroma of every 4x4 TU is the parent's, and the 4x4 chroma blocks follow
  // the last luma TU (blkIdx 3)
  HV_BIG void write_tu_nxn(int x, int y, const int* m, bool cb_cb, bool cb_cr) __restrict__ {
    HV_LDS(this);
    HV_LDS(ctx);
    HV_LDS(P);
    e.encode(cb_cb, ctx[CTX_CBF_CHROMA + 0]);
    e.encode(cb_cr, ctx[CTX_CBF_CHROMA + 0]);
    for (int k = 0; k < 4; ++k) {
      const int xk = x + (k & 1) * 4, yk = y + (k >> 1) * 4;
      const bool cy = any_nonzero(0, xk, yk, 4);
      e.encode(cy, ctx[CTX_CBF_LUMA + 0]);
      if (P->cu_qp_delta && !qp_coded && (cy || cb_cb || cb_cr)) write_qp_delta();
      if (cy) write_residual(0, xk, yk, 2, mdcs(m[k]), 1);
    }
    if (cb_cb) write_residual(1, x / 2, y / 2, 2, mdcs(m[0]), 1);
    if (cb_cr) write_residual(2, x / 2, y / 2, 2, mdcs(m[0]), 1);
  }

  // ref_idx_lX (9.3.3.1 TR, cMax = num_ref_idx_active - 1): two context-coded bins, then bypass
  HV_FN void write_ref_idx(int r, int cmax) __restrict__ {
    for (int i = 0; i < cmax; ++i) {
      const int b = r > i;
      if (i < 2) e.encode(b, ctx[CTX_REF_IDX + i]);
      else e.bypass(b);
      if (!b) break;
    }
  }

  HV_FN void write_merge_idx(int idx) __restrict__ {
    if (P->max_merge <= 1) return;
    e.encode(idx > 0, ctx[CTX_MERGE_IDX]);
    for (int k = 1; k < P->max_merge - 1 && idx >= k; ++k) e.bypass(idx > k);
  }

  HV_FN void write_mvd_pair(int dx, int dy) __restrict__ {
    const int ax = hv_abs(dx), ay = hv_abs(dy);
    e.encode(ax > 0, ctx[CTX_MVD_G0]);
    e.encode(ay > 0, ctx[CTX_MVD_G0]);
    if (ax > 0) e.encode(ax > 1, ctx[CTX_MVD_G1]);
    if (ay > 0) e.encode(ay > 1, ctx[CTX_MVD_G1]);
    if (ax > 0) {
      if (ax > 1) write_egk(static_cast<uint32_t>(ax - 2), 1);
      e.bypass(dx < 0);
    }
    if (ay > 0) {
      if (ay > 1) write_egk(static_cast<uint32_t>(ay - 2), 1);
      e.bypass(dy < 0);
    }
  }

  // inter CU whose residual quadtree splits once (CuInfo flags bit 4): split_transform_flag,
  // chroma cbfs at depth 0, then per quarter TU (z-order) its chroma cbfs under a set parent,
  // cbf_luma (always coded below depth 0) and the transform unit
  HV_BIG void write_tu_inter_split(int x, int y, int log2, bool cb_cb, bool cb_cr) __restrict__ {
    HV_LDS(this);
    HV_LDS(ctx);
    HV_LDS(P);
    if (P->tu_inter_depth < 1 || log2 < 4) fail(CE_INTER_SPLIT);
    e.encode(1, ctx[CTX_SPLIT_TRANSFORM + 5 - log2]);
    e.encode(cb_cb, ctx[CTX_CBF_CHROMA + 0]);
    e.encode(cb_cr, ctx[CTX_CBF_CHROMA + 0]);
    const int h = 1 << (log2 - 1);
    for (int k = 0; k < 4; ++k) {
      const int xc = x + (k & 1) * h, yc = y + (k >> 1) * h;
      const bool ccb = cb_cb && any_nonzero(1, xc / 2, yc / 2, h / 2);
      const bool ccr = cb_cr && any_nonzero(2, xc / 2, yc / 2, h / 2);
      if (cb_cb) e.encode(ccb, ctx[CTX_CBF_CHROMA + 1]);
      if (cb_cr) e.encode(ccr, ctx[CTX_CBF_CHROMA + 1]);
      const bool cy = any_nonzero(0, xc, yc, h);
      e.encode(cy, ctx[CTX_CBF_LUMA + 0]);
      if (P->cu_qp_delta && !qp_coded && (cy || ccb || ccr)) write_qp_delta();
      if (cy) write_residual(0, xc, yc, log2 - 1, 0, block_mask(0, xc, yc, h));
      if (ccb) write_residual(1, xc / 2, yc / 2, log2 - 2, 0, block_mask(1, xc / 2, yc / 2, h / 2));
      if (ccr) write_residual(2, xc / 2, yc / 2, log2 - 2, 0, block_mask(2, xc / 2, yc / 2, h / 2));
    }
  }

  // transform_tree at depth 0 with TU = CU (7.3.8.8 / 7.3.8.10)
  HV_BIG void write_tu(int x, int y, int log2, bool intra, int m, bool cb_y, bool cb_cb, bool cb_cr) __restrict__ {
    HV_LDS(this);
    HV_LDS(ctx);
    HV_LDS(P);
    // split_transform_flag 0 where the inter depth allows a split (intra: depth 0 at 2Nx2N)
    if (!intra && P->tu_inter_depth > 0 && log2 > 2) e.encode(0, ctx[CTX_SPLIT_TRANSFORM + 5 - log2]);
    e.encode(cb_cb, ctx[CTX_CBF_CHROMA + 0]);
    e.encode(cb_cr, ctx[CTX_CBF_CHROMA + 0]);
    if (intra || cb_cb || cb_cr) e.encode(cb_y, ctx[CTX_CBF_LUMA + 1]);
    else if (!cb_y) fail(CE_CBF_LUMA);
    if (P->cu_qp_delta && !qp_coded && (cb_y || cb_cb || cb_cr)) write_qp_delta();
    if (cb_y) {
      const int scan = (intra && log2 == 3) ? mdcs(m) : 0;
      write_residual(0, x, y, log2, scan, block_mask(0, x, y, 1 << log2));
    }
    const int scan_c = (intra && log2 - 1 == 2) ? mdcs(m) : 0;
    const int nc = 1 << (log2 - 1);
    if (cb_cb) write_residual(1, x / 2, y / 2, log2 - 1, scan_c, block_mask(1, x / 2, y / 2, nc));
    if (cb_cr) write_residual(2, x / 2, y / 2, log2 - 1, scan_c, block_mask(2, x / 2, y / 2, nc));
  }

  // cu_qp_delta_abs (9.3.3.10: TR prefix cMax 5, ctxInc 0 then 1; EG0 bypass suffix) and
  // the bypass sign, in the first TU of the quantization group with a coded block
  HV_BIG void write_qp_delta() __restrict__ {
    HV_LDS(this);
    HV_LDS(ctx);
    HV_LDS(P);
    const int d = qp_ctb - qp_pred_cur;
    const int qbd = 6 * (P->bit_depth - 8);
    if (d < -(26 + qbd / 2) || d > 25 + qbd / 2) fail(CE_QP_DELTA);
    const int a = hv_abs(d), pre = hv_min(a, 5);
    for (int i = 0; i < pre; ++i) e.encode(1, ctx[CTX_CU_QP_DELTA + (i > 0)]);
    if (pre < 5) e.encode(0, ctx[CTX_CU_QP_DELTA + (pre > 0)]);
    else write_egk(static_cast<uint32_t>(a - 5), 0);
    if (a) e.bypass(d < 0);
    qp_coded = true;
  }
  HV_FN void write_egk(uint32_t v, int k) __restrict__ {  // 9.3.3.3 k-th order Exp-Golomb, bypass
    while (v >= (1u << k)) {
      e.bypass(1);
      v -= 1u << k;
      ++k;
    }
    e.bypass(0);
    while (k--) e.bypass((v >> k) & 1);
  }

  // qPY_PRED of the quantization group at (xq, yq) (8.6.1): the average of the QpY left of and
  // above it when those lie in the same CTB, each replaced by qPY_PREV otherwise
  HV_FN int qg_pred(int xq, int yq) const __restrict__ {
    const bool la = avail(xq - 1, yq) && ((xq - 1) >> L) == (xq >> L) && (yq >> L) == (yq >> L);
    const bool lb = avail(xq, yq - 1) && (xq >> L) == (xq >> L) && ((yq - 1) >> L) == (yq >> L);
    const int qa = la ? S.qpy[g(xq - 1, yq)] : qp_prev;
    const int qb = lb ? S.qpy[g(xq, yq - 1)] : qp_prev;
    return (qa + qb + 1) >> 1;
  }

  // coding_quadtree (7.3.8.4) of one CTU (CTU coordinates)
  HV_BIG void write_ctu(int cx, int cy) __restrict__ {
    HV_LDS(this);
    HV_LDS(ctx);
    HV_LDS(P);
    if (!P->ctu64) {
      write_block_tree(cx, cy, 0);
      return;
    }
    const int x0 = cx << 6, y0 = cy << 6;
    const bool inside64 = x0 + 64 <= W && y0 + 64 <= H;
    const bool one = inside64 && cu64_ok(cx, cy);
    if (inside64) e.encode(!one, ctx[CTX_SPLIT_CU + split_ctx(x0, y0, 0)]);  // else the split is inferred
    if (one) {
      write_cu64_skip(x0, y0);
      return;
    }
    for (int q = 0; q < 4; ++q) {
      const int bx = (x0 >> 5) + (q & 1), by = (y0 >> 5) + (q >> 1);
      if ((bx << 5) < W && (by << 5) < H) write_block_tree(bx, by, 1);
    }
  }

  HV_FN int split_ctx(int x, int y, int d) const __restrict__ {
    return nb_deeper(x - 1, y, d) + nb_deeper(x, y - 1, d);
  }

  // one 32x32 record block = one quantization group; dofs: its depth in the CTU quadtree
  HV_BIG void write_block_tree(int rx, int ry, int dofs) __restrict__ {
    HV_LDS(this);
    HV_LDS(ctx);
    HV_LDS(P);
    const CtuInfo& t = ctu[ry * wctb + rx];
    const int x0 = rx * kCtb, y0 = ry * kCtb;
    qp_ctb = t.qp;
    qp_coded = false;
    qp_pred_cur = P->cu_qp_delta ? qg_pred(x0, y0) : P->qp;
    scan_ctb_nz(x0, y0);
    const bool s32 = t.split & 1;
    e.encode(s32, ctx[CTX_SPLIT_CU + split_ctx(x0, y0, dofs)]);
    if (!s32) {
      write_cu(x0, y0, 5, dofs);
    } else {
      for (int q = 0; q < 4; ++q) {
        const int x1 = x0 + (q & 1) * 16, y1 = y0 + (q >> 1) * 16;
        const bool s16 = (t.split >> (1 + q)) & 1;
        e.encode(s16, ctx[CTX_SPLIT_CU + split_ctx(x1, y1, dofs + 1)]);
        if (!s16) {
          write_cu(x1, y1, 4, dofs + 1);
          continue;
        }
        for (int r = 0; r < 4; ++r) write_cu(x1 + (r & 1) * 8, y1 + (r >> 1) * 8, 3, dofs + 2);
      }
    }
    // qPY_PREV of the next quantization group: the QpY of this group's last CU
    if (P->cu_qp_delta) qp_prev = qp_coded ? qp_ctb : qp_pred_cur;
  }

  // a 64x64 skip CU stands for the CTU's four blocks when each is one 32x32 inter CU, all with
  // one motion, no level anywhere, and that motion is in the 64x64 CU's merge list (the
  // reconstruction is the same: motion compensation is per sample and every inner edge has
  // boundary strength 0)
  HV_BIG bool cu64_ok(int cx, int cy) __restrict__ {
    HV_LDS(this);
    HV_LDS(ctx);
    HV_LDS(P);
    const int x0 = cx << 6, y0 = cy << 6;
    if (!inter_slice) return false;
    Motion m0 = motion_none();
    for (int q = 0; q < 4; ++q) {
      const int bx = (x0 >> 5) + (q & 1), by = (y0 >> 5) + (q >> 1);
      const CtuInfo& t = ctu[by * wctb + bx];
      const CuInfo& ci = cu_at(bx << 5, by << 5);
      if ((t.split & 1) || ci.pred != CU_INTER) return false;
      Motion m = cu_motion(ci);
      for (int X = 0; X < 2; ++X)
        if (!((m.dir >> X) & 1)) {
          m.m[X] = Mv{0, 0};
          m.r[X] = 0;
        }
      if (q == 0) m0 = m;
      else if (!(m == m0)) return false;
      scan_ctb_nz(bx << 5, by << 5);
      if (nz_luma || nz_chroma[0] || nz_chroma[1]) return false;
    }
    Motion ml[5];
    const int nm = merge_list(x0, y0, 64, ml);
    cu64_midx = -1;
    for (int k = 0; k < nm && cu64_midx < 0; ++k)
      if (ml[k] == m0) cu64_midx = k;
    cu64_mot = m0;
    return cu64_midx >= 0;
  }
  HV_FN void write_cu64_skip(int x0, int y0) __restrict__ {
    const int skip_ctx = nb_skip(x0 - 1, y0) + nb_skip(x0, y0 - 1);
    e.encode(1, ctx[CTX_CU_SKIP + skip_ctx]);
    write_merge_idx(cu64_midx);
    mark(x0, y0, 64, 0, 1, CU_INTER, 1, cu64_mot);
    ++st.skip_cus;
    // one quantization group per CU at least as large as the group: QpY = the prediction
    const int q = P->cu_qp_delta ? qg_pred(x0, y0) : P->qp;
    for (int yy = y0; yy < y0 + 64; yy += 8)
      for (int xx = x0; xx < x0 + 64; xx += 8) S.qpy[g(xx, yy)] = static_cast<int8_t>(q);
    if (P->cu_qp_delta) qp_prev = q;
  }

  // SAO + coding quadtree of CTU (rx, ry) and its end_of_slice_segment_flag; with WPP, a
  // row's last CTU also codes end_of_subset_one_bit, flushes and byte-aligns its substream
  HV_BIG void code_ctu(int rx, int ry) __restrict__ {
    HV_LDS(this);
    HV_LDS(ctx);
    HV_LDS(P);
    const ProfScope prof_scope(prof, CP_CTU);
    if (P->sao) write_sao(rx, ry);
    write_ctu(rx, ry);
    const bool last = ry == P->hctu - 1 && rx == P->wctu - 1;
    e.terminate(last);  // end_of_slice_segment_flag
    if (P->wpp && rx == P->wctu - 1 && !last) e.terminate(1);  // end_of_subset_one_bit
    if (last || (P->wpp && rx == P->wctu - 1)) {
      e.finish();
      // byte_alignment() after end_of_subset_one_bit; the last stop bit is the
      // rbsp_slice_segment_trailing_bits
      e.out->put(1, 1);
      e.out->align_zero();
    }
  }
};

}  // namespace hevc
}  // namespace mivc
