// H.265 / HEVC constant tables shared by the host bitstream library (CABAC writer,
// independent CPU decoder) and the gfx950 HIP kernels.
//
// Each table names its clause of ITU-T H.265 (v1 / Main and Main 10 profiles).
// The reference repository has no codec code: its HEVC path is the string
// "-vcodec libx265 -crf 26" handed to ffmpeg (server.go:67-68, client.go:115).
#pragma once
#include <cstdint>

#include "h264_tables.h"  // MIVC_HD

namespace mivc {
namespace hevc {

// ---------------------------------------------------------------- coding structure of this encoder
constexpr int kCtbLog2 = 5;                  // 32x32 coding tree blocks
constexpr int kCtb = 1 << kCtbLog2;
constexpr int kMinCbLog2 = 3;                // 8x8 minimum coding block
constexpr int kCusPerCtb = (kCtb / 8) * (kCtb / 8);  // 8x8 granules per CTB (z-order)

// ---------------------------------------------------------------- intra prediction (8.4.4.2.6)
// intraPredAngle for predModeIntra 0..34 (0/1 planar/DC unused)
static constexpr int8_t kIntraPredAngle[35] = {0,   0,   32,  26,  21,  17,  13,  9,   5,  2,  0,  -2,
                                               -5,  -9,  -13, -17, -21, -26, -32, -26, -21, -17, -13, -9,
                                               -5,  -2,  0,   2,   5,   9,   13,  17,  21,  26,  32};
// invAngle for predModeIntra 11..25 (index mode - 11)
static constexpr int16_t kInvAngle[15] = {-4096, -1638, -910, -630, -482, -390, -315, -256,
                                          -315,  -390,  -482, -630, -910, -1638, -4096};

// ---------------------------------------------------------------- transform (8.6.4.2)
// Entry (k, n) of the 32-point DCT-like matrix transMatrix.  The N-point matrix uses
// rows k * 32 / N.  Magnitudes by angle class: cos(m*pi/64) (k odd), cos(m*pi/32),
// cos(m*pi/16), cos(m*pi/8), cos(pi/4) -- the values of the standard's table.
MIVC_HD int dct_coef(int k, int n) {
  if (k == 0) return 64;
  int t = ((2 * n + 1) * k) & 127;  // angle in units of pi/64, period 2*pi
  int sign = 1;
  if (t > 64) t = 128 - t;          // cos(2pi - a) = cos(a)
  if (t > 32) {                     // cos(pi - a) = -cos(a)
    t = 64 - t;
    sign = -1;
  }
  int mag;
  if (t == 0) mag = 64 * 1;         // unreachable for k > 0 with odd (2n+1)*k multiple of 64 except k = 0
  else if (t & 1) {
    const int v[16] = {90, 90, 88, 85, 82, 78, 73, 67, 61, 54, 46, 38, 31, 22, 13, 4};
    mag = v[(t - 1) >> 1];
  } else if (t & 2) {
    const int v[8] = {90, 87, 80, 70, 57, 43, 25, 9};
    mag = v[((t >> 1) - 1) >> 1];
  } else if (t & 4) {
    const int v[4] = {89, 75, 50, 18};
    mag = v[((t >> 2) - 1) >> 1];
  } else if (t & 8) {
    mag = (t >> 3) == 1 ? 83 : 36;
  } else if (t == 16) {
    mag = 64;
  } else {
    mag = 0;  // t == 32: cos(pi/2)
  }
  return sign * mag;
}

// 4x4 DST-VII (intra 4x4 luma; unused by this encoder's 8x8 minimum, kept for the decoder)
static constexpr int8_t kDst4[4][4] = {{29, 55, 74, 84}, {74, 74, 0, -74}, {84, -29, -74, 55}, {55, -84, 74, -29}};

// ---------------------------------------------------------------- quantisation (8.6.2 / 8.6.3)
static constexpr int kLevelScale[6] = {40, 45, 51, 57, 64, 72};
static constexpr int kQuantScale[6] = {26214, 23302, 20560, 18396, 16384, 14564};  // encoder side

// QpC as a function of qPi for ChromaArrayType == 1 (Table 8-10)
MIVC_HD int chroma_qp_map(int qpi) {
  if (qpi < 30) return qpi;
  if (qpi > 43) return qpi - 6;
  const int t[14] = {29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37, 37};
  return t[qpi - 30];
}

// ---------------------------------------------------------------- deblocking (Table 8-12)
static constexpr uint8_t kTcTable[54] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1,
                                         1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4,
                                         5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24};
static constexpr uint8_t kBetaTable[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  6,  7,
                                           8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 20, 22, 24, 26, 28, 30, 32,
                                           34, 36, 38, 40, 42, 44, 46, 48, 50, 52, 54, 56, 58, 60, 62, 64};

// ---------------------------------------------------------------- scans (6.5.3 - 6.5.5)
// scanIdx 0 diagonal up-right, 1 horizontal, 2 vertical.  Position p of the scan of
// a (1 << log2size)^2 grid: returns x | (y << 8).  4x4 coefficient groups and the
// sub-block grids of 8x8 / 16x16 / 32x32 TUs use the same constructions.
MIVC_HD int scan_pos(int scan_idx, int log2size, int p) {
  const int n = 1 << log2size;
  if (scan_idx == 1) return (p % n) | ((p / n) << 8);
  if (scan_idx == 2) return (p / n) | ((p % n) << 8);
  // diagonal up-right: walk anti-diagonals, bottom-left to top-right
  int i = 0;
  for (int d = 0; d < 2 * n - 1; ++d) {
    for (int y = d; y >= 0; --y) {
      const int x = d - y;
      if (x < n && y < n) {
        if (i == p) return x | (y << 8);
        ++i;
      }
    }
  }
  return 0;
}

// ---------------------------------------------------------------- CABAC context initialisation (9.3.2.2)
// Context index offsets of the syntax elements the encoder's CABAC writer uses:
enum Ctx : int {
  CTX_SAO_MERGE = 0,         // 1
  CTX_SAO_TYPE = 1,          // 1
  CTX_SPLIT_CU = 2,          // 3
  CTX_CU_SKIP = 5,           // 3
  CTX_PRED_MODE = 8,         // 1
  CTX_PART_MODE = 9,         // 4
  CTX_PREV_INTRA = 13,       // 1
  CTX_CHROMA_MODE = 14,      // 1
  CTX_MERGE_FLAG = 15,       // 1
  CTX_MERGE_IDX = 16,        // 1
  CTX_MVD_G0 = 17,           // 1
  CTX_MVD_G1 = 18,           // 1
  CTX_MVP_IDX = 19,          // 1
  CTX_RQT_ROOT_CBF = 20,     // 1
  CTX_SPLIT_TRANSFORM = 21,  // 3
  CTX_CBF_LUMA = 24,         // 2
  CTX_CBF_CHROMA = 26,       // 4
  CTX_LAST_X = 30,           // 18
  CTX_LAST_Y = 48,           // 18
  CTX_CSBF = 66,             // 4
  CTX_SIG = 70,              // 42 (27 luma + 15 chroma)
  CTX_GT1 = 112,             // 24 (16 luma + 8 chroma)
  CTX_GT2 = 136,             // 6 (4 luma + 2 chroma)
  CTX_REF_IDX = 142,         // 2
  CTX_CU_QP_DELTA = 144,     // 2
  CTX_INTER_PRED = 146,      // 5 (inter_pred_idc: ctxInc = CtDepth for the first bin, 4 for the second)
  kNumCtx = 151,
};

// initValues of these contexts for the three initTypes come from the full spec table of the
// decoder (csrc/host/hevc_ctx_tables.h) through kWriterCtxToSpec (hevc_cabac.h)

// ---------------------------------------------------------------- CABAC engine tables (9.3.4.3.2)
static constexpr uint8_t kRangeLps[64][4] = {
    {128, 176, 208, 240}, {128, 167, 197, 227}, {128, 158, 187, 216}, {123, 150, 178, 205}, {116, 142, 169, 195},
    {111, 135, 160, 185}, {105, 128, 152, 175}, {100, 122, 144, 166}, {95, 116, 137, 158},  {90, 110, 130, 150},
    {85, 104, 123, 142},  {81, 99, 117, 135},   {77, 94, 111, 128},   {73, 89, 105, 122},   {69, 85, 100, 116},
    {66, 80, 95, 110},    {62, 76, 90, 104},    {59, 72, 86, 99},     {56, 69, 81, 94},     {53, 65, 77, 89},
    {51, 62, 73, 85},     {48, 59, 69, 80},     {46, 56, 66, 76},     {43, 53, 63, 72},     {41, 50, 59, 69},
    {39, 48, 56, 65},     {37, 45, 54, 62},     {35, 43, 51, 59},     {33, 41, 48, 56},     {32, 39, 46, 53},
    {30, 37, 43, 50},     {29, 35, 41, 48},     {27, 33, 39, 45},     {26, 31, 37, 43},     {24, 30, 35, 41},
    {23, 28, 33, 39},     {22, 27, 32, 37},     {21, 26, 30, 35},     {20, 24, 29, 33},     {19, 23, 27, 31},
    {18, 22, 26, 30},     {17, 21, 25, 28},     {16, 20, 23, 27},     {15, 19, 22, 25},     {14, 18, 21, 24},
    {14, 17, 20, 23},     {13, 16, 19, 22},     {12, 15, 18, 21},     {12, 14, 17, 20},     {11, 14, 16, 19},
    {11, 13, 15, 18},     {10, 12, 15, 17},     {10, 12, 14, 16},     {9, 11, 13, 15},      {9, 11, 12, 14},
    {8, 10, 12, 14},      {8, 9, 11, 13},       {7, 9, 11, 12},       {7, 9, 10, 12},       {7, 8, 10, 11},
    {6, 8, 9, 11},        {6, 7, 9, 10},        {6, 7, 8, 9},         {2, 2, 2, 2}};
static constexpr uint8_t kTransIdxLps[64] = {0,  0,  1,  2,  2,  4,  4,  5,  6,  7,  8,  9,  9,  11, 11, 12,
                                             13, 13, 15, 15, 16, 16, 18, 18, 19, 19, 21, 21, 22, 22, 23, 24,
                                             24, 25, 26, 26, 27, 27, 28, 29, 29, 30, 30, 30, 31, 32, 32, 33,
                                             33, 33, 34, 34, 35, 35, 35, 36, 36, 36, 37, 37, 37, 38, 38, 63};

// ---------------------------------------------------------------- decision records (encoder <-> writer)
// One CtuInfo per 32x32 CTB and one CuInfo per 8x8 granule (z-order inside the CTB);
// a coding unit's fields are replicated into every granule it covers.  Quantised
// levels live in coefficient planes shaped like the picture: the level (u, v) of the
// transform block at (x0, y0) is stored at [y0 + v][x0 + u] (TU = CU for luma,
// half size for 4:2:0 chroma).
// Per-CTB QP (cu_qp_delta, one quantization group per CTB = x265 --qg-size 32): `qp` is
// the QpY the CTB is quantised with.  CUs of the CTB before the first one with a coded
// residual (z-order granule < qp_first) carry QpY = qp_pred, the prediction from the
// previous quantization group (8.6.1); a CTB without any coded residual has qp == qp_pred
// after the encoder's fix-up pass (hevc_qp_fixup), and qp_first = 16.
struct alignas(16) CtuInfo {
  uint8_t split;        // bit0: 32x32 -> 16x16; bit (1 + q): 16x16 quadrant q -> 8x8
  int8_t qp;            // QpY of the CTB
  uint8_t sao_type[2];  // [luma, chroma]: 0 off, 1 band offset, 2 edge offset
  uint8_t sao_class[2]; // edge-offset class (0 hor, 1 ver, 2 135deg, 3 45deg)
  uint8_t sao_band[3];  // band position per component
  uint8_t pad0;
  int8_t sao_off[3][4]; // offsets per component (edge: categories 1..4; band: 4 bands)
  int8_t qp_pred;       // qPY_PRED of the CTB's quantization group
  uint8_t qp_first;     // z-order granule of the first CU with a coded residual (16: none)
  uint8_t pad1[6];
};
static_assert(sizeof(CtuInfo) == 32, "CtuInfo is 32 bytes");

enum CuPred : uint8_t { CU_INTRA = 0, CU_INTER = 1 };

// inter prediction direction of a CU (inter_pred_idc + 1): bit 0 list 0, bit 1 list 1
enum CuDir : uint8_t { DIR_L0 = 1, DIR_L1 = 2, DIR_BI = 3 };

struct alignas(8) CuInfo {
  uint8_t pred;   // CuPred
  uint8_t mode;   // intra luma mode 0..34 (intra)
  uint8_t cbf;    // informational: bit0 Y, bit1 Cb, bit2 Cr (the writer recomputes it)
  uint8_t flags;  // bits 1-2: log2 CU size - 3; bit 3: intra PART_NxN; bit 4: inter TU split once
                  // (cbf then describes the quarter TU covering this granule)
  int16_t mv[2];  // quarter-sample L0 motion vector (inter)
  int16_t mv1[2]; // quarter-sample L1 motion vector (inter, B slices)
  uint8_t dir;    // CuDir of an inter CU (0 is read as DIR_L0: P-slice records)
  uint8_t pad[3]; // pad[0] / pad[1]: refIdx L0 / L1 of an inter CU (x265 --ref); pad[2] unused
};
static_assert(sizeof(CuInfo) == 16, "CuInfo is 16 bytes");
constexpr int kCuInfoBytes = 16;

MIVC_HD int cu_dir(const CuInfo& c) { return c.dir ? c.dir : DIR_L0; }

// z-order index of 8x8 granule (gx, gy) inside a 32x32 CTB
MIVC_HD int zorder8(int gx, int gy) {
  return (gx & 1) | ((gy & 1) << 1) | ((gx & 2) << 1) | ((gy & 2) << 2);
}

}  // namespace hevc
}  // namespace mivc
