// Per-macroblock decision record: the contract between the encoder front end
// (gfx950 HIP kernels or the CPU reference encoder) and the entropy coders
// (host C++ CAVLC writer, GPU CAVLC kernels).
//
// One MbHeader (64 B) + kCoefPerMb int16 coefficients per 16x16 macroblock.
// Coefficients are quantised levels in *scan order* (zig-zag), exactly what the
// residual_block() syntax carries; blocks are in luma4x4BlkIdx order.
#pragma once
#include <cstdint>

#include "h264_tables.h"

namespace mivc {
namespace h264 {

enum SliceType { SLICE_P = 0, SLICE_B = 1, SLICE_I = 2 };

enum MbKind : uint8_t {
  MBK_I4x4 = 0,
  MBK_I16x16 = 1,
  MBK_P16x16 = 2,
  MBK_PSKIP = 3,  // hint only: the writer re-derives skip from cbp == 0 && mv == mvp_skip
  MBK_IPCM = 4,
  MBK_P16x8 = 5,
  MBK_P8x16 = 6,
  MBK_P8x8 = 7,   // four 8x8 sub-macroblocks, each 8x8 (sub_mb_type 0)
  MBK_I8x8 = 8,   // I_NxN with transform_size_8x8_flag (High profile)
  // B slices: the prediction list(s) of every partition are given by ref[l][q] >= 0
  MBK_B16x16 = 9,
  MBK_B16x8 = 10,
  MBK_B8x16 = 11,
  MBK_B8x8 = 12,     // sub_mb_type 8x8 per quadrant, or B_Direct_8x8 where sub_direct bit q
  MBK_BDIRECT = 13,  // B_Direct_16x16 (B_Skip when cbp == 0): motion from the direct derivation
};

MIVC_HD bool mbk_is_intra(int k) { return k == MBK_I4x4 || k == MBK_I16x16 || k == MBK_IPCM || k == MBK_I8x8; }
MIVC_HD bool mbk_is_b(int k) { return k >= MBK_B16x16 && k <= MBK_BDIRECT; }

// Coefficient layout (int16 each)
enum : int {
  COEF_LUMA = 0,          // 16 blocks x 16 (scan order; for I16x16 index 0 unused); with the 8x8
                          // transform: 4 blocks x 64 (8x8 zig-zag), block b8 at b8 * 64
  COEF_LUMA_DC = 256,     // 16 (I16x16 DC, scan order)
  COEF_CHROMA_DC = 272,   // 2 x 4 (Cb, Cr; raster c00,c10,c01,c11)
  COEF_CHROMA_AC = 280,   // 2 x 4 blocks x 16 (index 0 unused)
  kCoefPerMb = 408,
};

enum : uint8_t {
  MBF_SKIP = 1,     // encoder proposes P_Skip / B_Skip
  MBF_T8x8 = 2,     // transform_size_8x8_flag
  MBF_SUB4 = 4,     // decoder records: motion below 8x8; the per-4x4 vectors are a side-pool
                    // entry whose index is in i4_modes[0..3] (uint32; inter MBs only)
};

// side-pool entry (int16 units): mv[list][raster 4x4][2], then ref_idx int8[list][raster 4x4]
enum : int { kSubEntry = 80 };

// 64 bytes; the first 48 (everything but the intra modes) are what the deblocking
// filter reads.
struct alignas(16) MbHeader {
  uint8_t kind;         // MbKind
  uint8_t cbp;          // informational; writers recompute it from the coefficients
  int8_t qp;            // QP_Y this MB was quantised with
  uint8_t i16_mode;     // Intra16x16PredMode: 0 V, 1 H, 2 DC, 3 Plane
  uint8_t chroma_mode;  // intra_chroma_pred_mode: 0 DC, 1 H, 2 V, 3 Plane
  uint8_t flags;        // MBF_*
  uint8_t sub_direct;   // MBK_B8x8: bit q set = quadrant q is B_Direct_8x8
  uint8_t pad0;
  int8_t ref[2][4];     // ref_idx per 8x8 quadrant (raster 0..3), list 0 / 1; -1 = list unused
  int16_t mv[2][4][2];  // quarter-pel MV per quadrant and list; all equal for 16x16
  uint8_t i4_modes[16]; // Intra4x4PredMode per luma4x4BlkIdx (I8x8: the 8x8 mode in all four)
};
static_assert(sizeof(MbHeader) == 64, "MbHeader must stay 64 bytes (GPU kernels write it)");

}  // namespace h264
}  // namespace mivc
