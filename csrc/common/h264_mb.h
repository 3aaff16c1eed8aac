// Per-macroblock decision record: the contract between the encoder front end
// (gfx950 HIP kernels or the CPU reference encoder) and the entropy coders
// (host C++ CAVLC writer, GPU CAVLC kernels).
//
// One MbHeader (48 B) + kCoefPerMb int16 coefficients per 16x16 macroblock.
// Coefficients are quantised levels in *scan order* (zig-zag), exactly what the
// residual_block() syntax carries; blocks are in luma4x4BlkIdx order.
#pragma once
#include <cstdint>

#include "h264_tables.h"

namespace mivc {
namespace h264 {

enum MbKind : uint8_t {
  MBK_I4x4 = 0,
  MBK_I16x16 = 1,
  MBK_P16x16 = 2,
  MBK_PSKIP = 3,  // hint only: the writer re-derives skip from cbp == 0 && mv == mvp_skip
  MBK_IPCM = 4,
  MBK_P16x8 = 5,
  MBK_P8x16 = 6,
  MBK_P8x8 = 7,   // four 8x8 sub-macroblocks, each 8x8 (sub_mb_type 0), ref 0
};

MIVC_HD bool mbk_is_intra(int k) { return k == MBK_I4x4 || k == MBK_I16x16 || k == MBK_IPCM; }

// Coefficient layout (int16 each)
enum : int {
  COEF_LUMA = 0,          // 16 blocks x 16 (scan order; for I16x16 index 0 unused)
  COEF_LUMA_DC = 256,     // 16 (I16x16 DC, scan order)
  COEF_CHROMA_DC = 272,   // 2 x 4 (Cb, Cr; raster c00,c10,c01,c11)
  COEF_CHROMA_AC = 280,   // 2 x 4 blocks x 16 (index 0 unused)
  kCoefPerMb = 408,
};

struct alignas(16) MbHeader {
  uint8_t kind;         // MbKind
  uint8_t cbp;          // informational; writers recompute it from the coefficients
  int8_t qp;            // QP_Y this MB was quantised with
  uint8_t i16_mode;     // Intra16x16PredMode: 0 V, 1 H, 2 DC, 3 Plane
  uint8_t chroma_mode;  // intra_chroma_pred_mode: 0 DC, 1 H, 2 V, 3 Plane
  uint8_t flags;        // bit0: encoder proposes P_Skip
  uint8_t pad0[2];
  int16_t mv[4][2];     // quarter-pel L0 MV per 8x8 quadrant (raster 0..3); all equal for 16x16
  uint8_t i4_modes[16]; // Intra4x4PredMode per luma4x4BlkIdx
  uint8_t pcm_pad[8];
};
static_assert(sizeof(MbHeader) == 48, "MbHeader must stay 48 bytes (GPU kernels write it)");

}  // namespace h264
}  // namespace mivc
