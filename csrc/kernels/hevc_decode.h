// Launch parameters of the gfx950 HEVC decode reconstruction (hevc_decode.hip), shared
// with the pybind11 shim (bindings_hip.cc, plain C++).  Record layouts are those of
// csrc/host/hevc_dec.h (DecMv4 12 B, DecTu 12 B, DecIntraOp 12 B, DecRefEntry 16 B,
// DecCtb 8 B, DecSao 24 B, DecSlice 8 B); per-slot arrays are concatenated over the B
// slots of one picture step with per-slot bases.
#pragma once
#include <cstdint>

namespace mivc {
namespace gpu {

struct HevcDecParams {
  int B, W, H, D;              // slots, coded size, DPB buffers per slot
  int bd, bdc, log2_ctb, wctb, hctb;
  uint16_t* dpb[3];            // [B, D, plane]
  int16_t* res[3];             // residual planes [B, plane]
  uint16_t* tmp[3];            // deblocked copy (SAO input) [B, plane]
  const int8_t* cur;           // [B] DPB buffer of the picture being decoded
  const int8_t* reftab;        // [B, 16] DPB buffer of every DecPicture::ref_ids entry
  const int8_t* run;           // [B] 1 = the slot decodes a picture this step
  const int32_t* meta;         // [B, 24] picture meta (hevc_parse layout)
  const uint8_t* mvf;          // [B, H/8, W/8, 12] per 8x8 block (DM_SPLIT: index into mvf_sub)
  const uint8_t* mvf_sub;      // [NS * 4, 12] per-4x4 records of split 8x8 blocks
  const uint8_t* bs;           // [B, h4, w4]
  const uint8_t* ctbs;         // [B, nctb, 8]
  const uint8_t* sao;          // [B, nctb, 24]
  const uint8_t* tus;          // [NT, 12]
  const int32_t* tu_base;      // [B + 1]
  const int16_t* coefs;
  const int64_t* coef_base;    // [B]
  const uint8_t* ops;          // [NO, 12]
  const int32_t* op_base;      // [B]
  const uint32_t* ctb_ops;     // [B, nctb + 1]
  const uint8_t* refs;         // [NR, 16]
  const int32_t* ref_base;     // [B]
  const uint8_t* slices;       // [NS, 8]
  const int32_t* slice_base;   // [B]
  const uint8_t* scaling;      // [B, 8160] ScalingFactor, or null (flat)
  int max_tus;                 // most TUs of any slot this step (residual grid)
  int* err;
  // stage 6 (emit): the step's pictures to their display positions of the output
  void* out[3];                // [B, Fo, out_h, out_w] (chroma halved) uint8 (out_u8) or int16
  int out_u8, Fo, out_w, out_h, crop_x, crop_y;
  const int16_t* disp;         // [B] output position of this step's picture, -1 = not output
};

// meta columns (hevc_parse "meta")
enum HevcMeta : int {
  HM_DECODE_IDX = 0, HM_POC, HM_CVS, HM_OUTPUT, HM_IRAP, HM_IDR, HM_SLICE_TYPE, HM_SLICE_QP, HM_W, HM_H, HM_WIDTH,
  HM_HEIGHT, HM_CROP_X, HM_CROP_Y, HM_BD, HM_BDC, HM_LOG2_CTB, HM_CONSTRAINED_INTRA, HM_STRONG_INTRA,
  HM_LF_ACROSS_TILES, HM_CB_QP_OFF, HM_CR_QP_OFF, HM_DEBLOCK_ANY, HM_SAO_ANY, HM_COLS = 24
};

}  // namespace gpu
}  // namespace mivc
