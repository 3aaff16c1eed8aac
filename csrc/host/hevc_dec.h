// General HEVC (H.265) Main / Main 10 decoder: bitstream parse (host) + CPU
// reconstruction (the bit-exact oracle) + GPU hand-off records (hevc_decode.hip).
//
// Reference parity: the reference worker decodes whatever codec its piece holds with
// `ffmpeg -i <idx>.mp4` (client.go:115) and splits any input with the stream-copying
// segment muxer (server.go:199-201); the north star lists "H.264/HEVC decode" as native
// kernels.  This decoder covers the Main / Main 10 profiles of ITU-T H.265 (4:2:0, 8..10
// bits): VPS/SPS/PPS with any ids, CTB 16/32/64, every PartMode incl. AMP, intra NxN,
// the full transform tree (4x4..32x32, DST, transform_skip, cu_transquant_bypass, PCM),
// scaling lists (SPS/PPS/default, predicted), cu_qp_delta, P and B slices (merge with the
// temporal candidate and combined bi-predictive candidates, AMVP with scaling, TMVP,
// explicit weighted prediction), long-term and short-term RPS (incl. inter-RPS
// prediction, slice-level sets), list modification, multiple slices and dependent slice
// segments, tiles, WPP, deblocking (with slice overrides, across-slice/tile controls)
// and SAO.  RASL pictures of a CRA that starts the stream are skipped (as ffmpeg does).
//
// Written from the standard text (clauses 6-9), independently of the encoder-side writer
// (hevc_writer.cc); only the constant tables are shared.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "hevc_codec.h"

namespace mivc {
namespace hevc {

// ---------------------------------------------------------------- GPU hand-off records
// Everything the gfx950 reconstruction needs is resolved on the host: motion vectors
// (merge / AMVP / TMVP done), reference pictures as entries of a per-picture table,
// weights, QPs, deblocking boundary strengths, SAO parameters.  The GPU does the sample
// work: dequantisation + inverse transforms, motion compensation, intra prediction in
// CTB wavefront order, deblocking, SAO (csrc/kernels/hevc_decode.hip).

// motion / flags / QpY of a luma block (DecPicture::mvf: 8x8 blocks, mvf_sub: 4x4 blocks)
struct DecMv4 {
  int16_t mv[2][2];   // quarter-sample L0 / L1 vectors
  uint8_t ref[2];     // index into DecPicture::refs, 0xFF = list unused
  uint8_t flags;      // DM_* bits
  int8_t qp;          // QpY of the coding unit
};
static_assert(sizeof(DecMv4) == 12, "DecMv4 is 12 bytes");
enum : uint8_t { DM_INTRA = 1, DM_NOFILTER = 2, DM_INTER = 4, DM_SPLIT = 8 };

// deblocking edge strengths per 4x4 luma block: bits 0-1 bS of its left edge, bits 2-3 bS
// of its top edge (0 = not filtered: not an edge, picture / slice / tile restriction or a
// disabled slice)
using DecBs = uint8_t;

// one coded transform block: coefficients (n x n int16, raster) at DecPicture::coefs[coef]
struct DecTu {
  uint16_t x, y;      // position in component samples
  uint8_t log2;       // 2..5
  uint8_t cidx;       // 0 Y, 1 Cb, 2 Cr
  uint8_t qp;         // Qp'Y / Qp'Cb / Qp'Cr (QP + QpBdOffset)
  uint8_t flags;      // DT_* bits
  uint32_t coef;
};
static_assert(sizeof(DecTu) == 12, "DecTu is 12 bytes");
enum : uint8_t { DT_DST = 1, DT_TSKIP = 2, DT_BYPASS = 4, DT_INTRA = 8, DT_SCALING = 16, DT_PCM = 32 };

// intra prediction of one transform block, in decoding order per CTB
struct DecIntraOp {
  uint16_t x, y;      // component samples
  uint8_t log2;       // 2..5
  uint8_t cidx;
  uint8_t mode;       // 0..34, 0xFF = PCM (no prediction: the "residual" holds the samples)
  uint8_t flags;      // unused (0)
  uint32_t tu;        // index into tus of its residual, 0xFFFFFFFF = none
};
static_assert(sizeof(DecIntraOp) == 12, "DecIntraOp is 12 bytes");

// reference entry: one (slice, list, ref_idx) with its weights
struct DecRefEntry {
  int8_t pic;          // index into DecPicture::ref_ids
  uint8_t log2wd_y;    // luma_log2_weight_denom (explicit weights)
  uint8_t log2wd_c;    // ChromaLog2WeightDenom
  uint8_t weighted;    // 1: explicit weighted prediction
  int16_t w[3], o[3];  // weights and offsets (offsets already << (BitDepth - 8))
};
static_assert(sizeof(DecRefEntry) == 16, "DecRefEntry is 16 bytes");

struct DecCtb {
  uint16_t slice;      // index into DecPicture::slices
  uint16_t tile;       // TileId
  uint32_t ts;         // CtbAddrRsToTs (decoding order)
};
static_assert(sizeof(DecCtb) == 8, "DecCtb is 8 bytes");

struct DecSao {
  uint8_t type[3];     // 0 off, 1 band, 2 edge
  uint8_t band[3];     // sao_band_position
  uint8_t eo[3];       // edge class
  uint8_t pad;
  int8_t off[3][4];    // SaoOffsetVal[1..4]
  uint8_t pad2[2];
};
static_assert(sizeof(DecSao) == 24, "DecSao is 24 bytes");

struct DecSlice {
  int8_t beta_off, tc_off;  // slice_beta_offset_div2 * 2, slice_tc_offset_div2 * 2
  uint8_t deblock_off;      // slice_deblocking_filter_disabled_flag
  uint8_t lf_across;        // slice_loop_filter_across_slices_enabled_flag
  uint32_t addr_rs;         // SliceAddrRs (first CTB of the independent slice)
};
static_assert(sizeof(DecSlice) == 8, "DecSlice is 8 bytes");

// one decoded picture (decoding order)
struct DecPicture {
  int decode_idx = 0;       // position in decoding order within this decoder
  int poc = 0;
  int cvs = 0;              // coded video sequence ordinal (output order = (cvs, poc))
  int output = 1;           // PicOutputFlag
  int irap = 0, idr = 0, nal_type = 0, slice_type = 2, slice_qp = 0;
  int W = 0, H = 0;         // coded size (pic_width / height_in_luma_samples)
  int width = 0, height = 0, crop_x = 0, crop_y = 0;  // conformance window (luma samples)
  int bit_depth = 8, bit_depth_c = 8;
  int log2_ctb = 4, wctb = 0, hctb = 0;
  // picture-level filter / prediction parameters
  int constrained_intra = 0, strong_intra = 0, lf_across_tiles = 1, cb_qp_off = 0, cr_qp_off = 0;
  int deblock_any = 0, sao_any = 0;
  // GPU records (filled when DecodeOptions::gpu_records)
  std::vector<int> ref_ids;         // decode_idx of every picture referenced by refs
  std::vector<DecRefEntry> refs;
  std::vector<DecMv4> mvf;          // [H/8][W/8] per 8x8 block; DM_SPLIT: mv bytes 0-3 = entry of
  std::vector<DecMv4> mvf_sub;      // 4 records (raster 4x4 blocks) per split 8x8 block
  std::vector<DecBs> bs;            // [H/4][W/4]
  std::vector<DecTu> tus;
  std::vector<int16_t> coefs;
  std::vector<DecIntraOp> ops;
  std::vector<uint32_t> ops_off;    // [wctb * hctb + 1]: ops of CTB (raster) r are [ops_off[r], ops_off[r+1])
  std::vector<DecCtb> ctbs;         // [wctb * hctb] raster
  std::vector<DecSao> sao;          // [wctb * hctb] raster
  std::vector<DecSlice> slices;
  std::vector<uint8_t> scaling;     // ScalingFactor (kScalingBytes) when scaling lists are on, else empty
  // CPU reconstruction (DecodeOptions::recon): coded-size planes
  std::vector<uint16_t> y, u, v;
  // encoder decision records (32x32-CTB streams only, DecodeOptions::enc_records)
  std::vector<CtuInfo> ctu;
  std::vector<CuInfo> cu;
  std::vector<int16_t> coef_y, coef_cb, coef_cr;
};

// ScalingFactor layout: sizeId 0..3, matrixId 0..5, raster (x + y * n): 6 x (16 + 64 + 256 + 1024)
constexpr int kScalingOff[4] = {0, 96, 96 + 384, 96 + 384 + 1536};
constexpr int kScalingBytes = 96 + 384 + 1536 + 6144;

struct DecodeOptions {
  bool recon = true;         // CPU reconstruction (oracle / fallback)
  bool gpu_records = false;  // fill the GPU hand-off records
  bool skip_filters = false; // CPU recon: no deblocking / SAO (tests)
  bool enc_records = false;  // export the encoder's decision records (32x32 CTBs)
};

class HevcStreamDecoder {
 public:
  explicit HevcStreamDecoder(const DecodeOptions& o);
  ~HevcStreamDecoder();
  // decode a whole Annex-B buffer; pictures are appended in decoding order
  void decode(const uint8_t* data, size_t n);
  std::vector<DecPicture>& pictures() { return pics_; }
  // display order of pictures(): indices sorted by (cvs, poc), PicOutputFlag 0 excluded
  std::vector<int> output_order() const;
  struct Impl;

 private:
  std::unique_ptr<Impl> impl_;
  std::vector<DecPicture> pics_;
};

// stream-level facts for probing / splitting (first SPS / VUI)
struct HevcStreamInfo {
  int width = 0, height = 0, bit_depth = 8;
  double fps = 0.0;
  int pictures = 0, irap = 0;
};
HevcStreamInfo hevc_stream_info(const uint8_t* p, size_t n);

// split an Annex-B HEVC stream into pieces starting at IRAP access units (IDR / CRA / BLA),
// with the VPS / SPS / PPS re-emitted at the front of every piece; a new piece starts only
// once >= min_frames pictures are in the current one
std::vector<std::vector<uint8_t>> hevc_split_pieces(const uint8_t* p, size_t n, int min_frames);

}  // namespace hevc
}  // namespace mivc
