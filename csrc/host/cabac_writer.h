// CABAC slice writer (H.264 clauses 7.3.4, 7.3.5, 9.3): the host instance of the shared
// macroblock-layer coder in csrc/common/h264_cabac.h (the gfx950 kernel runs the same
// code), framed as a slice NAL unit.
#pragma once
#include <cstdint>
#include <vector>

#include "../common/h264_mb.h"
#include "cavlc_writer.h"
#include "h264_syntax.h"

namespace mivc {
namespace h264 {

// Encode MBs [first_mb, first_mb + num_mbs) of a picture (mbs / coef cover the whole
// picture) into a complete Annex-B slice NAL unit.  Requires pps.entropy_coding_mode and
// sh.cabac_init_idc == 0.
std::vector<uint8_t> write_slice_nal_cabac(const SPS& sps, const PPS& pps, const SliceHeader& sh, const MbHeader* mbs,
                                           const int16_t* coef, int num_mbs, SliceStats* stats = nullptr);

// slice_data() bytes only (after a byte-aligned slice header)
std::vector<uint8_t> cabac_slice_data(const SPS& sps, const PPS& pps, const SliceHeader& sh, const MbHeader* mbs,
                                      const int16_t* coef, int num_mbs, SliceStats* stats = nullptr);

// Slice data through the symbol path (per-MB binarisation, then arithmetic coding): the
// decomposition the GPU uses.  Returns the bytes and the symbol count.
std::vector<uint8_t> cabac_slice_data_symbols(const SPS& sps, const PPS& pps, const SliceHeader& sh, const MbHeader* mbs,
                                              const int16_t* coef, int num_mbs, int* nsyms);

}  // namespace h264
}  // namespace mivc
