// CAVLC slice writer (H.264 clauses 7.3.4, 7.3.5, 9.2): turns the per-MB decision
// records produced by the encoder front end into slice_data() bits.
#pragma once
#include <cstdint>
#include <vector>

#include "../common/h264_mb.h"
#include "bitstream.h"
#include "h264_syntax.h"

namespace mivc {
namespace h264 {

struct SliceStats {
  int bits = 0;
  int skipped = 0;
  int intra = 0;
  int coded_inter = 0;
};

// Write one residual_block_cavlc() (clause 7.3.5.3.2).  coef is in scan order,
// start/end inclusive indices, max_num_coeff in {4, 15, 16}.  nc = -1 selects
// the chroma-DC coeff_token table.  Returns TotalCoeff.
int cavlc_write_block(BitWriter& bw, const int16_t* coef, int start, int end, int max_num_coeff, int nc);

// Canonical coded_block_pattern derived from the coefficients of one MB.
int derive_cbp(const MbHeader& mb, const int16_t* coef);

// Encode the macroblocks [first_mb, first_mb + num_mbs) of a picture into a
// complete NAL unit (Annex-B start code + header + slice header + slice data).
// mbs/coef cover the whole picture (width_mbs * height_mbs entries).
std::vector<uint8_t> write_slice_nal(const SPS& sps, const PPS& pps, const SliceHeader& sh, const MbHeader* mbs,
                                     const int16_t* coef, int num_mbs, SliceStats* stats = nullptr);

// Parameter-set NAL units (SPS + PPS), Annex-B framed.
std::vector<uint8_t> write_parameter_sets(const SPS& sps, const PPS& pps);

}  // namespace h264
}  // namespace mivc
