// Lookahead complexity analysis on half-resolution luma (the quantity x264's
// CRF rate control is driven by: per-frame sum of 8x8 lowres SATD costs).
// CPU implementation used by the cpu_ref backend and as the numerics oracle
// of the HIP lookahead kernel (csrc/kernels/lookahead.hip).
#pragma once
#include <cstddef>
#include <cstdint>

namespace mivc {

// frames: nframes tightly packed I420 frames of width x height.
// intra[f]: sum over 8x8 lowres blocks of the intra (DC/H/V) SATD cost.
// inter[f]: sum over blocks of min(intra, best inter SATD vs frame f-1) (intra for f == 0).
void lowres_frame_costs(const uint8_t* frames, int width, int height, int nframes, float* intra, float* inter);

}  // namespace mivc
