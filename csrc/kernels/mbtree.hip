// Macroblock-tree rate control (SURVEY.md K-C3 "MB-tree propagation"; x264 --mbtree, on
// in the libx264 defaults the reference's "264" preset runs with, server.go:69-70).
//
// Works on the lookahead's lowres blocks (one 8x8 lowres block per 16x16 MB) of B
// closed-GOP segments at once.  Going backwards through each segment, a block of frame t
// hands the share of its information that frame t-1 predicted,
//     amount = (intra + propagate_in) * (intra - min(inter, intra)) / intra,
// to the blocks of frame t-1 its lowres vector points at, split by overlap area (x264
// macroblock_tree_propagate).  The QP offset of a block is then
//     -strength * log2((intra + propagate_in) / intra),   strength = 5 (1 - qcomp),
// so blocks that later frames reference get more bits.
//
//   mbtree_propagate   one launch per frame t = F-1 .. 1 (frame t-1 accumulates atomically)
//   mbtree_offsets     all frames: float QP offsets [B, F, nblk]
//
// Determinism: the propagated amounts accumulate as 64-bit fixed point (kPropOne units)
// with integer atomics, which are order-independent, so the offsets -- and the rounded
// per-MB QPs and the bitstream -- are identical from run to run (a float atomicAdd sum
// depends on the order the waves arrive in).
#include "kcommon.h"

namespace mivc {
namespace gpu {

constexpr float kPropOne = 4096.f;  // fixed-point scale of the propagate accumulators

__global__ __launch_bounds__(256) void mbtree_propagate(int B, int F, int t, int lbw, int lbh,
                                                        const int* __restrict__ blk_cost, const int* __restrict__ blk_mv,
                                                        unsigned long long* __restrict__ prop) {
  const int nblk = lbw * lbh;
  const long long idx = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= static_cast<long long>(B) * nblk) return;
  const int b = static_cast<int>(idx / nblk), i = static_cast<int>(idx - static_cast<long long>(b) * nblk);
  const long long n = static_cast<long long>(b) * F + t;
  const float intra = static_cast<float>(blk_cost[(n * 2) * nblk + i]);
  const float inter = fminf(static_cast<float>(blk_cost[(n * 2 + 1) * nblk + i]), intra);
  const float pin = static_cast<float>(prop[n * nblk + i]) * (1.f / kPropOne);
  if (intra <= 0.f || inter >= intra) return;
  const float amount = (pin + intra) * (intra - inter) / intra;
  const int mv = blk_mv[n * nblk + i];
  const int mvx = static_cast<int16_t>(mv & 0xFFFF), mvy = mv >> 16;
  const int bx = i % lbw, by = i / lbw;
  const int x = bx * 8 + mvx, y = by * 8 + mvy;  // lowres position of the reference area
  const int x0 = x >> 3, y0 = y >> 3, fx = x & 7, fy = y & 7;
  unsigned long long* dst = prop + (n - 1) * nblk;
  const int wx[2] = {8 - fx, fx}, wy[2] = {8 - fy, fy};
#pragma unroll
  for (int dy = 0; dy < 2; ++dy)
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      const int cx = x0 + dx, cy = y0 + dy, area = wx[dx] * wy[dy];
      if (area > 0 && cx >= 0 && cx < lbw && cy >= 0 && cy < lbh)
        atomicAdd(dst + cy * lbw + cx,
                  static_cast<unsigned long long>(amount * (area * (kPropOne / 64.f)) + 0.5f));
    }
}

__global__ __launch_bounds__(256) void mbtree_offsets(long long total, const int* __restrict__ blk_cost,
                                                      const unsigned long long* __restrict__ prop, int nblk, float strength,
                                                      float* __restrict__ out) {
  const long long idx = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const long long n = idx / nblk, i = idx - n * nblk;
  const float intra = fmaxf(static_cast<float>(blk_cost[(n * 2) * nblk + i]), 1.f);
  out[idx] = -strength * log2f((intra + static_cast<float>(prop[idx]) * (1.f / kPropOne)) / intra);
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

// blk_cost [B*F, 2, lbh, lbw] int32, blk_mv [B*F, lbh, lbw] (lookahead outputs); prop:
// [B*F, lbh, lbw] uint64 fixed-point scratch (zeroed here); out: [B*F, lbh, lbw] float QP offsets.
extern "C" void mivc_launch_mbtree(int B, int F, int lbw, int lbh, const int* blk_cost, const int* blk_mv, void* prop_,
                                   float strength, float* out, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  unsigned long long* prop = static_cast<unsigned long long*>(prop_);
  const int nblk = lbw * lbh;
  const long long total = static_cast<long long>(B) * F * nblk;
  (void)hipMemsetAsync(prop, 0, sizeof(unsigned long long) * total, s);
  const unsigned g = static_cast<unsigned>((static_cast<long long>(B) * nblk + 255) / 256);
  for (int t = F - 1; t >= 1; --t)
    hipLaunchKernelGGL(mbtree_propagate, dim3(g), dim3(256), 0, s, B, F, t, lbw, lbh, blk_cost, blk_mv, prop);
  hipLaunchKernelGGL(mbtree_offsets, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256), 0, s, total,
                     blk_cost, prop, nblk, strength, out);
}
