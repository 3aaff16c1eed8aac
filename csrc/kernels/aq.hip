// Adaptive quantisation for the H.264 encoder (SURVEY.md K-C11, x264 --aq-mode 1, the
// libx264 default of the reference's "264" preset, server.go:69-70).
//
//   h264_aq_offsets   per-MB QP offsets from the AC energy of the source MB:
//                     energy = var(Y 16x16) + var(Cb 8x8) + var(Cr 8x8) (sum of squares minus
//                     squared sum / n, x264 ac_energy_var), offset = round(strength * 1.0397 *
//                     (log2(energy) - 14.427)), the x264 formula for 8-bit video.
//                     (+ the MB-tree offset of the MB when given, mbtree.hip)
//   h264_qp_flags     per MB: does it carry mb_qp_delta (coded residual, or Intra16x16)?
//                     (luma from the encoder's non-zero flags, which hold for every MB kind
//                     but Intra16x16, whose flag is set regardless)
//   h264_qp_fixup     an MB without mb_qp_delta inherits QP_pred (the QP of the previous MB
//                     in decoding order, the slice QP for the first): clause 7.4.5.  Its
//                     decision record gets that QP so that deblocking (which reads QP_Y of
//                     every MB) matches a decoder.  Per slot: segmented scan over raster order.
#include <cmath>

#include "kcommon.h"

namespace mivc {
namespace gpu {

using h264::MbHeader;

// 16 lanes per MB (4 MBs per wave, 16 per 256-thread workgroup): lane l of a group sums
// luma row l (4 dwords) and, for l < 8 Cb row l / for l >= 8 Cr row l - 8 (2 dwords); the
// group reductions are DPP row sums.  A workgroup walks kAqSpan groups of 16 MBs (one launch
// of ~nmb / 16 tiny workgroups per slot was dispatch-bound: 0.56 TB/s).
constexpr int kAqSpan = 8;

__global__ __launch_bounds__(256) void h264_aq_offsets(Geom g, const uint8_t* __restrict__ sy,
                                                       const uint8_t* __restrict__ su, const uint8_t* __restrict__ sv,
                                                       float strength, const float* __restrict__ extra,
                                                       long long extra_stride, int8_t* __restrict__ out,
                                                       const SlotRoute* rt) {
  const int l = lane_id() & 15;
  const int nmb = g.nmb();
  const int slot = blockIdx.y;
  // routed: `extra` is the batch's [B, F, nmb] MB-tree table; a slot coding a reference
  // picture takes the row of its display index, other pictures get variance AQ only
  if (extra && rt) {
    const SlotRoute& r = rt[slot];
    extra = (r.kind >= 0 && r.disp >= 0 && (r.flags & SF_REF)) ? extra + static_cast<size_t>(r.disp) * nmb : nullptr;
  }
  for (int it = 0; it < kAqSpan; ++it) {
  const int mb = (blockIdx.x * kAqSpan + it) * 16 + (threadIdx.x >> 4);
  if ((blockIdx.x * kAqSpan + it) * 16 >= nmb) break;  // (uniform)
  const bool live = mb < nmb;
  const int mbc = live ? mb : nmb - 1;
  const int mx = mbc % g.wmb, my = mbc / g.wmb;
  const uint4 wy = *reinterpret_cast<const uint4*>(sy + slot * g.ysize() + static_cast<size_t>(my * 16 + l) * g.W + mx * 16);
  const uint8_t* c = (l < 8 ? su : sv) + slot * g.csize();
  const uint2 wc = *reinterpret_cast<const uint2*>(c + static_cast<size_t>(my * 8 + (l & 7)) * g.cw() + mx * 8);
  int s = 0, ss = 0, cs = 0, css = 0;
  const uint32_t ly[4] = {wy.x, wy.y, wy.z, wy.w}, lc[2] = {wc.x, wc.y};
#pragma unroll
  for (int w = 0; w < 4; ++w)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int p = __builtin_amdgcn_ubfe(ly[w], 8 * k, 8);
      s += p;
      ss += p * p;
    }
#pragma unroll
  for (int w = 0; w < 2; ++w)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int q = __builtin_amdgcn_ubfe(lc[w], 8 * k, 8);
      cs += q;
      css += q * q;
    }
  // Cb in lanes 0..7, Cr in 8..15 of the group: reduce each half-row separately
  const int cb_s = sum8(cs), cb_ss = sum8(css);
  s = sum16(s);
  ss = sum16(ss);
  const int cr_s = __shfl(cb_s, (lane_id() & ~15) + 8, 64), cr_ss = __shfl(cb_ss, (lane_id() & ~15) + 8, 64);
  if (live && l == 0) {
    // the squared luma sum exceeds INT_MAX once the MB mean passes 181: unsigned products
    const uint32_t us = static_cast<uint32_t>(s);
    const uint32_t e = (static_cast<uint32_t>(ss) - ((us * us) >> 8)) +
                       static_cast<uint32_t>(cb_ss - ((cb_s * cb_s) >> 6)) + static_cast<uint32_t>(cr_ss - ((cr_s * cr_s) >> 6));
    float adj = strength * 1.0397f * (log2f(static_cast<float>(e > 1u ? e : 1u)) - 14.427f);
    if (extra) adj += extra[slot * extra_stride + mb];  // MB-tree offset of this frame
    out[static_cast<size_t>(slot) * nmb + mb] = static_cast<int8_t>(clampi(static_cast<int>(rintf(adj)), -24, 24));
  }
  }
}

// 16 lanes per MB (16 MBs per 256-thread workgroup).  The MB carries mb_qp_delta iff it
// is Intra16x16 or has a non-zero level (coded_block_pattern != 0): luma from the encoder's
// per-block non-zero flags (lane 9, 16 bytes), chroma AC from coefficient 1 (lanes 0..7),
// chroma DC (lane 8), the MB kind (lane 10).
__global__ __launch_bounds__(256) void h264_qp_flags(Geom g, const MbHeader* __restrict__ hdr,
                                                     const int16_t* __restrict__ coef, const uint8_t* __restrict__ nzf,
                                                     uint8_t* __restrict__ flags) {
  const int lane = lane_id(), sub = lane & 15, grp = lane >> 4;
  const int nmb = g.nmb();
  const int mb = blockIdx.x * 16 + (threadIdx.x >> 4), slot = blockIdx.y;
  const bool live = mb < nmb;
  const size_t o = static_cast<size_t>(slot) * nmb + (live ? mb : 0);
  const int16_t* c = coef + o * h264::kCoefPerMb;
  bool nz = false;
  if (live && sub < 8) {
    const uint4* p = reinterpret_cast<const uint4*>(c + h264::COEF_CHROMA_AC + sub * 16);
    const uint4 q0 = p[0], q1 = p[1];
    nz = ((q0.x & 0xFFFF0000u) | q0.y | q0.z | q0.w | q1.x | q1.y | q1.z | q1.w) != 0;  // position 0 unused
  } else if (live && sub == 8) {
    const uint4 q = *reinterpret_cast<const uint4*>(c + h264::COEF_CHROMA_DC);
    nz = (q.x | q.y | q.z | q.w) != 0;
  } else if (live && sub == 9) {
    const uint4 q = *reinterpret_cast<const uint4*>(nzf + o * 16);
    nz = (q.x | q.y | q.z | q.w) != 0;
  } else if (live && sub == 10) {
    nz = hdr[o].kind == h264::MBK_I16x16;
  }
  const uint64_t bal = __ballot(nz);
  if (live && sub == 0) flags[o] = ((bal >> (16 * grp)) & 0xFFFFu) != 0 ? 1 : 0;
}

// One workgroup per slice (slot-major, `per_slot` slices of `slice_mbs` MBs each): chunked
// segmented scan of "last MB with mb_qp_delta"; QP_pred starts from the slice QP at every
// slice's first MB (7.4.5).
__global__ __launch_bounds__(1024) void h264_qp_fixup(Geom g, MbHeader* __restrict__ hdr,
                                                      const uint8_t* __restrict__ flags, const int* __restrict__ slice_qp,
                                                      int slice_mbs, int per_slot) {
  const int slot = blockIdx.x / per_slot, sl = blockIdx.x - slot * per_slot;
  const int first = sl * slice_mbs;
  const int n = min(g.nmb() - first, slice_mbs);
  const size_t base = static_cast<size_t>(slot) * g.nmb() + first;
  __shared__ int s_last[1024];
  const int per = (n + blockDim.x - 1) / blockDim.x;
  const int i0 = threadIdx.x * per, i1 = min(n, i0 + per);
  int last = -1;
  for (int i = i0; i < i1; ++i)
    if (flags[base + i]) last = i;
  s_last[threadIdx.x] = last;
  __syncthreads();
  for (int off = 1; off < blockDim.x; off <<= 1) {  // inclusive max-scan (Hillis-Steele)
    const int v = threadIdx.x >= off ? s_last[threadIdx.x - off] : -1;
    __syncthreads();
    s_last[threadIdx.x] = max(s_last[threadIdx.x], v);
    __syncthreads();
  }
  last = threadIdx.x > 0 ? s_last[threadIdx.x - 1] : -1;
  int qp = last >= 0 ? hdr[base + last].qp : slice_qp[slot];
  for (int i = i0; i < i1; ++i) {
    if (flags[base + i]) qp = hdr[base + i].qp;
    else hdr[base + i].qp = static_cast<int8_t>(qp);
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

// extra: optional per-MB float QP offsets added before rounding (MB-tree), slot s of this
// frame at extra + s * extra_stride
extern "C" void mivc_launch_aq_offsets(int B, int wmb, int hmb, const uint8_t* sy, const uint8_t* su,
                                       const uint8_t* sv, float strength, const float* extra, long long extra_stride,
                                       int8_t* out, void* stream, const void* route) {
  const Geom g{B, wmb, hmb, wmb * 16, hmb * 16};
  hipLaunchKernelGGL(h264_aq_offsets, dim3((wmb * hmb + 16 * kAqSpan - 1) / (16 * kAqSpan), B), dim3(256), 0,
                     static_cast<hipStream_t>(stream), g,
                     sy, su, sv, strength, extra, extra_stride, out, static_cast<const SlotRoute*>(route));
}

extern "C" void mivc_launch_qp_fixup(int B, int wmb, int hmb, void* hdr, const int16_t* coef, const uint8_t* nz,
                                     uint8_t* flags, const int* slice_qp, void* stream, int slice_rows) {
  const Geom g{B, wmb, hmb, wmb * 16, hmb * 16};
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int rows = (slice_rows > 0 && slice_rows < hmb) ? slice_rows : hmb;
  const int per_slot = (hmb + rows - 1) / rows;
  hipLaunchKernelGGL(h264_qp_flags, dim3((wmb * hmb + 15) / 16, B), dim3(256), 0, s, g,
                     static_cast<const mivc::h264::MbHeader*>(hdr), coef, nz, flags);
  hipLaunchKernelGGL(h264_qp_fixup, dim3(B * per_slot), dim3(1024), 0, s, g, static_cast<mivc::h264::MbHeader*>(hdr),
                     flags, slice_qp, rows * wmb, per_slot);
}
