// Explicit weighted P prediction (x264 --weightp, weighted_pred_flag = 1; clause 8.4.2.3.2).
//
//   wp_stats   per (slot, display picture): sum and sum of squares of every plane of the
//              source clip -- x264 decides its weights in the lookahead from source
//              statistics too, so the whole batch is analysed once, before the first
//              picture is coded, and the weights are known to the host slice-header writer
//              without any per-picture synchronisation.
//   wp_src     the motion search of a weighted P picture runs against the *unweighted*
//              reference planes (half-sample planes included) with the source mapped through
//              the inverse weight, s' = ((s - o) << d) / w: the candidate whose unweighted
//              prediction p best matches s' is the one whose weighted prediction
//              ((p * w + 2^(d-1)) >> d) + o best matches s.  encode_inter applies the forward
//              weight to the chosen prediction (luma and chroma), exactly as a decoder does.
#include "kcommon.h"

namespace mivc {
namespace gpu {

// grid (chunks, B * F); each block of 256 threads reduces a slice of one picture's three planes
__global__ __launch_bounds__(256) void wp_stats(const uint8_t* __restrict__ y, const uint8_t* __restrict__ u,
                                                const uint8_t* __restrict__ v, int w, int h,
                                                unsigned long long* __restrict__ out) {
  const int pic = blockIdx.y;
  const size_t ny = static_cast<size_t>(w) * h, nc = ny / 4;
  const uint8_t* P[3] = {y + pic * ny, u + pic * nc, v + pic * nc};
  const size_t N[3] = {ny, nc, nc};
  __shared__ unsigned long long red[6][4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    // 4-byte words of this block's slice of plane c (planes are w * h / 4-byte multiples for
    // even w, h; the tail bytes are picked up one at a time)
    const size_t words = N[c] / 4;
    const size_t per = (words + gridDim.x - 1) / gridDim.x;
    const size_t w0 = blockIdx.x * per, w1 = min(words, w0 + per);
    unsigned int s = 0;
    unsigned long long s2 = 0;
    const uint32_t* p32 = reinterpret_cast<const uint32_t*>(P[c]);
    if (reinterpret_cast<uintptr_t>(P[c]) & 3) {  // odd chroma plane sizes: byte loads
      for (size_t i = 4 * w0 + threadIdx.x; i < 4 * w1; i += 256) {
        const unsigned int b = P[c][i];
        s += b;
        s2 += b * b;
      }
    } else
    for (size_t i = w0 + threadIdx.x; i < w1; i += 256) {
      const uint32_t x = p32[i];
      unsigned int q = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const unsigned int b = (x >> (8 * k)) & 255u;
        s += b;
        q += b * b;
      }
      s2 += q;
    }
    if (blockIdx.x == 0)
      for (size_t i = words * 4 + threadIdx.x; i < N[c]; i += 256) {
        const unsigned int b = P[c][i];
        s += b;
        s2 += b * b;
      }
    unsigned long long s64 = s;
    for (int off = 32; off > 0; off >>= 1) {
      s64 += __shfl_xor(s64, off, 64);
      s2 += __shfl_xor(s2, off, 64);
    }
    if (lane == 0) {
      red[2 * c][wv] = s64;
      red[2 * c + 1][wv] = s2;
    }
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    const unsigned long long t = red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3];
    atomicAdd(out + static_cast<size_t>(pic) * 6 + threadIdx.x, t);
  }
}

// The same statistics of 16-bit samples (Main 10 input, int16 planes holding 0..1023)
__global__ __launch_bounds__(256) void wp_stats16(const uint16_t* __restrict__ y, const uint16_t* __restrict__ u,
                                                  const uint16_t* __restrict__ v, int w, int h,
                                                  unsigned long long* __restrict__ out) {
  const int pic = blockIdx.y;
  const size_t ny = static_cast<size_t>(w) * h, nc = ny / 4;
  const uint16_t* P[3] = {y + pic * ny, u + pic * nc, v + pic * nc};
  const size_t N[3] = {ny, nc, nc};
  __shared__ unsigned long long red[6][4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const size_t per = (N[c] + gridDim.x - 1) / gridDim.x;
    const size_t i0 = blockIdx.x * per, i1 = min(N[c], i0 + per);
    unsigned long long s = 0, s2 = 0;
    for (size_t i = i0 + threadIdx.x; i < i1; i += 256) {
      const unsigned int b = P[c][i];
      s += b;
      s2 += b * b;
    }
    for (int off = 32; off > 0; off >>= 1) {
      s += __shfl_xor(s, off, 64);
      s2 += __shfl_xor(s2, off, 64);
    }
    if (lane == 0) {
      red[2 * c][wv] = s;
      red[2 * c + 1][wv] = s2;
    }
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    const unsigned long long t = red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3];
    atomicAdd(out + static_cast<size_t>(pic) * 6 + threadIdx.x, t);
  }
}

// wt: [B, 3] (w, o, log2 denominator) of the luma weight per slot; w == 1 << d && o == 0:
// identity (plain copy)
__global__ __launch_bounds__(256) void wp_src(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                              const int* __restrict__ wt, size_t words_per_slot) {
  const int slot = blockIdx.y;
  const int w = wt[slot * 3], o = wt[slot * 3 + 1], d = wt[slot * 3 + 2];
  const uint32_t* s = reinterpret_cast<const uint32_t*>(src) + slot * words_per_slot;
  uint32_t* t = reinterpret_cast<uint32_t*>(dst) + slot * words_per_slot;
  const bool ident = w == (1 << d) && o == 0;
  const int wd = w > 0 ? w : 1;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < words_per_slot; i += gridDim.x * 256) {
    const uint32_t x = s[i];
    if (ident) {
      t[i] = x;
      continue;
    }
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int b = static_cast<int>((x >> (8 * k)) & 255u);
      const int num = ((b - o) << d) + (wd >> 1);
      const int q = num >= 0 ? num / wd : -((-num + wd - 1) / wd);
      r |= static_cast<uint32_t>(clampi(q, 0, 255)) << (8 * k);
    }
    t[i] = r;
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

extern "C" void mivc_launch_wp_stats(const uint8_t* y, const uint8_t* u, const uint8_t* v, int w, int h, int npics,
                                     unsigned long long* out, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  (void)hipMemsetAsync(out, 0, static_cast<size_t>(npics) * 6 * sizeof(unsigned long long), s);
  const int chunks = max(1, min(64, (w * h) / (256 * 64)));
  hipLaunchKernelGGL(wp_stats, dim3(chunks, npics), dim3(256), 0, s, y, u, v, w, h, out);
}

extern "C" void mivc_launch_wp_stats16(const uint16_t* y, const uint16_t* u, const uint16_t* v, int w, int h,
                                       int npics, unsigned long long* out, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  (void)hipMemsetAsync(out, 0, static_cast<size_t>(npics) * 6 * sizeof(unsigned long long), s);
  const int chunks = max(1, min(64, (w * h) / (256 * 64)));
  hipLaunchKernelGGL(wp_stats16, dim3(chunks, npics), dim3(256), 0, s, y, u, v, w, h, out);
}

extern "C" void mivc_launch_wp_src(const uint8_t* src, uint8_t* dst, const int* wt, int B, long long plane_bytes,
                                   void* stream) {
  const size_t words = static_cast<size_t>(plane_bytes) / 4;
  const size_t nb = (words + 255) / 256;
  const int blocks = static_cast<int>(nb < 256 ? nb : 256);
  hipLaunchKernelGGL(wp_src, dim3(blocks, B), dim3(256), 0, static_cast<hipStream_t>(stream), src, dst, wt, words);
}
