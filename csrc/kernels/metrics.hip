// Quality metrics: per-slot sum of squared errors between the
// source and the deblocked reconstruction over the display window, per plane,
// plus an 8x8-window SSIM sum on luma.  PSNR/SSIM are finished on the host.
#include "h264_trellis.h"

namespace mivc {
namespace gpu {

// sse: [B, 3] uint64 (Y, U, V).  Grid (blocks_per_slot, B); each block strides over
// rows, each thread over 16-byte column chunks; one atomic per block and plane.
__device__ __forceinline__ unsigned sq_diff16(uint4 a, uint4 b, int valid) {
  const uint8_t* pa = reinterpret_cast<const uint8_t*>(&a);
  const uint8_t* pb = reinterpret_cast<const uint8_t*>(&b);
  unsigned s = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    int d = static_cast<int>(pa[k]) - pb[k];
    s += k < valid ? static_cast<unsigned>(d * d) : 0u;
  }
  return s;
}

__global__ void sse_planes(const uint8_t* sy, const uint8_t* su, const uint8_t* sv, const uint8_t* ry,
                           const uint8_t* ru, const uint8_t* rv, int W, int H, int w, int h,
                           unsigned long long* sse, const SlotRoute* rt, int nbuf) {
  const int slot = blockIdx.y;
  if (!route_active(rt, slot, -1)) return;
  // source [B, plane]; reconstruction: [B, plane], or the slot's current picture of the pool (rt)
  const size_t ro = route_index(rt, nbuf, slot, RO_CUR);
  const size_t yo = static_cast<size_t>(slot) * W * H, co = static_cast<size_t>(slot) * (W / 2) * (H / 2);
  const size_t ryo = ro * W * H, rco = ro * (W / 2) * (H / 2);
  unsigned long long acc[3] = {0, 0, 0};
  const int chunks_y = (w + 15) / 16, chunks_c = (w / 2 + 15) / 16;
  const int tid = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
  for (int i = tid; i < chunks_y * h; i += nth) {
    int r = i / chunks_y, c = (i % chunks_y) * 16;
    size_t off = yo + static_cast<size_t>(r) * W + c;
    acc[0] += sq_diff16(*reinterpret_cast<const uint4*>(sy + off), *reinterpret_cast<const uint4*>(ry + off - yo + ryo), w - c);
  }
  for (int i = tid; i < chunks_c * (h / 2); i += nth) {
    int r = i / chunks_c, c = (i % chunks_c) * 16;
    size_t off = co + static_cast<size_t>(r) * (W / 2) + c;
    acc[1] += sq_diff16(*reinterpret_cast<const uint4*>(su + off), *reinterpret_cast<const uint4*>(ru + off - co + rco), w / 2 - c);
    acc[2] += sq_diff16(*reinterpret_cast<const uint4*>(sv + off), *reinterpret_cast<const uint4*>(rv + off - co + rco), w / 2 - c);
  }
  __shared__ unsigned long long red[3][4];
  for (int p = 0; p < 3; ++p) {
    unsigned long long v = acc[p];
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((threadIdx.x & 63) == 0) red[p][threadIdx.x >> 6] = v;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    unsigned long long v = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) v += red[threadIdx.x][k];
    if (v) atomicAdd(sse + slot * 3 + threadIdx.x, v);
  }
}

// SSIM over non-overlapping 8x8 luma windows; ssim_sum: [B] float accumulators, count in windows
__global__ void ssim8(const uint8_t* sy, const uint8_t* ry, int W, int H, int w, int h, float* ssim_sum,
                      const SlotRoute* rt, int nbuf) {
  int slot = blockIdx.y;
  if (!route_active(rt, slot, -1)) return;
  const size_t ryo = route_index(rt, nbuf, slot, RO_CUR) * W * H;
  int wx = blockIdx.x * blockDim.x + threadIdx.x;
  int nwx = w / 8, nwy = h / 8;
  float s = 0.f;
  if (wx < nwx * nwy) {
    int bx = (wx % nwx) * 8, by = (wx / nwx) * 8;
    const size_t yo = static_cast<size_t>(slot) * W * H;
    float ma = 0, mb = 0, va = 0, vb = 0, cov = 0;
    for (int y = 0; y < 8; ++y)
      for (int x = 0; x < 8; ++x) {
        float A = sy[yo + static_cast<size_t>(by + y) * W + bx + x], B = ry[ryo + static_cast<size_t>(by + y) * W + bx + x];
        ma += A;
        mb += B;
        va += A * A;
        vb += B * B;
        cov += A * B;
      }
    ma /= 64.f;
    mb /= 64.f;
    va = va / 64.f - ma * ma;
    vb = vb / 64.f - mb * mb;
    cov = cov / 64.f - ma * mb;
    const float C1 = 6.5025f, C2 = 58.5225f;
    s = ((2 * ma * mb + C1) * (2 * cov + C2)) / ((ma * ma + mb * mb + C1) * (va + vb + C2));
  }
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(ssim_sum + slot, s);
}

// Known-answer check of the SATD primitives the decision kernels use (tests/test_gpu_satd.py):
// block i = 16 source and 16 prediction bytes (raster 4x4); mode 0 = satd16 on unpacked
// residuals (the reference form), 1 = satd4x4_u8 (packed 16-bit).
__global__ __launch_bounds__(64) void satd_blocks(const uint8_t* src, const uint8_t* pred, int* out, int n, int mode) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  const int ic = i < n ? i : n - 1;
  uint32_t a[4], b[4];
#pragma unroll
  for (int y = 0; y < 4; ++y) {
    a[y] = reinterpret_cast<const uint32_t*>(src + static_cast<size_t>(ic) * 16)[y];
    b[y] = reinterpret_cast<const uint32_t*>(pred + static_cast<size_t>(ic) * 16)[y];
  }
  int v;
  if (mode == 0) {
    int r[16];
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int x = 0; x < 4; ++x) r[y * 4 + x] = static_cast<int>((a[y] >> (8 * x)) & 255u) - static_cast<int>((b[y] >> (8 * x)) & 255u);
    v = satd16(r);
  } else {
    v = satd4x4_u8(a, b);
  }
  if (i < n) out[i] = v;
}

// Known-answer check of the two trellis forms (tests/test_gpu_satd.py): w = [n, 16] raster
// forward-transform coefficients, out = [n, 16] raster levels.  mode 0: the serial pass
// (trellis_lite4x4, one lane per block); mode 1: the lane-parallel grp_trellis4x4 (4 lanes per
// block, one row each).  skip_dc: scan index 0 is coded elsewhere (start = 1).
__global__ __launch_bounds__(64) void trellis_blocks(const int* w, int* out, int n, int qp, int mode, int skip_dc) {
  const int qm = qp % 6, qbits = 15 + qp / 6;
  const float lam = trellis_lambda4(1.0f, qp);
  const int mf0 = h264::kQuantMF[qm][0], mf1 = h264::kQuantMF[qm][1], mf2 = h264::kQuantMF[qm][2];
  if (mode == 0) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    const int ic = i < n ? i : n - 1;
    int c[16], lv[16];
    const int mf[3] = {mf0, mf1, mf2};
#pragma unroll
    for (int r = 0; r < 16; ++r) c[r] = w[static_cast<size_t>(ic) * 16 + r];
    trellis_lite4x4(c, lv, mf, qbits, lam, skip_dc ? 1 : 0);
    if (i < n)
#pragma unroll
      for (int r = 0; r < 16; ++r) out[static_cast<size_t>(i) * 16 + r] = lv[r];
  } else {
    const int lane = threadIdx.x, gy = lane & 3;
    const int b = blockIdx.x * 16 + (lane >> 2);
    const int bc = b < n ? b : n - 1;
    int c[4], lv[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) c[x] = w[static_cast<size_t>(bc) * 16 + gy * 4 + x];
    grp_trellis4x4(c, lv, gy, mf0, mf1, mf2, qbits, lam, skip_dc != 0);
    if (b < n)
#pragma unroll
      for (int x = 0; x < 4; ++x) out[static_cast<size_t>(b) * 16 + gy * 4 + x] = lv[x];
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

extern "C" void mivc_launch_trellis_blocks(const int* w, int* out, int n, int qp, int mode, int skip_dc, void* stream) {
  const int grid = mode == 0 ? (n + 63) / 64 : (n + 15) / 16;
  hipLaunchKernelGGL(trellis_blocks, dim3(grid), dim3(64), 0, static_cast<hipStream_t>(stream), w, out, n, qp, mode,
                     skip_dc);
}

extern "C" void mivc_launch_satd_blocks(const uint8_t* src, const uint8_t* pred, int* out, int n, int mode, void* stream) {
  hipLaunchKernelGGL(satd_blocks, dim3((n + 63) / 64), dim3(64), 0, static_cast<hipStream_t>(stream), src, pred, out, n,
                     mode);
}

extern "C" void mivc_launch_sse(int B, int W, int H, int w, int h, const uint8_t* sy, const uint8_t* su,
                                const uint8_t* sv, const uint8_t* ry, const uint8_t* ru, const uint8_t* rv,
                                unsigned long long* sse, float* ssim_sum, void* stream, const void* route, int nbuf) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const SlotRoute* rt = static_cast<const SlotRoute*>(route);
  hipLaunchKernelGGL(sse_planes, dim3(32, B), dim3(256), 0, s, sy, su, sv, ry, ru, rv, W, H, w, h, sse, rt, nbuf);
  if (ssim_sum) {
    int nwin = (w / 8) * (h / 8);
    hipLaunchKernelGGL(ssim8, dim3((nwin + 255) / 256, B), dim3(256), 0, s, sy, ry, W, H, w, h, ssim_sum, rt, nbuf);
  }
}
