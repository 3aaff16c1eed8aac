// Quality metrics: per-slot sum of squared errors between the
// source and the deblocked reconstruction over the display window, per plane,
// plus an 8x8-window SSIM sum on luma.  PSNR/SSIM are finished on the host.
#include "kcommon.h"

namespace mivc {
namespace gpu {

// sse: [B, 3] uint64 (Y, U, V).  One block of 256 threads per (row-group, slot).
__global__ void sse_planes(const uint8_t* sy, const uint8_t* su, const uint8_t* sv, const uint8_t* ry,
                           const uint8_t* ru, const uint8_t* rv, int W, int H, int w, int h,
                           unsigned long long* sse) {
  int slot = blockIdx.y;
  int row = blockIdx.x;  // luma row; chroma handled by even rows
  const size_t yo = static_cast<size_t>(slot) * W * H, co = static_cast<size_t>(slot) * (W / 2) * (H / 2);
  unsigned long long acc[3] = {0, 0, 0};
  if (row < h) {
    for (int x = threadIdx.x; x < w; x += blockDim.x) {
      int d = static_cast<int>(sy[yo + static_cast<size_t>(row) * W + x]) - ry[yo + static_cast<size_t>(row) * W + x];
      acc[0] += static_cast<unsigned long long>(d * d);
    }
    if ((row & 1) == 0) {
      int cr = row >> 1;
      for (int x = threadIdx.x; x < w / 2; x += blockDim.x) {
        size_t i = co + static_cast<size_t>(cr) * (W / 2) + x;
        int du = static_cast<int>(su[i]) - ru[i];
        int dv = static_cast<int>(sv[i]) - rv[i];
        acc[1] += static_cast<unsigned long long>(du * du);
        acc[2] += static_cast<unsigned long long>(dv * dv);
      }
    }
  }
  for (int p = 0; p < 3; ++p) {
    unsigned long long v = acc[p];
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(sse + slot * 3 + p, v);
  }
}

// SSIM over non-overlapping 8x8 luma windows; ssim_sum: [B] float accumulators, count in windows
__global__ void ssim8(const uint8_t* sy, const uint8_t* ry, int W, int H, int w, int h, float* ssim_sum) {
  int slot = blockIdx.y;
  int wx = blockIdx.x * blockDim.x + threadIdx.x;
  int nwx = w / 8, nwy = h / 8;
  float s = 0.f;
  if (wx < nwx * nwy) {
    int bx = (wx % nwx) * 8, by = (wx / nwx) * 8;
    const size_t yo = static_cast<size_t>(slot) * W * H;
    float ma = 0, mb = 0, va = 0, vb = 0, cov = 0;
    for (int y = 0; y < 8; ++y)
      for (int x = 0; x < 8; ++x) {
        float A = sy[yo + static_cast<size_t>(by + y) * W + bx + x], B = ry[yo + static_cast<size_t>(by + y) * W + bx + x];
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

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

extern "C" void mivc_launch_sse(int B, int W, int H, int w, int h, const uint8_t* sy, const uint8_t* su,
                                const uint8_t* sv, const uint8_t* ry, const uint8_t* ru, const uint8_t* rv,
                                unsigned long long* sse, float* ssim_sum, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(sse_planes, dim3(h, B), dim3(256), 0, s, sy, su, sv, ry, ru, rv, W, H, w, h, sse);
  if (ssim_sum) {
    int nwin = (w / 8) * (h / 8);
    hipLaunchKernelGGL(ssim8, dim3((nwin + 255) / 256, B), dim3(256), 0, s, sy, ry, W, H, w, h, ssim_sum);
  }
}
