// Frame preparation: display-size I420 -> coded-size (multiple of 16) planar
// frames with edge replication, and a packed-RGB -> I420 colour conversion (BT.601
// limited range, ops/scale.py rgb_to_i420).  Resampling (`-s WxH`, server.go:87-90)
// is the bicubic filter of scale.hip.  SURVEY.md K-C2 (csc_scale).
#include "kcommon.h"

namespace mivc {
namespace gpu {

struct PrepArgs {
  const uint8_t* in_y;  // [N, h, w]
  const uint8_t* in_u;  // [N, h/2, w/2]
  const uint8_t* in_v;
  int w, h;             // input size
  int64_t in_frame_stride_y, in_frame_stride_c;  // elements between consecutive input frames
  uint8_t* out_y;       // [N, H, W] coded
  uint8_t* out_u;
  uint8_t* out_v;
  int ow, oh;           // output display size (== w, h: inputs arrive resampled)
  int W, H;             // coded size
  // per-slot frame selection (per-slot GOP plans: every slot codes its own display picture
  // this step): input frame n starts fsel[n] frames after in_* + n * in_frame_stride (nullable)
  const int* fsel;
  int64_t fstep_y, fstep_c;
};

// Copy + edge replication into the coded padding (resampling runs before, in scale.hip).
__global__ void prep_plane(PrepArgs a, int plane) {
  int x = blockIdx.x * blockDim.x + threadIdx.x;
  int y = blockIdx.y;
  int n = blockIdx.z;
  int sh = plane ? 1 : 0;
  int W = a.W >> sh, H = a.H >> sh;
  if (x >= W) return;
  int w = a.w >> sh, h = a.h >> sh;
  const uint8_t* in = plane == 0 ? a.in_y : (plane == 1 ? a.in_u : a.in_v);
  in += n * (plane ? a.in_frame_stride_c : a.in_frame_stride_y);
  if (a.fsel) in += a.fsel[n] * (plane ? a.fstep_c : a.fstep_y);
  uint8_t* out = plane == 0 ? a.out_y : (plane == 1 ? a.out_u : a.out_v);
  out += static_cast<size_t>(n) * W * H;
  int cx = min(x, w - 1), cy = min(y, h - 1);
  out[static_cast<size_t>(y) * W + x] = in[static_cast<size_t>(cy) * w + cx];
}

// Fast path (no resampling, 16-byte aligned rows): a 256-thread workgroup copies kPrepRows
// rows of one frame as 16-byte chunks, every thread several (the one-wave-per-1 KiB grid of
// round 3 made half a million tiny workgroups per plane and step at 1080p x 256 slots).
constexpr int kPrepRows = 8;

__global__ __launch_bounds__(256) void prep_plane_copy16(PrepArgs a, int plane) {
  const int sh = plane ? 1 : 0;
  const int W = a.W >> sh, H = a.H >> sh;
  const int w = a.w >> sh, h = a.h >> sh;
  const int n = blockIdx.y;
  const int cpr = W >> 4;  // 16-byte chunks per output row
  const int y0 = blockIdx.x * kPrepRows;
  const int rows = min(kPrepRows, H - y0);
  const uint8_t* in = plane == 0 ? a.in_y : (plane == 1 ? a.in_u : a.in_v);
  in += n * (plane ? a.in_frame_stride_c : a.in_frame_stride_y);
  if (a.fsel) in += a.fsel[n] * (plane ? a.fstep_c : a.fstep_y);
  uint8_t* out = (plane == 0 ? a.out_y : (plane == 1 ? a.out_u : a.out_v)) + static_cast<size_t>(n) * W * H;
  for (int i = threadIdx.x; i < rows * cpr; i += 256) {
    const int r = i / cpr, x = (i - r * cpr) * 16, y = y0 + r;
    const uint8_t* row = in + static_cast<size_t>(min(y, h - 1)) * w;
    uint4 v;
    if (x + 16 <= w) {
      v = *reinterpret_cast<const uint4*>(row + x);
    } else {
      uint8_t b[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) b[k] = row[min(x + k, w - 1)];
      v = *reinterpret_cast<const uint4*>(b);
    }
    *reinterpret_cast<uint4*>(out + static_cast<size_t>(y) * W + x) = v;
  }
}

// packed RGB24 [N, h, w, 3] -> I420 display-size planes (BT.601 limited range)
__global__ void rgb_to_i420(const uint8_t* rgb, int w, int h, uint8_t* oy, uint8_t* ou, uint8_t* ov) {
  int x2 = blockIdx.x * blockDim.x + threadIdx.x;  // chroma column
  int y2 = blockIdx.y;
  int n = blockIdx.z;
  if (x2 >= w / 2) return;
  const uint8_t* f = rgb + static_cast<size_t>(n) * w * h * 3;
  float su = 0, sv = 0;
  for (int dy = 0; dy < 2; ++dy)
    for (int dx = 0; dx < 2; ++dx) {
      int x = 2 * x2 + dx, y = 2 * y2 + dy;
      const uint8_t* p = f + (static_cast<size_t>(y) * w + x) * 3;
      float r = p[0], g = p[1], b = p[2];
      float Y = 16.f + 0.257f * r + 0.504f * g + 0.098f * b;
      su += 128.f - 0.148f * r - 0.291f * g + 0.439f * b;
      sv += 128.f + 0.439f * r - 0.368f * g - 0.071f * b;
      oy[static_cast<size_t>(n) * w * h + static_cast<size_t>(y) * w + x] = static_cast<uint8_t>(fminf(fmaxf(Y + 0.5f, 0.f), 255.f));
    }
  size_t ci = static_cast<size_t>(n) * (w / 2) * (h / 2) + static_cast<size_t>(y2) * (w / 2) + x2;
  ou[ci] = static_cast<uint8_t>(fminf(fmaxf(su * 0.25f + 0.5f, 0.f), 255.f));
  ov[ci] = static_cast<uint8_t>(fminf(fmaxf(sv * 0.25f + 0.5f, 0.f), 255.f));
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

extern "C" void mivc_launch_prep(const uint8_t* in_y, const uint8_t* in_u, const uint8_t* in_v, int w, int h,
                                 int64_t in_stride_y, int64_t in_stride_c, int nframes, uint8_t* out_y, uint8_t* out_u,
                                 uint8_t* out_v, int ow, int oh, int W, int H, void* stream, const int* fsel) {
  PrepArgs a{in_y, in_u, in_v, w, h, in_stride_y, in_stride_c, out_y, out_u, out_v, ow, oh, W, H,
             fsel, static_cast<int64_t>(w) * h, static_cast<int64_t>(w / 2) * (h / 2)};
  hipStream_t s = static_cast<hipStream_t>(stream);
  bool aligned = (w % 32 == 0) && (in_stride_y % 16 == 0) && (in_stride_c % 16 == 0) &&
                 (reinterpret_cast<uintptr_t>(in_y) % 16 == 0) && (reinterpret_cast<uintptr_t>(in_u) % 16 == 0) &&
                 (reinterpret_cast<uintptr_t>(in_v) % 16 == 0) && W % 32 == 0;
  if (ow != w || oh != h) return;  // scale.hip resamples before prep (the binding rejects this)
  if (aligned) {
    hipLaunchKernelGGL(prep_plane_copy16, dim3((H + kPrepRows - 1) / kPrepRows, nframes), dim3(256), 0, s, a, 0);
    hipLaunchKernelGGL(prep_plane_copy16, dim3((H / 2 + kPrepRows - 1) / kPrepRows, nframes), dim3(256), 0, s, a, 1);
    hipLaunchKernelGGL(prep_plane_copy16, dim3((H / 2 + kPrepRows - 1) / kPrepRows, nframes), dim3(256), 0, s, a, 2);
    return;
  }
  hipLaunchKernelGGL(prep_plane, dim3((W + 255) / 256, H, nframes), dim3(256), 0, s, a, 0);
  hipLaunchKernelGGL(prep_plane, dim3((W / 2 + 255) / 256, H / 2, nframes), dim3(256), 0, s, a, 1);
  hipLaunchKernelGGL(prep_plane, dim3((W / 2 + 255) / 256, H / 2, nframes), dim3(256), 0, s, a, 2);
}

extern "C" void mivc_launch_rgb_to_i420(const uint8_t* rgb, int w, int h, int nframes, uint8_t* y, uint8_t* u,
                                        uint8_t* v, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(rgb_to_i420, dim3((w / 2 + 127) / 128, h / 2, nframes), dim3(128), 0, s, rgb, w, h, y, u, v);
}
