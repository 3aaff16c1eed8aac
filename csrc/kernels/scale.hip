// Picture resampling (the `-s WxH` the reference's operators passed to ffmpeg,
// server.go:87-90; SURVEY.md K-C2 csc_scale).  ffmpeg's swscale default is SWS_BICUBIC
// (Mitchell-Netravali family, B = 0, C = 0.6); this is the same separable kernel with
// swscale-style support widening when downscaling (taps = 4 * ceil(in / out)), 14-bit
// fixed-point coefficients per output column / row built on the host
// (govideocompressor_amd/ops/scale.py), and an integer pipeline that the numpy golden
// model reproduces exactly:
//   h = (sum_k cx[k] * in) >> (bd - 1)        (rounded, 15-bit intermediate headroom)
//   out = clip((sum_k cy[k] * h) >> (29 - bd)) (rounded)
//
// One workgroup (256 threads) computes an output tile: the input region it needs (tile
// footprint + filter halo, clamped at the picture edges) is staged in LDS once, the
// horizontal pass runs over the staged rows into an LDS int32 tile, the vertical pass
// reads it and writes the output.  Output columns / rows past the display size (the
// coded-size padding of the encoders) replicate the last display column / row.
// 8-bit (uint8) and 10-bit (uint16) samples; frames along grid z.
#include "kcommon.h"

namespace mivc {
namespace gpu {

struct ScaleArgs {
  const void* in;
  int w, h;
  long long in_stride;   // samples between input frames
  long long in_pitch;    // samples between input rows
  void* out;
  int ow, oh;            // display size of the output
  int W, H;              // written size (>= ow, oh: padding replicates)
  long long out_stride;
  long long out_pitch;
  const int* fx;         // [ow] first input column of output column x
  const int16_t* cx;     // [ow][tx]
  int tx;
  const int* fy;         // [oh]
  const int16_t* cy;     // [oh][ty]
  int ty;
  int tile_w, tile_h;    // output tile
  int in_cols, in_rows;  // staged input region capacity
  int bd;                // bit depth (8 or 10)
};

template <typename T>
__global__ __launch_bounds__(256) void scale_bicubic(ScaleArgs a) {
  extern __shared__ int smem[];
  const int n = blockIdx.z;
  const int ox0 = blockIdx.x * a.tile_w, oy0 = blockIdx.y * a.tile_h;
  const int tw = min(a.tile_w, a.W - ox0), th = min(a.tile_h, a.H - oy0);
  const int xa = min(ox0, a.ow - 1), xb = min(ox0 + tw - 1, a.ow - 1);
  const int ya = min(oy0, a.oh - 1), yb = min(oy0 + th - 1, a.oh - 1);
  const int c0 = a.fx[xa], r0 = a.fy[ya];
  const int ncols = a.fx[xb] + a.tx - c0, nrows = a.fy[yb] + a.ty - r0;
  uint16_t* stage = reinterpret_cast<uint16_t*>(smem);                           // [in_rows][in_cols]
  int* hb = smem + (a.in_rows * a.in_cols + 1) / 2;                              // [in_rows][tile_w]
  const T* in = static_cast<const T*>(a.in) + static_cast<long long>(n) * a.in_stride;
  if (ncols > a.in_cols || nrows > a.in_rows) return;  // host sizing guarantees this never happens
  for (int i = threadIdx.x; i < nrows * ncols; i += blockDim.x) {
    const int r = i / ncols, c = i - r * ncols;
    const int y = clampi(r0 + r, 0, a.h - 1), x = clampi(c0 + c, 0, a.w - 1);
    stage[r * a.in_cols + c] = static_cast<uint16_t>(in[static_cast<long long>(y) * a.in_pitch + x]);
  }
  __syncthreads();
  const int sh = a.bd - 1;
  for (int i = threadIdx.x; i < nrows * tw; i += blockDim.x) {
    const int r = i / tw, xo = i - r * tw;
    const int x = min(ox0 + xo, a.ow - 1);
    const int16_t* c = a.cx + static_cast<long long>(x) * a.tx;
    const uint16_t* s = stage + r * a.in_cols + (a.fx[x] - c0);
    int acc = 0;
    for (int k = 0; k < a.tx; ++k) acc += c[k] * static_cast<int>(s[k]);
    hb[r * a.tile_w + xo] = (acc + (1 << (sh - 1))) >> sh;
  }
  __syncthreads();
  const int sv = 29 - a.bd, maxv = (1 << a.bd) - 1;
  T* out = static_cast<T*>(a.out) + static_cast<long long>(n) * a.out_stride;
  for (int i = threadIdx.x; i < th * tw; i += blockDim.x) {
    const int yo = i / tw, xo = i - yo * tw;
    const int y = min(oy0 + yo, a.oh - 1);
    const int16_t* c = a.cy + static_cast<long long>(y) * a.ty;
    const int* col = hb + (a.fy[y] - r0) * a.tile_w + xo;
    int acc = 0;
    for (int k = 0; k < a.ty; ++k) acc += c[k] * col[k * a.tile_w];
    out[static_cast<long long>(oy0 + yo) * a.out_pitch + ox0 + xo] =
        static_cast<T>(clampi((acc + (1 << (sv - 1))) >> sv, 0, maxv));
  }
}

}  // namespace gpu
}  // namespace mivc

using namespace mivc::gpu;

// Returns 0, or -1 when the staged region does not fit the LDS budget (the caller picks
// smaller tiles).
extern "C" int mivc_launch_scale(const void* in, int w, int h, long long in_stride, long long in_pitch, void* out,
                                 int ow, int oh, int W, int H, long long out_stride, long long out_pitch, int nframes,
                                 const int* fx, const int16_t* cx, int tx, const int* fy, const int16_t* cy, int ty,
                                 int tile_w, int tile_h, int in_cols, int in_rows, int bd, void* stream) {
  ScaleArgs a{in, w, h, in_stride, in_pitch, out, ow, oh, W, H, out_stride, out_pitch, fx, cx, tx, fy, cy, ty,
              tile_w, tile_h, in_cols, in_rows, bd};
  const size_t lds = static_cast<size_t>((in_rows * in_cols + 1) / 2) * 4 + static_cast<size_t>(in_rows) * tile_w * 4;
  if (lds > 64 * 1024 || (bd != 8 && bd != 10)) return -1;
  dim3 grid((W + tile_w - 1) / tile_w, (H + tile_h - 1) / tile_h, nframes);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (bd == 8) hipLaunchKernelGGL(scale_bicubic<uint8_t>, grid, dim3(256), lds, s, a);
  else hipLaunchKernelGGL(scale_bicubic<uint16_t>, grid, dim3(256), lds, s, a);
  return 0;
}
